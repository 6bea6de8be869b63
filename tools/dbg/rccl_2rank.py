"""Can two ranks share one GPU over RCCL?  (torchrun --nproc-per-node 2; every rank on cuda:0)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
r, n = dist.get_rank(), dist.get_world_size()
t = torch.full((4,), float(r + 1), device="cuda")
dist.all_reduce(t)
print(f"rank {r}: torch all_reduce {t.tolist()}", flush=True)
import hipfm  # noqa: E402
from hipfm.parallel.sharded import RcclEngine  # noqa: E402

e = RcclEngine()
a = torch.arange(8 * n, dtype=torch.int32, device="cuda") + 100 * r
b = torch.zeros_like(a)
e.alltoall(a, b, 8 * 4)
torch.cuda.synchronize()
print(f"rank {r}: native alltoall {b.tolist()}", flush=True)
dist.barrier()
dist.destroy_process_group()
