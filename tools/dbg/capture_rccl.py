"""Isolate: HIP-graph capture of native RCCL collectives on forked side streams (1 rank)."""
import os, sys, socket
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.distributed as dist
import hipfm
from hipfm.ops import kernels as KN
from hipfm.parallel.sharded import RcclEngine

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
e1, e2, e3 = RcclEngine(), RcclEngine(), RcclEngine()
a = torch.arange(1024, dtype=torch.int32, device="cuda"); b = torch.zeros_like(a)
c = torch.arange(1024, dtype=torch.int32, device="cuda"); d = torch.zeros_like(c)
g = torch.ones(4096, device="cuda")
side = torch.cuda.Stream(); side2 = torch.cuda.Stream()
mode = sys.argv[1]

def step():
    main = torch.cuda.current_stream()
    if "late" in mode:
        e1.alltoall(a, b, 4096)
    if "kernel" in mode:
        side.wait_stream(main)
        with torch.cuda.stream(side):
            c.add_(1)
        main.wait_stream(side)
    if "route" in mode:
        side.wait_stream(main)
        with torch.cuda.stream(side):
            if "memset" in mode:
                torch.cuda.current_stream()
                c.fill_(3)
            if "ag" in mode:
                e3.allgather(c, d, 4096)
            else:
                e3.alltoall(c, d, 4096)
    e1.alltoall(a, b, 4096)
    if "dense" in mode:
        side2.wait_stream(main)
        with torch.cuda.stream(side2):
            e2.allreduce_(g)
    e1.alltoall(b, a, 4096)
    if "dense" in mode:
        main.wait_stream(side2)
    if "route" in mode:
        main.wait_stream(side)

step(); torch.cuda.synchronize()
print(mode, "eager ok", flush=True)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    step()
gr.replay(); torch.cuda.synchronize()
print(mode, "ok", int(d.sum()), int(a.sum()), float(g[0]))
if "close" in mode:
    for e in (e1, e2, e3): e.close()
    print("closed", flush=True)
if "destroy" in mode:
    dist.destroy_process_group()
    print("destroyed", flush=True)
os._exit(0)
