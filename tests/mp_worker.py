"""Rank program of the multi-PROCESS tests (tests/test_gpu_multiproc.py): one torchrun rank.

Under HIPFM_SAME_DEVICE=1 every rank runs on device 0 and exchanges through the same-device
engine (parallel/loopback.py); the model, exchange, routing, graphs and step are the production
ones (parallel/sharded.py / replicated.py over the native kernels).  Each rank trains its slice
of the global batches and writes its table shard + dense parameters to ``<out>/rank<r>.pt``; the
test compares them with one model trained on the global batch.

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tests/mp_worker.py '<json>'
json: {"out": dir, "sharded": bool, "update": "lazy"|"tf1_dense", "mode": "run"|"prefetch"|"eager",
       "steps": int, "B": int, "opt": "Adam", "lr": float}
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def main():
    cfg = json.loads(sys.argv[1])
    import hipfm  # noqa: F401
    from hipfm.parallel.dist import same_device_env
    # this rank's CU slice, before the first HIP call of the process creates a queue
    os.environ.update(same_device_env(int(os.environ["LOCAL_RANK"]), int(os.environ["LOCAL_WORLD_SIZE"])))
    import torch
    import torch.distributed as dist
    import hipfm  # noqa: F401
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import init_params
    from hipfm.parallel.dist import Comm, init_distributed, local_device_index, same_device

    assert same_device(), "mp_worker: run under HIPFM_SAME_DEVICE=1"
    torch.cuda.set_device(local_device_index())
    dev = torch.device("cuda", local_device_index())
    init_distributed()
    rank, N = dist.get_rank(), dist.get_world_size()
    synth = make_synth("criteo_kaggle", seed=4)
    F, K, layers, keep, B = synth.F, 8, [64, 32], [1.0, 1.0], int(cfg.get("B", 512))
    V = synth.feature_size
    steps = int(cfg.get("steps", 3))
    params = init_params(V, F, K, layers, False, seed=7)
    data = [synth.batch(N * B, step=s, device=dev, id_dtype=torch.int32) for s in range(steps)]
    mine = [(ids[rank * B:(rank + 1) * B].contiguous(), vals[rank * B:(rank + 1) * B].contiguous(),
             lab[rank * B:(rank + 1) * B].contiguous()) for ids, vals, lab in data]
    comm = Comm(sharded=bool(cfg.get("sharded", True)))
    m = NativeDeepFM(V, F, K, layers, keep, optimizer=cfg.get("opt", "Adam"),
                     sparse_update=cfg.get("update", "lazy"), learning_rate=float(cfg.get("lr", 1e-3)),
                     batch_size=B, device=dev, init=False, comm=comm, field_ranges=synth.field_ranges())
    m.load_tf_params(params)
    x = m.shx if m.shx is not None else m.rpx
    assert x is not None and x.N == N and type(comm.engine).__name__ == "LoopbackEngine"
    x.trace = []
    torch.cuda.synchronize()
    mode = cfg.get("mode", "run")
    graphs0 = len(m._graphs)
    if mode == "run":
        # the bench's first rung: a captured multi-step graph with run-level routing (the model's
        # first step runs eagerly, the rest of the run is one graph), then the same run replayed
        n = m.train_steps(mine)
        assert n == steps
    elif mode == "prefetch":
        for i, (ids, vals, lab) in enumerate(mine):
            nxt = (mine[i + 1][0] if i + 1 < steps else None, mine[i + 2][0] if i + 2 < steps else None)
            m.train_step(ids, vals, lab, use_graph=True, next_ids=nxt)
    else:
        for ids, vals, lab in mine:
            m.train_step(ids, vals, lab)
    torch.cuda.synchronize()
    m.check_errors()
    out = {"tv": m.tv.float().cpu(), "tw": m.tw.float().cpu(), "p": m.p.cpu(),
           "graphs": torch.tensor(len(m._graphs) - graphs0),
           "trace": torch.tensor([[k, nb] for g in x.trace for k, nb in g] or [[0, 0]], dtype=torch.int64),
           "bytes_sent": torch.tensor(comm.bytes_sent)}
    torch.save(out, os.path.join(cfg["out"], f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
