#!/usr/bin/env python
"""Flagship benchmark: DeepFM training throughput (samples/s, whole node) + eval AUC.

Config (BASELINE.json config #4, "Criteo-1TB-shape"): F = 39 fields (13 dense + 26
categorical with the Criteo-Terabyte per-field cardinalities, V = 882.8M feature ids),
embedding K = 8, deep layers 128,64,32 with keep-prob 0.5 dropout (the notebooks' model,
NBPS:82), Adam lr 5e-4 x world size (HVD:149), l2 1e-4 on fm_w/fm_v, bf16 MLP operands with
fp32 accumulation and fp32 tables / optimizer state.  The 882.8M-row table is replicated at
N=1 and row-sharded across ranks (all-to-all) at N>1; updates are "lazy" (touched rows only,
SURVEY Q8 — a TF1-dense sweep of 882.8M rows per step is what the reference would do).

Data: synthetic Criteo-shaped batches (Zipf ids, teacher labels), generated on the GPU and
kept HBM-resident (the reference's ``cache()`` analogue); random-init weights.  Weak scaling:
the per-GPU batch is fixed as N grows.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch_size B] [--preset criteo_1tb]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = ("samples/sec (whole node) + eval AUC, Criteo-1TB-shape DeepFM at 1/2/4/8 MI355X")

# Multi-GPU execution ladder (bench supervisor, below): the fastest path first, then paths with
# fewer moving parts.  Every rung is the same full training step (same model, optimizer, data),
# and in EVERY rung all collectives of a step run on one communicator, grouped, on the step's
# main stream in a fixed order (parallel/sharded.py) -- no rung has side-stream collectives.
# The first rung routes every batch of a captured run at its start (one grouped ids all-to-all,
# then per step G1 + G2 on one queue: parallel/sharded.py "Run-level routing"); the second is the
# per-step pipelined routing of round 2 (side-stream routing kernels, serve ahead), also
# captured; the last launches eagerly without the routing prefetch and without the fused dense
# exchange (dense all-reduce in the gradient group, 7-launch routing).
_PLAIN_EXCHANGE = {"HIPFM_SH_APPLY_DENSE": "0", "HIPFM_SH_ROUTE2": "0"}
LADDER = [
    ("graph+run-routing", {}),                               # HIP graphs, run-level routing
    ("graph+prefetch", {"HIPFM_RUN_SORT": "0"}),             # HIP graphs, next-batch routing prefetch
    ("eager", {"HIPFM_BENCH_NO_GRAPH": "1", "HIPFM_SHARD_PIPELINE": "0", **_PLAIN_EXCHANGE}),
]
# hang detection: a rung's child must write its first progress mark within FIRST_S (the parent
# supervisor already imported torch, so the child's imports hit a warm page cache) and then
# update it at least every HANG_S (every graph run / step chunk marks progress)
FIRST_S = 90.0
HANG_S = 45.0


def ladder_budget_s(rungs: int = len(LADDER), first_s: float = FIRST_S, hang_s: float = HANG_S,
                    setup_s: float = 60.0) -> float:
    """Worst-case wall time of a ladder whose every rung hangs: per rung, the child reaches its
    last progress mark after at most ``setup_s`` (model + communicator setup, measured well under
    that) or never marks (``first_s``), then ``hang_s`` of silence -- plus the teardown."""
    return rungs * (max(first_s, setup_s + hang_s) + 5.0)


_SHAPE_NAMES = {"criteo_1tb": "Criteo-1TB-shape", "criteo_kaggle": "Criteo-Kaggle-shape",
                "reference": "reference-notebook-shape"}


def _free_port() -> int:
    """A rendezvous port below the kernel's ephemeral range (hipfm/utils/net.py says why), checked
    by a bind; inlined so the supervisor process imports nothing of the package."""
    import random
    import socket
    rnd = random.SystemRandom()
    for _ in range(64):
        p = rnd.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
            return p
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def supervise(argv) -> int:
    """Multi-rank supervisor (one per torchrun worker; never touches the GPU).

    Runs the benchmark in a child process per rung of LADDER.  If any rank's child fails (non-zero
    exit) or stops making progress (no progress-file update for HIPFM_BENCH_HANG_S seconds), every
    rank kills its child and the job moves to the next rung on a fresh rendezvous port, so one
    misbehaving execution mode costs a retry instead of the whole measurement.  Ranks coordinate
    through torchrun's agent store (keys ``hipfm_bench/*``).  Returns the exit code."""
    import shutil
    import signal
    import subprocess
    import tempfile
    import time

    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                          world, is_master=False, timeout=__import__("datetime").timedelta(seconds=600))
    hang_s = float(os.environ.get("HIPFM_BENCH_HANG_S", str(HANG_S)))
    first_s = float(os.environ.get("HIPFM_BENCH_FIRST_S", str(FIRST_S)))
    ladder = LADDER[int(os.environ.get("HIPFM_BENCH_FIRST_RUNG", "0")):]
    for k, (name, extra) in enumerate(ladder):
        if rank == 0:
            store.set(f"hipfm_bench/port{k}", str(_free_port()))
        port = store.get(f"hipfm_bench/port{k}").decode()
        # a fresh directory per rung: a progress file left by an earlier process with the same
        # (recycled) pid would read as an old mark and declare the new child hung at once
        rdir = tempfile.mkdtemp(prefix=f"hipfm_bench_{os.getpid()}_{k}_")
        prog = os.path.join(rdir, "progress")
        result = os.path.join(rdir, "result.json")
        env = dict(os.environ, HIPFM_BENCH_CHILD="1", HIPFM_BENCH_RUNG=name, MASTER_PORT=port,
                   TORCHELASTIC_USE_AGENT_STORE="False", HIPFM_BENCH_PROGRESS=prog,
                   HIPFM_BENCH_RESULT=result, **extra)
        env.update(_same_device_env())
        child = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                 start_new_session=True)
        failed = False
        t_start = time.time()
        last = None
        while True:
            rc = child.poll()
            if rc is not None:
                failed = rc != 0
                break
            if store.check([f"hipfm_bench/fail{k}"]):
                failed = True
                break
            try:
                mt = os.path.getmtime(prog)
                last = mt if last is None else max(last, mt)
            except OSError:
                pass
            now = time.time()
            if (last is None and now - t_start > first_s) or (last is not None and now - last > hang_s):
                print(f"[bench rank {rank}] rung {name}: no progress for "
                      f"{(now - t_start) if last is None else (now - last):.0f}s", flush=True)
                failed = True
                break
            time.sleep(0.5)
        if child.poll() is None:
            os.killpg(child.pid, signal.SIGKILL)
            child.wait()
        if not failed:
            # the rung counts only when every rank's child succeeded
            store.set(f"hipfm_bench/ok{k}_{rank}", "1")
            oks = [f"hipfm_bench/ok{k}_{r}" for r in range(world)]
            while not store.check(oks) and not store.check([f"hipfm_bench/fail{k}"]):
                time.sleep(0.2)
            if store.check(oks):
                if rank == 0 and os.path.exists(result):
                    print(open(result).read().strip(), flush=True)
                shutil.rmtree(rdir, ignore_errors=True)
                return 0
            failed = True
        shutil.rmtree(rdir, ignore_errors=True)
        store.set(f"hipfm_bench/fail{k}", "1")
        print(f"[bench rank {rank}] rung {name} failed (rc={child.returncode}); "
              f"{'retrying with ' + ladder[k + 1][0] if k + 1 < len(ladder) else 'no rung left'}",
              flush=True)
        # every rank's child of this rung is gone before the next rung starts
        store.set(f"hipfm_bench/down{k}_{rank}", "1")
        store.wait([f"hipfm_bench/down{k}_{r}" for r in range(world)])
    return 1


def _same_device_env() -> dict:
    """(HIPFM_SAME_DEVICE=1 only) this rank's CU slice of the shared GPU (parallel/dist.py)."""
    if os.environ.get("HIPFM_SAME_DEVICE") != "1":
        return {}
    from hipfm.parallel.dist import same_device_env
    return same_device_env(int(os.environ.get("LOCAL_RANK", "0")),
                           int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))


def _emit(line: str):
    """The result line: printed directly, or (under the supervisor) handed over in a file and
    printed by rank 0's supervisor once every rank finished this execution rung."""
    p = os.environ.get("HIPFM_BENCH_RESULT")
    if p:
        with open(p, "w") as f:
            f.write(line + "\n")
    else:
        print(line, flush=True)


def _progress():
    p = os.environ.get("HIPFM_BENCH_PROGRESS")
    if p:
        with open(p, "w") as f:
            f.write("x")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch_size", type=int, default=16384, help="per-GPU batch")
    ap.add_argument("--preset", default="criteo_1tb")
    ap.add_argument("--embedding_size", type=int, default=8)
    ap.add_argument("--deep_layers", default="128,64,32")
    ap.add_argument("--dropout", default="0.5,0.5,0.5")
    ap.add_argument("--batch_norm", action="store_true", help="batch norm after each hidden layer (HVD:207-208)")
    ap.add_argument("--optimizer", default="Adam")
    ap.add_argument("--sparse_update", default="lazy")
    ap.add_argument("--embedding_mode", default="auto")
    ap.add_argument("--mlp_dtype", default="bf16", choices=["bf16", "fp8"],
                    help="deep-tower forward GEMM operands (fp8 = OCP e4m3 MFMA, config #5)")
    ap.add_argument("--exchange_rows", default="fp32", choices=["fp32", "bf16"],
                    help="row-sharded exchange (N > 1): fp32 served rows (the default, the library's "
                         "and the reference's precision: bitwise the one-GPU reads) or bf16 v (a "
                         "labelled variant: half the G1 bytes; the FM terms then read bf16-rounded v)")
    ap.add_argument("--emb_dtype", default="fp32", choices=["fp32", "bf16"],
                    help="fm_v rows + optimizer slots (bf16 = mixed-precision embeddings, config #5)")
    ap.add_argument("--pool", type=int, default=128,
                    help="resident synthetic batches per rank (the HBM-cached epoch; a 16-batch pool "
                         "replayed hundreds of times memorizes its ids: train loss -> 0, eval AUC drops)")
    ap.add_argument("--eval_batches", type=int, default=8)
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--graph_steps", type=int, default=int(os.environ.get("HIPFM_GRAPH_STEPS", "32")),
                    help="consecutive training steps captured per HIP graph (divides --pool)")
    ap.add_argument("--infer", action="store_true", help="serving mode (1 GPU): forward-only "
                    "predictions/s of the same model over resident batches, graph-captured")
    ap.add_argument("--data", default="", help="file-fed mode: TFRecord dir (tr*/va*): reports the "
                    "host ingest rate and the CLI/Estimator train rate (epoch 0 streamed, then cached)")
    ap.add_argument("--epochs", type=int, default=4, help="--data: epochs (0 streams + caches)")
    ap.add_argument("--threads", type=int, default=16, help="--data: loader threads")
    ap.add_argument("--stream_only", action="store_true", help="--data: only the streamed (uncached) arm")
    ap.add_argument("--field_major_ids", type=int, default=1,
                    help="1: store the resident batches' ids field-major ([F, B] storage: the run sort "
                         "and the tower gather read each field contiguously); 0: row-major")
    ap.add_argument("--force_exchange", action="store_true",
                    help="run the multi-GPU (row-sharded exchange) step on a 1-rank group")
    args = ap.parse_args()
    if os.environ.get("HIPFM_BENCH_NO_GRAPH") == "1":
        args.no_graph = True
    if os.environ.get("HIPFM_BENCH_FM_IDS") in ("0", "1"):
        args.field_major_ids = int(os.environ["HIPFM_BENCH_FM_IDS"])
    fake = os.environ.get("HIPFM_BENCH_FAKE")          # supervisor tests (CPU): fake rank work
    if fake:
        return _fake_child(args, fake)
    if args.data:
        return data_bench(args)
    if args.infer:
        return infer_bench(args)

    _progress()
    import torch
    import torch.distributed as dist
    import hipfm
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.ops.metrics import auc_from_hist
    from hipfm.parallel.dist import Comm, init_distributed, local_device_index, same_device

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device_index()        # LOCAL_RANK; 0 for every rank under HIPFM_SAME_DEVICE=1
    if args.gpus != world and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: measuring {world} rank(s)",
              file=sys.stderr, flush=True)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    synth = make_synth(args.preset, seed=2024)
    comm = None
    B = args.batch_size
    pool = [synth.batch(B, step=rank * 100000 + i, device=dev, id_dtype=torch.int32)
            for i in range(args.pool)]
    _progress()
    if world > 1 or args.force_exchange:
        init_distributed("nccl")         # (gloo + the same-device engine under HIPFM_SAME_DEVICE=1)
        _progress()
        mode = "sharded" if args.embedding_mode == "auto" else args.embedding_mode
        # capacity of the fixed-size exchanges: measured on EVERY batch this rank will route (the
        # resident pool and the eval batches), +5 % + 256 margin, then agreed across ranks (MAX).
        # Overflow raises, never drops rows.  sharded: unique ids per owner (all-to-all blocks);
        # replicated: unique ids per batch (all-gather blocks)
        ev = [synth.batch(B, step=10_000_000 + rank * 1000 + i, device=dev, id_dtype=torch.int32)[0]
              for i in range(args.eval_batches)]
        from hipfm.parallel.dist import exchange_capacity
        cap = exchange_capacity([b[0] for b in pool] + (ev if mode == "sharded" else []), world,
                                sharded=(mode == "sharded"))
        comm = Comm(sharded=(mode == "sharded"), force_exchange=args.force_exchange, capacity=cap)

    F = synth.F
    layers = [int(x) for x in args.deep_layers.split(",")]
    keep = [float(x) for x in args.dropout.split(",")]
    model = NativeDeepFM(synth.feature_size, F, args.embedding_size, layers, keep, l2_reg=1e-4,
                         learning_rate=5e-4, optimizer=args.optimizer,
                         sparse_update=args.sparse_update, seed=1234, batch_size=B, device=dev,
                         comm=comm, field_ranges=synth.field_ranges(), mlp_dtype=args.mlp_dtype,
                         emb_dtype=args.emb_dtype, exchange_rows=args.exchange_rows,
                         batch_norm=args.batch_norm)
    _progress()
    if args.field_major_ids:
        # ids stored field-major ([F, B] storage, [B, F] view: the layout the Estimator's HBM
        # cache stores, data/pipeline.py iter_epoch): the run-level sort's 39 per-field
        # workgroups each read one contiguous field (row-major: a 4-B id per 156-B row, 107 vs
        # 201 us per 20-batch run sort, 0.1121 vs 0.1141 ms/step; profiles/r4c_*)
        pool = [(ids.t().contiguous().t(), vals, labels) for ids, vals, labels in pool]
    use_graph = not args.no_graph
    P = len(pool)
    # (multi-rank graphs capture 2 RCCL groups per step + 1 per run; HIPFM_BENCH_XGRAPH caps them:
    # 1-rank proxy, driver window: 16 -> 0.162-0.166, 20 -> 0.156-0.158, 32 -> 0.159 ms/step)
    G = max(1, args.graph_steps if comm is None else
            min(args.graph_steps, int(os.environ.get("HIPFM_BENCH_XGRAPH", "32"))))
    torch.cuda.synchronize()
    _progress()

    def chunks(lo, hi):
        """Global step positions [lo, hi) cut into runs of consecutive pool batches: at most G
        steps, never across a pool wrap, and cut at the warm-up / timed boundary -- so the timed
        window starts a run, its runs are exactly runs captured before timing, and a short window
        (the driver's 20 steps) is ONE graph replay."""
        t = lo
        while t < hi:
            e = min(hi, t + G, (t // P + 1) * P)
            if t < args.warmup < e:
                e = args.warmup
            yield t, e
            t = e

    runs = {}          # each run's batch list, built once: a replay of a known run skips host planning

    def run(lo, hi):
        for k, (t, e) in enumerate(chunks(lo, hi)):
            _progress()
            i = t % P
            # the two batches after the run: their sort / routing is prefetched
            nxt = (pool[e % P][0], pool[(e + 1) % P][0])
            if use_graph and G > 1:
                r = runs.get((i, e - t))
                if r is None:
                    r = runs[(i, e - t)] = pool[i:i + (e - t)]
                model.train_steps(r, next_ids=nxt)
            else:
                for j in range(e - t):
                    ids, vals, labels = pool[i + j]
                    model.train_step(ids, vals, labels, use_graph=use_graph,
                                     next_ids=(pool[(i + j + 1) % P][0], pool[(i + j + 2) % P][0]))

    if use_graph and (comm is None or comm.graph_safe):
        # the model's very first step runs eagerly (it warms up lazy library state); taking it
        # here lets the pass below capture EVERY run the warm-up and timed windows replay (else
        # the warm-up captured its own first run right before the timed window)
        model.warm_step(*pool[0])
        # every graph the warm-up and timed runs replay is captured here first (real steps), from
        # the same canonical plan state (nothing prefetched, set rotation at 0) the warm-up below
        # starts from: its runs and the timed runs then find their graphs under the same keys
        model.reset_plan_state()
        run(0, args.warmup + args.steps)
        model.reset_plan_state()
        torch.cuda.synchronize()
    _progress()
    # every long-lived object exists now (model, pool, captured graphs and their plans): move them
    # out of the collector's generations.  A full collection over them takes ~1 ms of host time;
    # landing inside the short timed window (as the allocation counts happened to make it with
    # --warmup 4-6) it stalled the graph launch: 0.157-0.187 instead of 0.114-0.117 ms/step
    gc.collect()
    gc.freeze()
    n_graphs = len(model._graphs)
    run(0, args.warmup)
    torch.cuda.synchronize()
    warm_captures = len(model._graphs) - n_graphs
    _progress()
    if comm is not None:
        dist.barrier()
    torch.cuda.synchronize()
    n_graphs = len(model._graphs)
    t0 = time.perf_counter()
    run(args.warmup, args.warmup + args.steps)
    torch.cuda.synchronize()
    if comm is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if os.environ.get("HIPFM_BENCH_STAMPS") and rank == 0:
        # diagnostic stamp build: per-workgroup phase stamps of the last timed step (tools/stamps.py)
        from hipfm.ops._lib import dump_stamps
        dump_stamps(os.environ["HIPFM_BENCH_STAMPS"])
    # graphs captured inside the timed window (should be 0: every run was captured before)
    timed_captures = len(model._graphs) - n_graphs
    if timed_captures and rank == 0:
        print(f"[bench] WARNING: {timed_captures} graph capture(s) inside the timed window",
              file=sys.stderr, flush=True)
    if os.environ.get("HIPFM_BENCH_DIAG") == "1" and rank == 0:
        # diagnostics (not part of the reported value): the same window re-timed after idle gaps
        for gap in (0.0, 0.0, 0.001, 0.01, 0.1, 0.5, 0.0):
            time.sleep(gap)
            t1 = time.perf_counter()
            run(args.warmup, args.warmup + args.steps)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            print(f"[bench diag] idle {gap * 1e3:6.1f} ms -> window {(time.perf_counter() - t1) * 1e3 / args.steps:.4f}"
                  f" ms/step (host enqueue {(t2 - t1) * 1e3:.3f} ms)", file=sys.stderr, flush=True)
    loss = model.loss_value(B)
    ms = elapsed * 1000.0 / max(1, args.steps)
    if comm is not None:
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())

    # eval AUC on held-out batches (distributed: every rank evaluates its shard, hist all-reduced)
    hist = torch.zeros(2, 201, dtype=torch.int64, device=dev)
    for i in range(args.eval_batches):
        ids, vals, labels = synth.batch(B, step=10_000_000 + rank * 1000 + i, device=dev,
                                        id_dtype=torch.int32)
        model.eval_batch(ids, vals, labels, hist)
    if comm is not None:
        dist.all_reduce(hist)
    auc = auc_from_hist(hist.cpu())

    value = world * B / (ms / 1000.0)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.mlp_dtype,
            "data": "synthetic (Criteo-shaped Zipf ids + teacher labels, HBM-resident), random-init weights",
            "config": {
                "model": f"DeepFM {_SHAPE_NAMES.get(args.preset, args.preset)} (F={F}, V={synth.feature_size}, "
                         f"K={args.embedding_size}, deep {args.deep_layers}, keep {args.dropout}"
                         f"{', batch norm' if args.batch_norm else ''})",
                "tower": "fused one-launch tower" if model.fused else (
                    "per-layer: hipBLASLt GEMMs + mlp.hip epilogue passes" if getattr(model, "cbuf", None) is not None and model.cbuf.numel()
                    else "per-layer GEMMs (mlp.hip)"),
                "global_batch": world * B,
                "per_gpu_batch": B,
                "seq_len": None,
                "fields": F,
                "parallelism": _parallelism(world, comm),
                "optimizer": f"{args.optimizer} ({args.sparse_update})",
                "hip_graph": use_graph,
                "timed_graph_captures": timed_captures,
                "warmup_graph_captures": warm_captures,
                "graph_steps": G if use_graph else 0,
                "exec": os.environ.get("HIPFM_BENCH_RUNG", ("graph+run-sort" if os.environ.get("HIPFM_RUN_SORT", "1") == "1"
                                                              else "graph+prefetch") if use_graph else "eager"),
                "mlp_dtype": args.mlp_dtype + (" fwd GEMMs, bf16 backward" if args.mlp_dtype == "fp8" else ""),
                "emb_dtype": args.emb_dtype + (" rows + slots (stochastic rounding), fp32 math"
                                               if args.emb_dtype == "bf16" else " tables + slots"),
                "ids_layout": "field-major [F, B]" if args.field_major_ids else "row-major [B, F]",
                "transport": ("same-device rehearsal: every rank on GPU 0, IPC staging + host barrier "
                              "(HIPFM_SAME_DEVICE=1)" if (comm is not None and same_device()) else
                              "RCCL" if comm is not None else "none (1 GPU)"),
            },
            "eval_auc": round(auc, 5),
            "train_loss": round(loss, 5),
            "hbm_peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1),
        }
        x = model.shx if model.shx is not None else model.rpx
        if x is not None:
            # modelled per-rank traffic of one step (fixed-capacity blocks): bytes sent to other
            # ranks, and bytes the step's collectives deliver incl. the rank's own block
            sb = x.step_bytes(G if use_graph else 0)
            out["comm_bytes_per_step"] = sb["sent"]
            out["comm_bytes_moved_per_step"] = sb["moved"]
            out["config"]["exchange_overlap"] = (
                "dense all-reduce beside the sparse backward (HIPFM_SH_OVERLAP=1)"
                if model._last_plan.overlap_dense else "off (one queue: dense gradient all-gathered with the rows)")
            if model.shx is not None:
                out["config"]["exchange_rows"] = (
                    f"served {'bf16 v + fp32 w' if model.shx.rbf16 else 'fp32 v + w'} ({model.shx.RWS * 4} B), "
                    f"gradient fp32 ({model.shx.RWG * 4} B); owners keep fp32 master rows + slots")
        _emit(json.dumps(out))
    model.check_errors()
    if comm is not None:
        dist.barrier()
        torch.cuda.synchronize()
        # (native RCCL communicators are left to process exit: ncclCommDestroy after graph
        # capture blocks on ROCm 7)
        dist.destroy_process_group()


def _parallelism(world: int, comm) -> str:
    """The config's parallelism label; a 1-rank run of the multi-GPU step says so (a proxy)."""
    if comm is None:
        return f"dp{world}"
    emb = "row-sharded" if comm.sharded else "replicated"
    if world == 1:
        return f"dp1 (1-rank {emb}-exchange proxy)"
    from hipfm.parallel.dist import same_device
    if same_device():
        return f"dp{world}+{emb}-embedding ({world} ranks on ONE GPU: same-device rehearsal)"
    return f"dp{world}+{emb}-embedding"


def infer_bench(args):
    """Serving throughput on one GPU: the predict path (the export's serving signature: feat_ids,
    feat_vals -> prob) of the same model and config.  Each request batch is copied into the
    model's input buffers and run through the fused forward-only tower (FM gather, MLP, sigmoid),
    and the probabilities are copied out; 16 requests are captured per HIP graph."""
    import torch
    import hipfm  # noqa: F401
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM, graph_capture

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    synth = make_synth(args.preset, seed=2024)
    B = args.batch_size
    layers = [int(x) for x in args.deep_layers.split(",")]
    keep = [float(x) for x in args.dropout.split(",")]
    model = NativeDeepFM(synth.feature_size, synth.F, args.embedding_size, layers, keep,
                         optimizer=args.optimizer, sparse_update=args.sparse_update, seed=1234,
                         batch_size=B, device=dev, field_ranges=synth.field_ranges(),
                         mlp_dtype=args.mlp_dtype, emb_dtype=args.emb_dtype)
    _progress()
    P = 16 * max(1, min(args.pool, 64) // 16)      # whole 16-request graphs
    reqs = [synth.batch(B, step=500_000 + i, device=dev, id_dtype=torch.int32) for i in range(P)]
    out = torch.zeros(P, B, device=dev)

    def serve(lo, hi):
        for i in range(lo, hi):
            ids, vals, _ = reqs[i]
            model.stage_batch(ids, vals, None)
            model.predict_enqueue(B, with_labels=False)
            out[i].copy_(model.prob[:B])
    G = 16
    serve(0, G)                                   # eager warm-up (lazy library state)
    torch.cuda.synchronize()
    graphs = []
    for g0 in range(0, P, G):
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            serve(g0, g0 + G)
        graphs.append(g)
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    _progress()
    n_rep = max(1, args.steps // P)
    t0 = time.perf_counter()
    for _ in range(n_rep):
        for g in graphs:
            g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nb = n_rep * len(graphs) * G
    # the captured path equals eager predict (spot check of the last request)
    ref = model.predict(reqs[-1][0], reqs[-1][1])
    assert torch.equal(ref, out[P - 1]), "graph-replayed predictions differ from eager predict"
    res = {"metric": "inference samples/s (1 GPU, forward-only predict path)",
           "value": round(nb * B / dt, 1), "unit": "samples/s", "n_gpus": 1,
           "us_per_batch": round(dt * 1e6 / nb, 2), "batches": nb, "batch": B,
           "higher_is_better": True, "dtype": "fp8" if args.mlp_dtype == "fp8" else "bf16",
           "data": "synthetic Criteo-shaped requests, random-init weights",
           "config": {"preset": args.preset, "K": args.embedding_size, "deep": args.deep_layers,
                      "graph_requests": G}}
    _emit(json.dumps(res))
    return 0


def data_bench(args):
    """File-fed throughput through the framework's own input path (1 GPU): the C++ TFRecord
    reader + Example decoder (host ingest alone, rows/s), then the Estimator training the same
    files -- epoch 0 streamed through pinned buffers + a copy stream and cached in HBM, later
    epochs replayed from the cache as multi-step graphs (the reference's cache() advice, DOC
    p.43-44)."""
    import torch
    import hipfm
    from hipfm.cli import _EpochView
    from hipfm.config import RunConfig
    from hipfm.data.native_io import NativeLoader
    from hipfm.data.pipeline import InputPipeline, discover_files
    from hipfm.data.synthetic import make_synth
    from hipfm.estimator import Estimator

    files = discover_files(args.data, "tr")
    va = discover_files(args.data, "va")
    if not files:
        raise SystemExit(f"no tr*.tfrecords under {args.data}")
    synth = make_synth(args.preset)
    F, B = synth.F, args.batch_size
    # 1. host ingest: read + CRC + decode into pinned int32 batches, no GPU work
    lab = torch.empty(B, pin_memory=True)
    ids = torch.empty(B, F, dtype=torch.int32, pin_memory=True)
    vals = torch.empty(B, F, pin_memory=True)
    ld = NativeLoader(files, F, B, threads=args.threads, ids32=True)
    rows, t0 = 0, time.perf_counter()
    while True:
        r = ld.next_into(lab, ids, vals)
        if r == 0:
            break
        rows += r
    ingest = rows / (time.perf_counter() - t0)
    ld.close()
    # 1b. host ingest of the GPU-decode wire: framing + raw Example bytes assembled into a ring of
    # pinned slots (the streamed path's host side, nothing on the GPU); the data CRCs checked on the
    # GPU (the pipeline's default: no per-byte host work) or on the host, interleaved twice
    slots = [(torch.empty(B * 2048, dtype=torch.uint8, pin_memory=True),
              torch.empty(B + 1, dtype=torch.int32, pin_memory=True)) for _ in range(8)]

    def ingest_raw_pass(device_crc):
        ld = NativeLoader(files, F, B, threads=args.threads, raw=True, device_crc=device_crc)
        ld.start_ring_raw(slots)
        n, nbytes, t0 = 0, 0, time.perf_counter()
        while True:
            r, slot, nb = ld.ring_take()
            if r <= 0:
                break
            n += r
            nbytes += nb
            ld.ring_give(slot)
        dt = time.perf_counter() - t0
        ld.close()
        return n / dt, nbytes, n
    raw_rates = {True: [], False: []}
    for dc in (True, False, True, False):
        rate, bytes_raw, rows_raw = ingest_raw_pass(dc)
        raw_rates[dc].append(round(rate, 1))
    ingest_raw = max(raw_rates[True])
    _progress()
    # 2. training through the Estimator (same code path as the CLI): the per-field vocabularies are
    # the data's (--field_sizes), so epoch 0 already sorts per field; streamed epochs go through
    # the staging ring as captured multi-step runs
    fr = synth.field_ranges()
    sizes = ",".join(str(hi - lo) for lo, hi in fr) if fr[0][0] == 0 and all(
        fr[i][1] == fr[i + 1][0] for i in range(len(fr) - 1)) else ""

    def train_arm(cache: bool):
        cfg = RunConfig(feature_size=synth.feature_size, field_size=F, embedding_size=args.embedding_size,
                        batch_size=B, deep_layers=args.deep_layers, dropout=args.dropout,
                        optimizer=args.optimizer, sparse_update=args.sparse_update, device="cuda",
                        log_steps=0, mlp_dtype=args.mlp_dtype, watchdog_secs=0, field_sizes=sizes,
                        graph_steps=args.graph_steps, num_threads=args.threads)
        est = Estimator(cfg)
        pipe = InputPipeline(files, F, B, 1, cache=cache, device=est.device, id_dtype=torch.int32,
                             threads=args.threads, seed=cfg.seed)
        per_epoch = []
        for e in range(args.epochs):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = est.train(_EpochView(pipe, e))
            torch.cuda.synchronize()
            per_epoch.append((n, time.perf_counter() - t0))
            if e == 0:
                est.adopt_field_ranges(pipe)
            _progress()
        return est, per_epoch, pipe

    est_s, per_epoch_s, pipe_s = train_arm(cache=False)    # every epoch streamed from the files
    # host-to-device bytes per streamed row (the last epoch's ring copies; HIPFM_WIRE_COMPACT)
    wire = round(pipe_s.h2d_bytes / max(1, per_epoch_s[-1][0] * B), 1)
    fill = {"take_s": round(pipe_s.fill_take_s, 4), "issue_s": round(pipe_s.fill_issue_s, 4)}   # (last epoch)
    if args.stream_only:                               # (profiling the streamed path alone)
        _emit(json.dumps({"metric": "streamed epochs samples/s (1 GPU)", "ingest_rows_per_s": round(ingest, 1),
                          "ingest_raw_rows_per_s": round(ingest_raw, 1),
                          "ingest_raw_passes": {"gpu_crc": raw_rates[True], "host_crc": raw_rates[False]},
                          "raw_bytes_per_row": round(bytes_raw / max(1, rows_raw), 1),
                          "streamed_epoch_samples_per_s": [round(n * B / t, 1) for n, t in per_epoch_s],
                          "epoch_s": [round(t, 4) for _, t in per_epoch_s], "wire_bytes_per_row": wire,
                          "fill_thread_last_epoch": fill,
                          "host_timer_totals_s": {k: round(v, 4) for k, v in est_s.timer.t.items()},
                          "host_timer_calls": dict(est_s.timer.n)}))
        return
    sig_s = (est_s.model.p.double().sum().item(), est_s.model.rec.double().sum().item())
    del est_s
    torch.cuda.empty_cache()
    est, per_epoch, _ = train_arm(cache=True)           # epoch 0 streamed + cached, then replayed
    sig = (est.model.p.double().sum().item(), est.model.rec.double().sum().item())
    ev = est.evaluate(InputPipeline(va, F, B, 1, device=est.device, id_dtype=torch.int32,
                                    shuffle_files=False, threads=args.threads)) if va else {"auc": None}
    sps = [n * B / t for n, t in per_epoch]
    steady = per_epoch[2:] if len(per_epoch) > 2 else per_epoch[-1:]
    steady_sps = sum(n for n, _ in steady) * B / sum(t for _, t in steady)
    sps_s = [n * B / t for n, t in per_epoch_s]
    out = {"metric": "file-fed training samples/s (1 GPU) + host ingest rows/s",
           "value": round(steady_sps, 1), "unit": "samples/s", "n_gpus": 1,
           "ingest_rows_per_s": round(ingest, 1), "ingest_threads": args.threads, "rows": rows,
           "epoch_samples_per_s": [round(x, 1) for x in sps],
           "streamed_epoch_samples_per_s": [round(x, 1) for x in sps_s],
           "streamed_bitwise_equal_cached": sig == sig_s, "wire_bytes_per_row": wire,
           "epoch0": "streamed from files (pinned ring + copy stream + staging ring of run graphs) and cached in HBM",
           "epoch1": "cache replay, graphs captured", "steady": "cache replay of captured graphs",
           "streamed": "no cache: every epoch streamed through the staging ring",
           "graph_steps": args.graph_steps, "per_field_sort": est.model.field_ranges is not None,
           "eval_auc": None if ev["auc"] is None else round(ev["auc"], 5),
           "config": {"preset": args.preset, "batch": B, "K": args.embedding_size,
                      "deep": args.deep_layers, "optimizer": f"{args.optimizer} ({args.sparse_update})",
                      "mlp_dtype": args.mlp_dtype}}
    _emit(json.dumps(out))
    return 0


def _fake_child(args, spec):
    """CPU stand-in for a bench child (tests of the supervisor): ``spec`` =
    '<rung>:<rank>:<fail|hang|stall>' entries separated by commas make that rank fail, hang before
    its first progress mark, or stall after one, in that rung; others print a line."""
    import time
    rank = int(os.environ.get("RANK", "0"))
    rung = os.environ.get("HIPFM_BENCH_RUNG", "")
    for item in spec.split(","):
        r_name, r_rank, what = item.split(":")
        if r_name == rung and int(r_rank) == rank:
            if what == "fail":
                sys.exit(3)
            if what == "stall":
                _progress()
            while True:             # hang without (further) progress
                time.sleep(1)
    _progress()
    if rank == 0:
        _emit(json.dumps({"metric": METRIC, "value": 1.0, "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                          "config": {"exec": rung}}))
    return 0


def _requested_gpus(argv) -> int:
    """--gpus N from argv without importing torch (the launching parent never touches the GPU)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ns, _ = ap.parse_known_args(argv)
    return ns.gpus


def self_launch(argv, n: int) -> int:
    """``python bench.py --gpus N`` (N > 1) outside a launcher: start one rank per GPU of this
    node (the reference's mpirun -np N / processes_per_host, NBHVD:87-92, HVD:295) through
    torch.distributed.run on 127.0.0.1, as a CHILD process -- this process has not initialised the
    GPU and only relays the exit code.  Each rank then runs the supervised bench below."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    if "WORLD_SIZE" not in os.environ and os.environ.get("HIPFM_BENCH_CHILD") != "1":
        n_req = _requested_gpus(sys.argv[1:])
        if n_req > 1:
            sys.exit(self_launch(sys.argv[1:], n_req))
    sup = os.environ.get("HIPFM_BENCH_SUPERVISE", "1")      # 0: off; force: also at 1 rank (tests)
    if (os.environ.get("HIPFM_BENCH_CHILD") != "1" and sup != "0" and "TORCHELASTIC_RUN_ID" in os.environ
            and (int(os.environ.get("WORLD_SIZE", "1")) > 1 or sup == "force")):
        sys.exit(supervise(sys.argv[1:]))
    sys.exit(main() or 0)
