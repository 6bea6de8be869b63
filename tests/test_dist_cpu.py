"""Multi-process data parallelism on CPU with gloo: the row-sharded
all-to-all algorithm and the replicated (Horovod-parity) gradient averaging both reproduce a
single-process run on the global batch; distributed evaluation sums AUC histograms."""
import os
import socket

import pytest
import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import hipfm

V, F, K, LAYERS = 600, 6, 4, [8]


def _port():
    from hipfm.utils.net import free_port
    s = socket.socket()
    s.bind(("127.0.0.1", free_port()))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(steps, B):
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(steps):
        ids = torch.randint(0, V, (B, F), generator=g)
        ids[:, 0] = 3                                         # a hot id shared by every row
        out.append((ids, torch.rand(B, F, generator=g), (torch.rand(B, generator=g) < 0.4).float()))
    return out


def _worker(rank, world, port, mode, opt, update, q):
    try:
        _worker_body(rank, world, port, mode, opt, update, q)
    except BaseException:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise


def _worker_body(rank, world, port, mode, opt, update, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipfm.models.reference import GoldenDeepFM, init_params
    from sharded_oracle import make_sharded_golden
    params = init_params(V, F, K, LAYERS, False, seed=9)
    kw = dict(keep_probs=[1.0], optimizer=opt, sparse_update=update, learning_rate=0.01, params=params)
    B = 32
    data = _batches(4, B * world)
    if mode == "sharded":
        m = make_sharded_golden(V, F, K, LAYERS, world=world, rank=rank, **kw)
        for ids, vals, lab in data:
            sl = slice(rank * B, (rank + 1) * B)
            m.train_step(ids[sl], vals[sl], lab[sl])
        fv, fw = m.full_table("fm_v"), m.full_table("fm_w")
        dense = {k: v for k, v in m.params.items() if k.startswith("Deep") or k == "fm_bias"}
    else:
        from hipfm.config import parse_flags
        m = GoldenDeepFM(V, F, K, LAYERS, world_size=world, **kw)

        def sync(grads, touched):
            out = {}
            for k, g in grads.items():
                t = g.contiguous().clone()
                dist.all_reduce(t)
                out[k] = t / world
            mask = torch.zeros(V, dtype=torch.int32)
            mask[touched] = 1
            dist.all_reduce(mask, op=dist.ReduceOp.MAX)
            return out, torch.nonzero(mask).reshape(-1)
        for ids, vals, lab in data:
            sl = slice(rank * B, (rank + 1) * B)
            m.train_step(ids[sl], vals[sl], lab[sl], grad_sync=sync)
        fv, fw = m.params["fm_v"], m.params["fm_w"]
        dense = {k: v for k, v in m.params.items() if k.startswith("Deep") or k == "fm_bias"}
    if rank == 0:
        # numpy copies: a torch tensor in a Queue travels as a shared-memory fd that dies with
        # this process, so the parent could read it only while the worker is still alive
        q.put({k: v.detach().numpy().copy() for k, v in {"fm_v": fv, "fm_w": fw, **dense}.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,opt,update", [("sharded", "Adam", "tf1_dense"), ("sharded", "Adam", "lazy"),
                                             ("sharded", "Adagrad", "lazy"), ("replicated", "Adam", "tf1_dense"),
                                             ("replicated", "ftrl", "lazy")])
def test_dp_matches_single_process_global_batch(mode, opt, update):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, opt, update, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    assert "error" not in got, got.get("error")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from hipfm.models.reference import GoldenDeepFM, init_params
    params = init_params(V, F, K, LAYERS, False, seed=9)
    ref = GoldenDeepFM(V, F, K, LAYERS, [1.0], optimizer=opt, sparse_update=update, learning_rate=0.01,
                       world_size=world, params=params)
    for ids, vals, lab in _batches(4, 32 * world):
        ref.train_step(ids, vals, lab)
    for k, v in got.items():
        v = torch.from_numpy(v)
        assert torch.allclose(v, ref.params[k], atol=2e-6, rtol=1e-5), (k, (v - ref.params[k]).abs().max())


def _eval_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipfm.ops.metrics import auc_from_hist, hist_torch
    g = torch.Generator().manual_seed(1)
    p = torch.rand(4000, generator=g)
    y = (torch.rand(4000, generator=g) < p).float()
    h = hist_torch(p[rank::world], y[rank::world])
    dist.all_reduce(h)
    if rank == 0:
        q.put((auc_from_hist(h), auc_from_hist(hist_torch(p, y))))
    dist.destroy_process_group()


def test_distributed_eval_histogram_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_eval_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    a, b = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert a == b


def test_launcher_cli_two_ranks_gloo(tmp_path):
    """python -m hipfm.launch --nproc_per_node 2 -m hipfm ... on CPU/gloo: both ranks train on
    disjoint file shards, evaluate their shard (histograms all-reduced) and save one checkpoint."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = tmp_path / "data"
    subprocess.check_call([sys.executable, os.path.join(repo, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:8000", "--train_rows", "2048",
                           "--val_rows", "512", "--files", "4"], cwd=repo)
    md = tmp_path / "model"
    env = dict(os.environ, PYTHONPATH=repo)
    r = subprocess.run([sys.executable, "-m", "hipfm.launch", "--nproc_per_node", "2",
                        "--master_port", str(_port()), "-m", "hipfm", "--task_type", "train",
                        "--training_data_dir", str(d), "--val_data_dir", str(d), "--model_dir", str(md),
                        "--feature_size", "8000", "--field_size", "39", "--embedding_size", "4",
                        "--batch_size", "64", "--deep_layers", "16", "--dropout", "1.0",
                        "--num_epochs", "1", "--device", "cpu", "--log_steps", "4"],
                       cwd=repo, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "auc = " in r.stdout
    import json as _json
    idx = _json.load(open(md / "hipfm_checkpoint.json"))
    # 2048 rows / 2 ranks / 64 per batch = 16 steps (same on both ranks: equal-steps rule)
    assert idx["latest"] == "ckpt-16"
    man = _json.load(open(md / "ckpt-16" / "manifest.json"))
    assert man["world"] == 2 and os.path.exists(md / "ckpt-16" / "rank1.bin")


def test_launcher_tf_config_mapping(monkeypatch):
    """PS-style TF_CONFIG (reference PS:414-428) -> node layout; ps/evaluator tasks idle."""
    import json
    from hipfm import launch
    cluster = {"chief": ["algo-1:2222"], "worker": ["algo-2:2222", "algo-3:2222"],
               "ps": ["algo-1:2223", "algo-2:2223", "algo-3:2223"]}
    monkeypatch.delenv("SM_HOSTS", raising=False)
    monkeypatch.setenv("TF_CONFIG", json.dumps({"cluster": cluster, "task": {"type": "worker", "index": 1}}))
    d = launch._tf_config_defaults()
    assert d == {"nnodes": 3, "node_rank": 2, "master_addr": "algo-1"}
    monkeypatch.setenv("TF_CONFIG", json.dumps({"cluster": cluster, "task": {"type": "ps", "index": 0}}))
    assert launch.main(["--nproc_per_node", "1", "-m", "hipfm"]) == 0


def _cap_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hipfm.parallel.dist import Comm
    # every rank measured a different per-peer capacity on its own batches
    c = Comm(sharded=True, capacity=64 * (rank + 1))
    q.put((rank, c.capacity))
    dist.barrier()
    dist.destroy_process_group()


def test_fixed_capacity_agreed_across_ranks():
    """The fixed-capacity all-to-all blocks must have one size on every rank: Comm takes the max
    of the per-rank capacity estimates (bench.py measures each rank's own batches)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_cap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v == 64 * world for v in got.values()), got


def test_two_rank_export_writes_one_shard_per_rank(tmp_path):
    """At world 2 every rank writes its own data shard of the TF1 checkpoint and of the
    SavedModel's variables bundle (model.ckpt-<s>.data-0000r-of-00002), rank 0 the merged index
    and saved_model.pb; the bundles read back complete."""
    import subprocess
    import sys
    from hipfm.ckpt import tf_bundle as tb
    from hipfm.ckpt.export import latest_export, load_servable
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = tmp_path / "data"
    subprocess.check_call([sys.executable, os.path.join(repo, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:300000", "--train_rows", "1024",
                           "--val_rows", "256", "--files", "2"], cwd=repo)
    md, ex = tmp_path / "model", tmp_path / "export"
    r = subprocess.run([sys.executable, "-m", "hipfm.launch", "--nproc_per_node", "2",
                        "--master_port", str(_port()), "-m", "hipfm", "--task_type", "train",
                        "--training_data_dir", str(d), "--val_data_dir", str(d), "--model_dir", str(md),
                        "--servable_model_dir", str(ex), "--feature_size", "300000", "--field_size", "39",
                        "--embedding_size", "4", "--batch_size", "64", "--deep_layers", "16",
                        "--dropout", "1.0", "--num_epochs", "1", "--device", "cpu", "--log_steps", "100"],
                       cwd=repo, env=dict(os.environ, PYTHONPATH=repo), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    prefix = str(md / "model.ckpt-8")
    for k in range(2):
        assert os.path.getsize(tb.data_path(prefix, k, 2)) > 0      # both ranks wrote a shard
    ck = tb.read_bundle(prefix)
    assert ck["fm_v"].shape == (300000, 4) and "fm_v/Adam" in ck and int(ck["global_step"]) == 8
    e = latest_export(str(ex))
    assert os.path.exists(os.path.join(e, "saved_model.pb"))
    sv = tb.read_bundle(os.path.join(e, "variables", "variables"))
    assert "fm_v/Adam" not in sv and np.array_equal(sv["fm_v"], ck["fm_v"])
    p = load_servable(e).predict(torch.zeros(3, 39, dtype=torch.int64), torch.ones(3, 39))
    assert p.shape == (3,)


def _ranges_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hipfm.data.pipeline import agreed_field_ranges

        class _Shard:                   # a rank's cached epoch: field f ids in [100 f, 100 f + 100)
            def field_minmax(self):
                # rank 0 saw small ids of field 1, rank 1 only large ones (and vice versa field 2)
                mn = torch.tensor([0, 130 if rank == 0 else 101, 200 if rank == 0 else 240])
                mx = torch.tensor([50, 150 if rank == 0 else 190, 220 if rank == 0 else 299])
                return mn, mx
        r = agreed_field_ranges(_Shard(), 1000, world)
        q.put({"rank": rank, "ranges": r})
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise


def test_field_ranges_agreed_over_all_ranks_shards():
    """ranges derived from one rank's shard can miss another rank's ids; the agreed
    ranges cover the union of every rank's min / max (and are identical on every rank)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_ranges_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert "error" not in r, r.get("error")
    a, b = (r["ranges"] for r in sorted(res, key=lambda r: r["rank"]))
    assert a == b == [(0, 101), (101, 200), (200, 1000)]


def _lockstep_worker(rank, world, port, lens, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hipfm.estimator import agree_cache, lockstep_batches
        seen = [b for b in lockstep_batches(list(range(lens[rank])), None, True)]
        capped = [b for b in lockstep_batches(list(range(lens[rank])), 2, True)]

        class _Pipe:                           # rank 0 alone outgrew its cache budget
            def __init__(self, cached):
                self._cached = [1] if cached else None
                self.dropped = False

            def drop_cache(self):
                self._cached, self.dropped = None, True
        p = _Pipe(cached=rank != 0)
        kept = agree_cache(p, world)
        q.put({"rank": rank, "seen": seen, "capped": capped, "kept": kept, "cached": p._cached})
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise


def test_eval_lockstep_and_cache_agreement_unequal_shards():
    """Distributed evaluation / predict over shards of unequal length (3 gloo ranks with 4, 1 and
    0 batches): every rank takes the same number of steps -- exhausted ranks get None, the slot in
    which they join the others' collective forward with a dummy batch -- and a rank alone over its
    cache budget makes EVERY rank drop its cache (one collective sequence on the communicator)."""
    world, lens = 3, [4, 1, 0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_lockstep_worker, args=(r, world, port, lens, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
    for r in res:
        assert "error" not in r, r.get("error")
    for r in res:
        n = lens[r["rank"]]
        assert len(r["seen"]) == 4
        assert r["seen"] == list(range(n)) + [None] * (4 - n)
        assert len(r["capped"]) == 2
        assert r["kept"] is False and r["cached"] is None
