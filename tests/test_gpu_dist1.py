"""The multi-rank executor code paths on ONE GPU: a 1-rank RCCL group with ``force_exchange``
runs the full row-sharded (sort -> unique -> all-to-all ids/rows -> fused backward -> all-to-all
grads -> owner dedup -> row update) and replicated (all-gather of unique rows) paths, which must
reproduce the single-rank fused path.  Real 2..8-GPU runs happen in the driver's scaling bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402
from hipfm.parallel.dist import Comm  # noqa: E402


@pytest.fixture(scope="module")
def group():
    if not dist.is_initialized():
        from hipfm.utils.net import free_port
        s = socket.socket()
        s.bind(("127.0.0.1", free_port()))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.fixture(autouse=True)
def _xrows(monkeypatch, request):
    """Exchanged rows: fp32 (bitwise the local step's reads) unless a test asks for bf16."""
    import hipfm.models.deepfm as D
    monkeypatch.setattr(D, "_XROWS", getattr(request, "param", "fp32"))


@pytest.mark.parametrize("sharded,update,prefetch", [(True, "lazy", False), (True, "tf1_dense", False),
                                                     (False, "lazy", False), (True, "lazy", True),
                                                     (False, "tf1_dense", False), (False, "lazy", True)])
def test_exchange_paths_match_local(group, sharded, update, prefetch):
    synth = make_synth("total:6000", seed=21)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=2)
    kw = dict(sparse_update=update, batch_size=512, device="cuda", init=False)
    a = NativeDeepFM(V, F, K, layers, keep, **kw)
    b = NativeDeepFM(V, F, K, layers, keep, comm=Comm(sharded=sharded, force_exchange=True), **kw)
    a.load_tf_params(params)
    b.load_tf_params(params)
    assert b.exchange and b.sharded == sharded
    data = [synth.batch(512, step=s % 3, device="cuda", id_dtype=torch.int32) for s in range(6)]
    for s in range(6):
        ids, vals, labels = data[s]
        a.train_step(ids, vals, labels)
        nxt = data[s + 1][0] if (prefetch and s + 1 < 6) else None
        # native RCCL engine: captured into graphs (next batch's routing on a side stream)
        b.train_step(ids, vals, labels, use_graph=True, next_ids=nxt)
    torch.cuda.synchronize()
    assert torch.allclose(a.tv, b.tv, atol=1e-6) and torch.allclose(a.tw, b.tw, atol=1e-6)
    assert torch.allclose(a.p, b.p, atol=1e-6)
    assert b.comm.bytes_sent > 0


def test_exchange_staged_batches_graph_replay(group):
    """Loader-style batches (int64 ids, staged into the model's own input buffers every step) on
    the row-sharded exchange with HIP graphs: routing is inline every step (staged content changes
    under the same addresses) and the routing sets rotate; must equal the local path."""
    synth = make_synth("total:6000", seed=23)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=5)
    kw = dict(sparse_update="lazy", batch_size=512, device="cuda", init=False)
    a = NativeDeepFM(V, F, K, layers, keep, **kw)
    b = NativeDeepFM(V, F, K, layers, keep, comm=Comm(sharded=True, force_exchange=True), **kw)
    a.load_tf_params(params)
    b.load_tf_params(params)
    for s in range(5):
        ids, vals, labels = synth.batch(512, step=s)               # CPU, int64: staged path
        a.train_step(ids, vals, labels)
        b.train_step(ids, vals, labels, use_graph=True)
    torch.cuda.synchronize()
    assert len(b._graphs) == b.shx.NSETS                           # ("staged", B) x routing sets
    assert torch.allclose(a.tv, b.tv, atol=1e-6) and torch.allclose(a.p, b.p, atol=1e-6)


def test_exchange_graph_runs_bitwise(group):
    """Row-sharded lazy step with multi-step graphs (routing of the next batch prefetched, its ids
    exchanged in the step's last collective group) gives bitwise the parameters of the same
    schedule launched eagerly step by step, and two graph runs are bitwise equal."""
    synth = make_synth("total:6000", seed=29)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=7)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]

    def run(graph):
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", batch_size=512, device="cuda",
                         init=False, comm=Comm(sharded=True, force_exchange=True))
        m.load_tf_params(params)
        for _ in range(3):                       # capture, then replays of the 4-step graphs
            if graph:
                m.train_steps(pool, next_ids=pool[0][0])
            else:
                for i, (ids, vals, lab) in enumerate(pool):
                    m.train_step(ids, vals, lab, next_ids=pool[(i + 1) % 4][0])
        torch.cuda.synchronize()
        m.check_errors()
        return m

    a, b, c = run(True), run(False), run(True)
    for x in (b, c):
        assert torch.equal(a.tv, x.tv) and torch.equal(a.tw, x.tw) and torch.equal(a.p, x.p)


def test_exchange_field_major_batches_bitwise(group):
    """Row-sharded step (1-rank RCCL group) on field-major resident batches: the routing sorts
    read them without a transpose; bitwise equal to row-major batches."""
    synth = make_synth("total:6000", seed=31)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=8)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]
    out = []
    for fm in (True, False):
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", batch_size=512, device="cuda",
                         init=False, comm=Comm(sharded=True, force_exchange=True),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        bl = [(i.t().contiguous().t() if fm else i, v, lab) for i, v, lab in pool]
        assert m._resident(*bl[0])
        for _ in range(2):
            m.train_steps(bl, next_ids=bl[0][0])
        torch.cuda.synchronize()
        m.check_errors()
        out.append((m.tv.clone(), m.tw.clone(), m.p.clone()))
    for x, y in zip(*out):
        assert torch.equal(x, y)


@pytest.mark.parametrize("update,fm,_xrows", [("lazy", False, "fp32"), ("tf1_dense", False, "fp32"),
                                              ("lazy", True, "fp32"), ("lazy", True, "bf16"),
                                              ("tf1_dense", False, "bf16")], indirect=["_xrows"])
def test_exchange_run_routing_bitwise(group, monkeypatch, update, fm, _xrows):
    """Run-level routing (FixedCapacityExchange.route_run: every batch of a multi-step graph
    sorted, routed and its ids exchanged at the graph's start; each step serves its rows inline)
    gives bitwise the parameters of the per-step pipelined routing (side-stream routing, serve
    ahead) and of single steps; the routed sets hold exactly each batch's routing."""
    import hipfm.models.deepfm as D
    synth = make_synth("total:6000", seed=37)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=9)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(5)]
    pool = [(i.t().contiguous().t() if fm else i, v, lab) for i, v, lab in pool]
    out = []
    for run, graph in ((True, True), (False, True), (False, False)):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, batch_size=512, device="cuda",
                         init=False, comm=Comm(sharded=True, force_exchange=True),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        for _ in range(3):
            if graph:
                m.train_steps(pool[:3], next_ids=(pool[3][0], pool[4][0]))
                m.train_steps(pool[3:], next_ids=(pool[0][0], pool[1][0]))
            else:
                for i, (ids, vals, lab) in enumerate(pool):
                    m.train_step(ids, vals, lab, next_ids=pool[(i + 1) % 5][0])
        torch.cuda.synchronize()
        m.check_errors()
        if run:
            assert len(m.shx.run_sets) == 3
            rs = m.shx.run_sets[0]                 # the last run routed pool[3], pool[4]
            n = 512 * F
            ids = pool[3][0].reshape(-1) if not fm else pool[3][0].contiguous().reshape(-1)
            rk, _ = torch.sort(ids.long(), stable=True)
            assert torch.equal(rs.sorted_keys[:n].long(), rk)
            assert int(rs.num_u.item()) == int(torch.unique(ids).numel())
        out.append((m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()))
        del m
    for ref in out[1:]:
        for x, y in zip(out[0], ref):
            assert torch.equal(x, y)


def test_exchange_growing_runs_keep_earlier_graphs_valid(group, monkeypatch):
    """Run routing: a longer run grows the packed ids buffer; graphs captured from shorter runs
    keep reading their own (retired, not freed) buffers and descriptors, so replaying them after
    the growth is bitwise the per-step pipelined routing."""
    import hipfm.models.deepfm as D
    synth = make_synth("total:6000", seed=38)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=10)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(6)]
    order = [(0, 2), (2, 4), (0, 6), (2, 4), (4, 6), (0, 6), (2, 4)]
    out = []
    for run in (True, False):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(V, F, K, layers, keep, batch_size=512, device="cuda", init=False,
                         comm=Comm(sharded=True, force_exchange=True), field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        for lo, hi in order:
            m.train_steps(pool[lo:hi], next_ids=(pool[hi % 6][0], pool[(hi + 1) % 6][0]))
        torch.cuda.synchronize()
        m.check_errors()
        if run:
            assert len(m.shx._run_retired) >= 1          # the growth happened
        out.append((m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()))
        del m
    for x, y in zip(*out):
        assert torch.equal(x, y)


def test_replicated_growing_runs_keep_earlier_graphs_valid(group, monkeypatch):
    """Replicated run steps: a run longer than the packed run-ids buffers regrows them; graphs
    captured from shorter runs keep their own (retired) ids buffers and route descriptors, so
    replaying them after the growth is bitwise the per-step path."""
    import hipfm.models.deepfm as D
    from hipfm.parallel.replicated import ReplicatedExchange
    monkeypatch.setattr(ReplicatedExchange, "RUN_CAP0", 2)
    synth = make_synth("total:6000", seed=39)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=11)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(6)]
    order = [(0, 2), (2, 4), (0, 6), (2, 4), (4, 6), (0, 6), (2, 4)]
    out = []
    for run in (True, False):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", batch_size=512, device="cuda",
                         init=False, comm=Comm(sharded=False, force_exchange=True),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        for lo, hi in order:
            m.train_steps(pool[lo:hi], next_ids=pool[hi % 6][0])
        torch.cuda.synchronize()
        m.check_errors()
        if run:
            assert len(m.rpx._retired) >= 1 and m.rpx.run_ids.shape[0] >= 6     # the growth happened
        out.append((m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()))
        del m
    for x, y in zip(*out):
        assert torch.equal(x, y)


@pytest.mark.parametrize("sharded", [True, False])
def test_estimator_calibrates_exchange_capacity(group, tmp_path, sharded):
    """the CLI's multi-GPU path ran on default_capacity (1.5x slots / N, ~3-4x the
    measured need).  After the first epoch is cached the Estimator measures the capacity on the
    cached batches (agreed MAX over ranks) and re-plans the exchange; training then continues on
    the calibrated exchange (graph replays from the cache) without a capacity error."""
    from hipfm.config import RunConfig
    from hipfm.data import native_io as nio
    from hipfm.data.pipeline import InputPipeline
    from hipfm.cli import _EpochView
    from hipfm.estimator import Estimator
    from hipfm.parallel.sharded import default_capacity
    synth = make_synth("total:6000", seed=41)
    F, B = synth.F, 512
    for k in range(2):
        ids, vals, lab = synth.batch(B * 4, step=k)
        nio.write_examples(str(tmp_path / f"tr-{k}.tfrecords"), lab.numpy(), ids.numpy(), vals.numpy())
    cfg = RunConfig(feature_size=synth.feature_size, field_size=F, embedding_size=8, batch_size=B,
                    deep_layers="64,32", dropout="1,1", sparse_update="lazy", device="cuda", log_steps=0,
                    watchdog_secs=0, graph_steps=4)
    est = Estimator(cfg)
    comm = Comm(sharded=sharded, force_exchange=True)
    est.model = NativeDeepFM(synth.feature_size, F, 8, [64, 32], [1.0, 1.0], sparse_update="lazy",
                             batch_size=B, device="cuda", comm=comm)
    m = est.model
    before = m.exchange_capacity()
    n = B * F
    assert before == (default_capacity(n, 1) + 63) // 64 * 64 if sharded else before >= n
    pipe = InputPipeline(sorted(str(p) for p in tmp_path.glob("tr-*")), F, B, 1, cache=True,
                         device=est.device, id_dtype=torch.int32, id_limit=synth.feature_size)
    est.train(_EpochView(pipe, 0))
    assert est.calibrate_exchange(pipe)
    after = m.exchange_capacity()
    uniq = max(int(torch.unique(b[0]).numel()) for b in pipe._cached)
    assert uniq <= after < before and after <= int(uniq * 1.3 + 1024) + 64
    est.train(_EpochView(pipe, 1))
    torch.cuda.synchronize()
    m.check_errors()
    assert est.global_step == 2 * len(pipe._cached)


@pytest.mark.parametrize("mode", ["fp8", "emb_bf16", "batch_norm", "tf1_dense_momentum", "replicated_fp8"])
def test_exchange_mode_matrix(group, mode):
    """the mode combinations the executor supports on the exchange path, each on
    the 1-rank RCCL group (force_exchange: the complete multi-GPU step, collectives included)
    against the local step over multi-step graphs: fp8 MLP x row-sharded, bf16 embeddings x
    row-sharded, batch norm x row-sharded (per-layer tower), tf1_dense x Momentum x row-sharded
    graphs, fp8 x replicated-table DP."""
    synth = make_synth("total:6000", seed=43)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, mode == "batch_norm", seed=11)
    kw = dict(sparse_update="lazy", batch_size=512, device="cuda", init=False,
              field_ranges=synth.field_ranges())
    sharded = True
    if mode in ("fp8", "replicated_fp8"):
        kw["mlp_dtype"] = "fp8"
        sharded = mode == "fp8"
    elif mode == "emb_bf16":
        kw["emb_dtype"] = "bf16"
    elif mode == "batch_norm":
        kw["batch_norm"] = True
    else:
        kw.update(sparse_update="tf1_dense", optimizer="Momentum")
    a = NativeDeepFM(V, F, K, layers, keep, **kw)
    b = NativeDeepFM(V, F, K, layers, keep, comm=Comm(sharded=sharded, force_exchange=True), **kw)
    a.load_tf_params(params)
    b.load_tf_params(params)
    assert b.exchange
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]
    for _ in range(2):
        a.train_steps(pool)
        b.train_steps(pool)
    torch.cuda.synchronize()
    b.check_errors()
    assert a.global_step() == b.global_step() == 8
    tol = 1e-6 if mode != "emb_bf16" else 2e-3
    assert torch.allclose(a.tv.float(), b.tv.float(), atol=tol) and torch.allclose(a.tw, b.tw, atol=1e-6)
    assert torch.allclose(a.p, b.p, atol=1e-6)


@pytest.mark.parametrize("emb", ["fp32", "bf16"])
def test_bf16_exchange_rows(group, emb):
    """Compact exchanged rows (v as bf16 + fp32 w: 24 B instead of 48 at K = 8; gradient rows
    K + 1 words).  A bf16 table's rows convert exactly: bitwise the fp32-row exchange.  An fp32
    table's forward / backward read bf16-rounded v (the compute dtype) while the owner keeps fp32
    master rows and optimizer state: close to the local step, not bitwise."""
    synth = make_synth("total:6000", seed=47)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=12)
    kw = dict(sparse_update="lazy", batch_size=512, device="cuda", init=False,
              field_ranges=synth.field_ranges(), emb_dtype=emb)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]
    out = []
    for xr in ("bf16", "fp32", None):
        comm = Comm(sharded=True, force_exchange=True) if xr else None
        m = NativeDeepFM(V, F, K, layers, keep, comm=comm, exchange_rows=xr, **kw)
        m.load_tf_params(params)
        p0 = m.p.clone()
        if xr:
            assert m.shx.rbf16 == (xr == "bf16")
            assert m.shx.RWS == (K // 2 + 2 if xr == "bf16" else K + 4) and m.shx.RWG == K + 1
        for _ in range(2):
            m.train_steps(pool, next_ids=(pool[0][0], pool[1][0]))
        torch.cuda.synchronize()
        m.check_errors()
        out.append((m.tv.float().clone(), m.tw.clone(), m.p.clone()))
        del m
    (bv, bw, bp), (fv, fw, fp), (lv, lw, lp) = out
    if emb == "bf16":
        assert torch.equal(bv, fv) and torch.equal(bw, fw) and torch.equal(bp, fp)
    else:
        assert torch.equal(fv, lv) or torch.allclose(fv, lv, atol=1e-6)
        # Adam normalizes each row's step, so a near-zero gradient whose sign the bf16 reads flip
        # moves that element by ~2 lr: compare the whole update, not the worst element
        v0 = torch.as_tensor(params["fm_v"]).to("cuda").float()
        w0 = torch.as_tensor(params["fm_w"]).to("cuda").float().reshape(-1)
        for b_, l_, x0 in ((bv, lv, v0), (bw, lw, w0)):
            b_, l_ = b_[: x0.shape[0]].reshape(x0.shape), l_[: x0.shape[0]].reshape(x0.shape)
            du = (b_ - x0) - (l_ - x0)
            assert du.norm().item() <= 0.05 * (l_ - x0).norm().item()
        assert ((bp - p0) - (lp - p0)).norm().item() <= 0.05 * (lp - p0).norm().item()
        assert not torch.equal(bv, lv)           # the bf16 reads did change the arithmetic


@pytest.mark.parametrize("update", ["lazy", "tf1_dense"])
def test_replicated_run_sort_bitwise(group, monkeypatch, update):
    """Replicated-table exchange (config #3) on the run-level sort: every batch of a multi-step
    graph sorted and routed at the graph's start, its ids gathered once, each step's requests
    tagged by its own sparse launch (tf1_dense split form: flagged for the owner launch's sweep
    too) -- one queue, no per-step sort branch.  Bitwise the per-step prefetched-sort path."""
    import hipfm.models.deepfm as D
    synth = make_synth("total:6000", seed=53)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=13)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]
    out = []
    for run in (True, False):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, batch_size=512, device="cuda",
                         init=False, comm=Comm(sharded=False, force_exchange=True),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        assert m.rpx is not None and (update == "lazy" or m.tf1_xsplit)
        for _ in range(3):
            m.train_steps(pool, next_ids=pool[0][0])
        torch.cuda.synchronize()
        m.check_errors()
        assert any(k[0] == "runsort" for k in m._graphs) == run
        out.append((m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()))
        del m
    for x, y in zip(*out):
        assert torch.equal(x, y)


@pytest.mark.parametrize("sharded,opt", [(True, "Adam"), (False, "Adam"), (True, "Adagrad")])
def test_tf1_split_under_exchange_equals_scatter_sweep(group, monkeypatch, sharded, opt):
    """tf1_dense (TF1 non-lazy optimizer semantics) under the native exchange: the split form --
    requested rows updated by the lazy owner launch and flagged (serve / tag kernel), every other
    row by the l2-only sweep workgroups of the same launch -- equals the gradient scatter + full
    table sweep form bitwise, over run graphs and single steps; every row moved."""
    import hipfm.models.deepfm as D
    synth = make_synth("total:6000", seed=59)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=14)
    pool = [synth.batch(512, step=s, device="cuda", id_dtype=torch.int32) for s in range(4)]
    out = []
    for split in (True, False):
        monkeypatch.setattr(D, "_TF1_SPLIT", split)
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update="tf1_dense", optimizer=opt, l2_reg=1e-3,
                         adam_epsilon=1e-2, batch_size=512, device="cuda", init=False,
                         comm=Comm(sharded=sharded, force_exchange=True), field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        assert m.tf1_xsplit == split
        t0 = m.tv.clone()
        for _ in range(2):
            m.train_steps(pool, next_ids=(pool[0][0], pool[1][0]))
        for i in range(3):
            m.train_step(*pool[i], use_graph=True)
        torch.cuda.synchronize()
        m.check_errors()
        if split:
            assert int(m._xflags.sum().item()) == 0          # the sweep cleared every flag
            moved = (m.tv != t0).any(dim=1)
            assert bool(moved[:V].all())                      # non-lazy: every row moved
        out.append((m.tv.clone(), m.tw.clone(), [s.clone() for s in m.sv], m.p.clone(), m.step.clone()))
        del m
    (av, aw, asv, ap, ast), (bv, bw, bsv, bp, bst) = out
    assert torch.equal(av, bv) and torch.equal(aw, bw) and torch.equal(ap, bp) and torch.equal(ast, bst)
    for x, y in zip(asv, bsv):
        assert torch.equal(x, y)
