"""Row-sharded fixed-capacity exchange (parallel/sharded.py + csrc/kernels/shard.hip) with N > 1
ranks on ONE GPU: N model instances run in N threads, each on its own HIP stream, and the
all-to-all / all-reduce of the native RCCL engine are replaced by stream-ordered copies between
the instances (MeshEngine).  Every HIP kernel of the multi-GPU step runs exactly as on N GPUs
(bucketing by owner = id % N, serving, owner-side rank-ordered sums, row updates); only the
transport differs.  The sharded run must reproduce one model trained on the global batch."""
import gc
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _fp32_exchange_rows(monkeypatch):
    """These tests compare N emulated ranks with ONE model on the global batch to 2e-5: fp32
    exchanged rows (the one-GPU step's reads).  bf16 rows: tests/test_gpu_dist1.py."""
    import hipfm.models.deepfm as D
    monkeypatch.setattr(D, "_XROWS", "fp32")


class _Hub:
    def __init__(self, N):
        self.N = N
        self.bar = threading.Barrier(N, timeout=60)
        self.slots = [None] * N
        self.done = [None] * N


class MeshEngine:
    """Stream-ordered stand-in for the RCCL engine between N in-process ranks."""

    def __init__(self, hub, rank):
        self.hub, self.rank, self.world = hub, rank, hub.N
        self.bytes_sent = 0

    def _publish(self, t):
        s = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(s)
        self.hub.slots[self.rank] = (t, ev)
        self.hub.bar.wait()
        return s

    def _finish(self, s):
        ev = torch.cuda.Event()
        ev.record(s)
        self.hub.done[self.rank] = ev
        self.hub.bar.wait()
        for p in range(self.world):           # peers finished reading my buffer
            s.wait_event(self.hub.done[p])
        self.hub.bar.wait()

    def alltoall(self, send, recv, bytes_per_peer):
        self.bytes_sent += bytes_per_peer * self.world
        s = self._publish(send)
        N, r = self.world, self.rank
        dst = recv.view(-1).view(torch.uint8).view(N, bytes_per_peer)
        for p in range(N):
            sp, evp = self.hub.slots[p]
            s.wait_event(evp)
            dst[p].copy_(sp.view(-1).view(torch.uint8).view(N, bytes_per_peer)[r])
        self._finish(s)

    def allgather(self, send, recv, bytes_per_rank):
        self.bytes_sent += bytes_per_rank * self.world
        s = self._publish(send)
        dst = recv.view(-1).view(torch.uint8).view(self.world, bytes_per_rank)
        for p in range(self.world):
            sp, evp = self.hub.slots[p]
            s.wait_event(evp)
            dst[p].copy_(sp.view(-1).view(torch.uint8))
        self._finish(s)

    def allreduce_(self, t):
        s = self._publish(t)
        acc = torch.zeros_like(t)
        for p in range(self.world):            # fixed rank order on every rank
            tp, evp = self.hub.slots[p]
            s.wait_event(evp)
            acc += tp
        self._finish(s)
        t.copy_(acc)

    def group(self, ops):
        """Grouped collectives (RcclEngine.group): run one after the other, same order on every
        rank (every op is a barrier-synchronized exchange between the in-process ranks)."""
        from hipfm.ops import kernels as KN
        for kind, send, recv, nb in ops:
            if kind == KN.COMM_A2A:
                self.alltoall(send, recv, nb)
            elif kind == KN.COMM_ALLGATHER:
                self.allgather(send, recv, nb)
            else:
                assert send.data_ptr() == recv.data_ptr()
                self.allreduce_(recv)


class MeshComm:
    def __init__(self, hub, rank, capacity=None, sharded=True):
        self.world_size, self.rank = hub.N, rank
        self.sharded = sharded
        self.force_exchange = False
        self.engine = MeshEngine(hub, rank)
        self.capacity = capacity
        self.graph_safe = False

    @property
    def bytes_sent(self):
        return self.engine.bytes_sent


def _rank_threads(models, fn, wait_origin=True):
    """Run ``fn(r)`` for every emulated rank r in its own thread, on its own HIP stream.
    torch's pool streams are non-blocking with respect to the legacy default stream, so every
    rank stream first waits for the stream that built the models (weights loaded, tables filled
    -- ``wait_origin``): without that wait a rank's first step can read embedding rows the fill
    kernels have not written yet.  Whether it does depends on whether anything (a hipMalloc by a
    cold caching allocator) happens to synchronize the device first -- the round-4 n8 failure
    that appeared only in the one-process GPU suite (test_rank_streams_wait_for_model_setup)."""
    errs = []
    origin = torch.cuda.current_stream()

    def body(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            if wait_origin:
                s.wait_stream(origin)
            with torch.cuda.stream(s):
                fn(r)
            s.synchronize()
        except BaseException as e:          # surface failures instead of hanging the barrier
            errs.append(e)
            for m in models:
                m.comm.engine.hub.bar.abort()
    th = [threading.Thread(target=body, args=(r,)) for r in range(len(models))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    if errs:
        raise errs[0]


def _run_ranks(models, batches, prefetch=False, wait_origin=True):
    def fn(r):
        bl = batches[r]
        for i, (ids, vals, lab) in enumerate(bl):
            nxt = bl[i + 1][0] if (prefetch and i + 1 < len(bl)) else None
            if prefetch == 2 and nxt is not None:      # two batches ahead
                nxt = (nxt, bl[i + 2][0] if i + 2 < len(bl) else None)
            models[r].train_step(ids, vals, lab, next_ids=nxt)
    _rank_threads(models, fn, wait_origin)


@pytest.mark.parametrize("N,opt,update,prefetch", [(2, "Adam", "lazy", False), (3, "Adagrad", "lazy", True),
                                                   (4, "Adam", "tf1_dense", False), (4, "Adam", "lazy", True),
                                                   (3, "Adam", "lazy", 2), (2, "ftrl", "tf1_dense", 2)])
def test_sharded_exchange_matches_global_batch(N, opt, update, prefetch):
    synth = make_synth("criteo_kaggle", seed=4)
    F, K, layers, keep, B = synth.F, 8, [64, 32], [1.0, 1.0], 512
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=7)
    lr = 1e-3
    steps = 3
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    ref = NativeDeepFM(V, F, K, layers, keep, optimizer=opt, sparse_update=update, learning_rate=lr * N,
                       batch_size=N * B, device=DEV, init=False, field_ranges=synth.field_ranges())
    ref.load_tf_params(params)
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, layers, keep, optimizer=opt, sparse_update=update, learning_rate=lr,
                         batch_size=B, device=DEV, init=False, comm=MeshComm(hub, r),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        assert m.shx is not None and m.shx.N == N
        models.append(m)
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    _run_ranks(models, batches, prefetch)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
        assert torch.equal(m.p, models[0].p)            # identical dense state on every rank
    full_v = torch.zeros_like(ref.tv)
    full_w = torch.zeros_like(ref.tw)
    for r, m in enumerate(models):
        rows = full_v[r::N].shape[0]
        full_v[r::N] = m.tv[:rows]
        full_w[r::N] = m.tw[:rows]
    scale = ref.tv.abs().max().item()
    assert (full_v - ref.tv).abs().max().item() <= 2e-5 * scale
    assert (full_w - ref.tw).abs().max().item() <= 2e-5 * max(1.0, ref.tw.abs().max().item())
    assert (models[0].p - ref.p).abs().max().item() <= 2e-5 * ref.p.abs().max().item()
    # something was actually exchanged, and untouched rows kept their initial values
    assert models[0].comm.bytes_sent > 0


def _run_ranks_steps(models, batches):
    """Each emulated rank trains its batches as ONE run (train_steps: run-level routing)."""
    _rank_threads(models, lambda r: models[r].train_steps(batches[r]))


@pytest.mark.parametrize("N,update,steps", [(2, "lazy", 3), (4, "lazy", 3), (3, "tf1_dense", 3), (4, "lazy", 5),
                                            (3, "lazy", 4)])
def test_run_routing_matches_global_batch(N, update, steps):
    """Run-level routing at N > 1 (emulated ranks, real data movement between them): every batch
    of the run routed and its ids exchanged in ONE packed all-to-all at the start, each step then
    G1 (rows) + G2 (gradients + dense), the next step's rows served inside the tower launch and
    patched by the owner update.  Bitwise equal to the per-step pipelined routing on the same
    emulated ranks; close to the global-batch model (the per-step test's tolerance: 3 steps --
    longer runs of Adam amplify fp32 summation-order differences on near-zero gradients); every
    rank issues the same collective sequence."""
    from hipfm.ops import kernels as KN
    import hipfm.models.deepfm as D
    synth = make_synth("criteo_kaggle", seed=4)
    F, K, layers, keep, B = synth.F, 8, [64, 32], [1.0, 1.0], 512
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=7)
    lr = 1e-3
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    outs = []
    old = D._RUN_SORT
    try:
        for run in (True, False):
            D._RUN_SORT = run
            hub = _Hub(N)
            models = []
            for r in range(N):
                m = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, learning_rate=lr, batch_size=B,
                                 device=DEV, init=False, comm=MeshComm(hub, r), field_ranges=synth.field_ranges())
                m.load_tf_params(params)
                m.shx.trace = []
                models.append(m)
            if run:
                _run_ranks_steps(models, batches)
            else:
                _run_ranks(models, batches, prefetch=2)
            torch.cuda.synchronize()
            for m in models:
                m.check_errors()
                assert torch.equal(m.p, models[0].p)
                assert len(m.shx.run_sets) == (steps if run else 0)
            outs.append(models)
    finally:
        D._RUN_SORT = old
    for a, b in zip(*outs):                               # run routing == pipelined, bitwise
        assert torch.equal(a.tv, b.tv) and torch.equal(a.tw, b.tw) and torch.equal(a.p, b.p)
    models = outs[0]
    if steps == 3:
        ref = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, learning_rate=lr * N,
                           batch_size=N * B, device=DEV, init=False, field_ranges=synth.field_ranges())
        ref.load_tf_params(params)
        for ids, vals, lab in data:
            ref.train_step(ids, vals, lab)
        full_v, full_w = torch.zeros_like(ref.tv), torch.zeros_like(ref.tw)
        for r, m in enumerate(models):
            rows = full_v[r::N].shape[0]
            full_v[r::N] = m.tv[:rows]
            full_w[r::N] = m.tw[:rows]
        scale = ref.tv.abs().max().item()
        assert (full_v - ref.tv).abs().max().item() <= 2e-5 * scale
        assert (full_w - ref.tw).abs().max().item() <= 2e-5 * max(1.0, ref.tw.abs().max().item())
        assert (models[0].p - ref.p).abs().max().item() <= 2e-5 * ref.p.abs().max().item()
    traces = [m.shx.trace for m in models]
    for t in traces[1:]:
        assert t == traces[0]
    C, RWS, RWG = models[0].shx.C, models[0].shx.RWS, models[0].shx.RWG
    t = traces[0]
    assert t[0] == ((KN.COMM_A2A, steps * C * 4),)               # the run's ids, one all-to-all
    assert len(t) == 1 + 2 * steps
    for j in range(steps):
        assert t[1 + 2 * j] == ((KN.COMM_A2A, C * RWS * 4),)      # G1: rows only
        assert t[2 + 2 * j][0] == (KN.COMM_A2A, C * RWG * 4)      # G2: gradient rows first


@pytest.mark.parametrize("N,run,sharded,update", [(2, True, True, "lazy"), (4, True, True, "lazy"),
                                                   (3, False, True, "lazy"), (3, False, False, "lazy"),
                                                   (3, False, True, "tf1_dense"), (2, True, True, "tf1_dense"),
                                                   (2, False, False, "tf1_dense")])
def test_overlapped_exchange_matches_default(monkeypatch, N, run, sharded, update):
    """HIPFM_SH_OVERLAP: the dense gradient in its own launch after the tower,
    all-reduced on the main stream (G2a) while the sparse backward runs on a graph branch, the
    gradient rows after the join (G2b).  Same parameters as the default exchange (all-gathered
    dense gradient summed in rank order by the owner launch) to fp32 reassociation, identical on
    every rank, one G2a all-reduce + one G2b group per step, identical sequences on every rank."""
    from hipfm.ops import kernels as KN
    import hipfm.models.deepfm as D
    synth = make_synth("criteo_kaggle", seed=6)
    F, K, layers, keep, B, steps = synth.F, 8, [64, 32], [0.5, 0.5], 512, 3
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=8)
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    monkeypatch.setattr(D, "_RUN_SORT", run)
    outs = []
    for ovl in (False, True):
        monkeypatch.setattr(D, "_SH_OVERLAP", ovl)
        hub = _Hub(N)
        models = []
        for r in range(N):
            m = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, learning_rate=1e-3, batch_size=B,
                             device=DEV, init=False, comm=MeshComm(hub, r, sharded=sharded),
                             field_ranges=synth.field_ranges())
            m.load_tf_params(params)
            assert update == "lazy" or m.tf1_xsplit          # (tf1_dense: the split form's owner sweep)
            x = m.shx if sharded else m.rpx
            x.trace = []
            models.append(m)
        if run:
            _run_ranks_steps(models, batches)
        else:
            _run_ranks(models, batches, prefetch=2)
        torch.cuda.synchronize()
        for m in models:
            m.check_errors()
            assert m._last_plan.overlap_dense == ovl
            assert torch.equal(m.p, models[0].p)
            assert sharded or torch.equal(m.tv, models[0].tv)       # (replicas: bitwise equal)
        x = [(m.shx if sharded else m.rpx) for m in models]
        for t in x[1:]:
            assert t.trace == x[0].trace
        ar = [g for g in x[0].trace if g == ((KN.COMM_ALLREDUCE, models[0].P * 4),)]
        assert len(ar) == (steps if ovl else 0)
        m0 = models[0]
        if sharded:                       # the whole table, reassembled from the row shards
            full_v = torch.zeros(V, K, device=DEV)
            full_w = torch.zeros(V, device=DEV)
            for r, m in enumerate(models):
                rows = full_v[r::N].shape[0]
                full_v[r::N], full_w[r::N] = m.tv[:rows], m.tw[:rows]
        else:
            full_v, full_w = m0.tv, m0.tw
        outs.append((full_v, full_w, m0.p))
    for u, v in zip(*outs):
        assert (u - v).abs().max().item() <= 2e-6 * max(1e-3, u.abs().max().item())


@pytest.mark.parametrize("sharded", [True, False])
def test_dense_allreduce_equals_rank_order_gather(monkeypatch, sharded):
    """HIPFM_DENSE_XCHG: the fused exchange's dense gradient all-gathered and summed in rank order
    by the owner launch (the default) or all-reduced (opt-in).  The emulated all-reduce sums
    in rank order too, so the two are bitwise equal here (RCCL's ring order differs only by
    reassociation); every rank ends identical."""
    from hipfm.ops import kernels as KN
    import hipfm.parallel.sharded as SH
    synth = make_synth("criteo_kaggle", seed=8)
    F, K, layers, keep, B, N, steps = synth.F, 8, [64, 32], [0.5, 0.5], 512, 4, 3
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=12)
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    outs = []
    for how in ("allgather", "allreduce"):
        monkeypatch.setattr(SH, "_DENSE_XCHG", how)
        hub = _Hub(N)
        models = []
        for r in range(N):
            m = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", learning_rate=1e-3, batch_size=B,
                             device=DEV, init=False, comm=MeshComm(hub, r, sharded=sharded),
                             field_ranges=synth.field_ranges())
            m.load_tf_params(params)
            x = m.shx if sharded else m.rpx
            x.trace = []
            models.append(m)
        _run_ranks_steps(models, batches)
        torch.cuda.synchronize()
        for m in models:
            m.check_errors()
            assert torch.equal(m.p, models[0].p)
        x = models[0].shx if sharded else models[0].rpx
        kinds = {k for g in x.trace for k, _ in g}
        assert (KN.COMM_ALLREDUCE in kinds) == (how == "allreduce")
        outs.append([torch.cat([m.tv.reshape(-1) for m in models]), models[0].p.clone()])
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.parametrize("update,depth", [("lazy", 1), ("tf1_dense", 1), ("lazy", 2)])
def test_collective_sequence_identical_across_ranks(update, depth):
    """Deadlock freedom by construction (parallel/sharded.py): every collective of a step is a
    group on ONE engine, issued on the step's main stream (``_issue`` raises otherwise) in a fixed
    order.  Record each emulated rank's sequence of groups (kinds + byte counts) over N = 4 ranks
    and 3 prefetching steps: the sequences are identical on every rank, with the per-step shape
    G0 (first step: inline ids) / G1 (rows) / G2 (gradients + dense + next ids)."""
    from hipfm.ops import kernels as KN
    N, B = 4, 256
    synth = make_synth("total:40000", seed=5)
    F, K, layers, keep = synth.F, 8, [64, 32], [1.0, 1.0]
    params = init_params(synth.feature_size, F, K, layers, False, seed=3)
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(synth.feature_size, F, K, layers, keep, sparse_update=update, batch_size=B,
                         device=DEV, init=False, comm=MeshComm(hub, r, capacity=2048))
        m.load_tf_params(params)
        m.shx.trace = []
        models.append(m)
    batches = [[tuple(t.to(DEV) for t in synth.batch(B, step=100 * r + s, id_dtype=torch.int32))
                for s in range(3)] for r in range(N)]
    _run_ranks(models, batches, prefetch=depth)
    torch.cuda.synchronize()
    traces = [m.shx.trace for m in models]
    for t in traces[1:]:
        assert t == traces[0]
    t = traces[0]
    C, RWS, RWG = models[0].shx.C, models[0].shx.RWS, models[0].shx.RWG
    ids_op, rows_op = (KN.COMM_A2A, C * 4), (KN.COMM_A2A, C * RWS * 4)
    grads_op = (KN.COMM_A2A, C * RWG * 4)
    assert t[0] == (ids_op,) and t[1] == (rows_op,)            # step 0: inline ids, then rows
    g2 = t[2]
    assert g2[0] == grads_op and g2[-1] == ids_op               # gradients first, next ids last
    assert len(t) == 7 and t[5] == (rows_op,)
    if depth == 1:
        assert t[3] == (rows_op,) and t[4][-1] == ids_op        # next ids with the gradients
    else:
        # batch 2 was routed during step 0: its ids travel with step 1's rows, its rows are
        # served ahead during step 1 (step 2 then neither routes nor serves)
        assert t[3] == (rows_op, ids_op) and t[4][-1] != ids_op
        assert models[0].shx.sets[models[0].shx.cur].stage is None
    assert t[6][-1] != ids_op                                   # last step: no next batch
    for m in models:
        m.check_errors()


@pytest.mark.parametrize("N,opt,update,fused,run", [(4, "Adam", "lazy", True, False), (3, "Adagrad", "lazy", True, False),
                                                    (4, "Adam", "tf1_dense", True, False), (2, "Adam", "lazy", False, False),
                                                    (4, "Adam", "lazy", True, True), (3, "Adam", "tf1_dense", True, True)])
def test_replicated_exchange_matches_global_batch(N, opt, update, fused, run):
    """Config #3 (Horovod parity) as a captured step: N replicated tables, each rank's unique
    (id, gradient row) pairs all-gathered in fixed-capacity blocks and summed in rank order by
    every rank.  The replicas stay bitwise identical, the collective sequence is identical on
    every rank (one group per step), and the result equals ONE model on the global batch."""
    from hipfm.parallel.replicated import estimate_unique_capacity
    synth = make_synth("criteo_kaggle", seed=6)
    F, K, layers, keep, B = synth.F, 8, [64, 32], [1.0, 1.0], 512
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=9)
    lr, steps = 1e-3, 3
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    cap = max(estimate_unique_capacity(b[0] for b in batches[r]) for r in range(N))
    # eps / initial accumulator 1e-2: the first updates stay continuous in the gradient, so the
    # different fp32 summation order (rank blocks vs one segmented sum) cannot flip the sign of a
    # near-zero gradient (an lr-sized jump with eps = 1e-8); the exchange itself is what is checked
    okw = dict(adam_epsilon=1e-2, adagrad_init=1e-2)
    ref = NativeDeepFM(V, F, K, layers, keep, optimizer=opt, sparse_update=update, learning_rate=lr * N,
                       batch_size=N * B, device=DEV, init=False, field_ranges=synth.field_ranges(),
                       fused=fused, **okw)
    ref.load_tf_params(params)
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, layers, keep, optimizer=opt, sparse_update=update, learning_rate=lr,
                         batch_size=B, device=DEV, init=False, field_ranges=synth.field_ranges(),
                         comm=MeshComm(hub, r, capacity=cap, sharded=False), fused=fused, **okw)
        m.load_tf_params(params)
        assert m.rpx is not None and m.shx is None and m.R == V
        m.rpx.trace = []
        models.append(m)
    if run:      # one run per rank: run-level sort + routing of every batch at the run start (lazy)
        _run_ranks_steps(models, batches)
        assert len(models[0].rpx.run_sets) == steps
    else:
        _run_ranks(models, batches, prefetch=True)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
        # (run mode: one more group at the run start, the all-gather of every step's ids)
        assert m.rpx.trace == models[0].rpx.trace and len(m.rpx.trace) == steps + (1 if run else 0)
        for a, b in ((m.tv, models[0].tv), (m.tw, models[0].tw), (m.p, models[0].p)):
            assert torch.equal(a, b)                          # replicas bitwise identical
    m = models[0]
    scale = ref.tv.abs().max().item()
    assert (m.tv - ref.tv).abs().max().item() <= 2e-5 * scale
    assert (m.tw - ref.tw).abs().max().item() <= 2e-5 * max(1.0, ref.tw.abs().max().item())
    assert (m.p - ref.p).abs().max().item() <= 2e-5 * ref.p.abs().max().item()
    assert m.comm.bytes_sent > 0


def test_rank_streams_wait_for_model_setup():
    """Regression (round-4 driver failure of the n8 test): the emulated ranks must not start
    training before the work that built their models on the launching stream has finished.
    Here the models are built on a pool stream (pool streams never order among themselves) and
    the table fill is held back behind a ~0.25 s spin on it: with each rank stream waiting for
    the launching stream the shards reproduce the one-model run; without the wait they train on
    unfilled rows.  (In the n8 case the launching stream is the legacy default stream, whose
    implicit ordering did not hold in the long one-process suite: rank 7 -- the last model
    filled -- served all-zero rows in its first step, profiles/r5_n8_root_cause.md.)"""
    synth = make_synth("criteo_kaggle", seed=5)
    F, K, layers, keep, B, N = synth.F, 8, [64, 32], [1.0, 1.0], 512, 2
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=9, tables=False)
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(2)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    ref = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", learning_rate=1e-3 * N, batch_size=N * B,
                       device=DEV, init=False, field_ranges=synth.field_ranges(), adam_epsilon=1e-2)
    ref.load_tf_params(params)
    _fill_tables(ref, 1, 0)
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    torch.cuda.synchronize()

    def run(wait_origin):
        setup = torch.cuda.Stream()
        setup.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(setup):
            hub = _Hub(N)
            models = []
            for r in range(N):
                m = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", learning_rate=1e-3, batch_size=B,
                                 device=DEV, init=False, comm=MeshComm(hub, r), field_ranges=synth.field_ranges(),
                                 adam_epsilon=1e-2)
                m.load_tf_params(params)
                models.append(m)
            torch.cuda._sleep(500_000_000)        # the launching stream is busy for a while ...
            for r, m in enumerate(models):        # ... before it fills the tables
                _fill_tables(m, N, r)
            _run_ranks(models, batches, prefetch=True, wait_origin=wait_origin)
        torch.cuda.synchronize()
        full_v = torch.zeros_like(ref.tv)
        for r, m in enumerate(models):
            full_v[r::N] = m.tv[:full_v[r::N].shape[0]]
        return (full_v - ref.tv).abs().max().item(), ref.tv.abs().max().item()

    err, scale = run(True)
    assert err <= 2e-5 * scale, (err, scale)
    err_nowait, _ = run(False)                    # the hazard the wait removes
    assert err_nowait > 1e-3 * scale, err_nowait


def _table_rows(gid, K):
    """Deterministic initial (w, v) of the GLOBAL ids ``gid`` (int64 tensor)."""
    h = (gid * 2654435761) % 4294967296
    w = ((h % 10007).float() / 10007.0 - 0.5) * 0.02
    v = torch.stack([(((h >> (k + 3)) % 9973).float() / 9973.0 - 0.5) * 0.02 for k in range(K)], 1)
    return w, v


def _fill_tables(m, N, r):
    """Deterministic initial table values as a function of the GLOBAL id (row * N + r), so the
    row-sharded ranks and the replicated reference start from identical rows."""
    R, K = m.R, m.K
    step = 1 << 25
    with torch.no_grad():
        for a in range(0, R, step):
            b = min(R, a + step)
            gid = torch.arange(a, b, device=DEV, dtype=torch.int64) * N + r
            m.tw[a:b], m.tv[a:b] = _table_rows(gid, K)


N8_SHAPE = dict(K=8, layers=[128, 64, 32], keep=[1.0, 1.0, 1.0], B=16384, N=8, lr=5e-4, steps=2)


def n8_data(seed=2024):
    """The n8 test's global batches (N * B samples per step) and their per-rank slices."""
    c = N8_SHAPE
    synth = make_synth("criteo_1tb", seed=seed)
    N, B = c["N"], c["B"]
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(c["steps"])]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    return synth, data, batches


def n8_dense(synth):
    from hipfm.models.reference import init_params as ip
    c = N8_SHAPE
    return ip(synth.feature_size, synth.F, c["K"], c["layers"], False, seed=11, tables=False)


def n8_sharded(synth, data, batches, uids):
    """Train N = 8 emulated row-sharded ranks; return (v, w) of the global rows ``uids`` and the
    dense parameters (identical on every rank, checked)."""
    from hipfm.parallel.sharded import estimate_capacity
    c = N8_SHAPE
    F, K, N, B = synth.F, c["K"], c["N"], c["B"]
    V = synth.feature_size
    dense = n8_dense(synth)
    cap = max(estimate_capacity((batches[r][s][0] for s in range(c["steps"])), N) for r in range(N))
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, c["layers"], c["keep"], optimizer="Adam", sparse_update="lazy",
                         learning_rate=c["lr"], batch_size=B, device=DEV, init=False,
                         comm=MeshComm(hub, r, capacity=cap), field_ranges=synth.field_ranges(),
                         adam_epsilon=1e-2)
        m.load_tf_params(dense)
        _fill_tables(m, N, r)
        assert m.shx is not None and m.shx.N == N and m.shx.C == cap
        # the request table follows the exchange size, not the 110M-row shard
        assert sum(rs.req_key.numel() * 8 * (1 + N) for rs in m.shx.sets) < 256 * (1 << 20)
        models.append(m)
    _run_ranks(models, batches, prefetch=2)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
        assert torch.equal(m.p, models[0].p)
    got_v = torch.empty(uids.numel(), K, device=DEV)
    got_w = torch.empty(uids.numel(), device=DEV)
    for r, m in enumerate(models):
        sel = (uids % N) == r
        rows = uids[sel] // N
        got_v[sel] = m.tv[rows]
        got_w[sel] = m.tw[rows]
    p = models[0].p.clone()
    got_dense = {k: v.clone() for k, v in models[0].dense_tf_params().items()}
    del models, hub, m
    gc.collect()            # (the models sit in reference cycles: free their ~100 GB now)
    torch.cuda.empty_cache()
    return got_v, got_w, p, got_dense


def n8_single(synth, data, uids):
    """ONE model trained on the global batch (N * B samples, lr * N): (v, w) of ``uids``, dense."""
    c = N8_SHAPE
    N = c["N"]
    ref = NativeDeepFM(synth.feature_size, synth.F, c["K"], c["layers"], c["keep"], optimizer="Adam",
                       sparse_update="lazy", learning_rate=c["lr"] * N, batch_size=N * c["B"],
                       device=DEV, init=False, field_ranges=synth.field_ranges(), adam_epsilon=1e-2)
    ref.load_tf_params(n8_dense(synth))
    _fill_tables(ref, 1, 0)
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    torch.cuda.synchronize()
    ref.check_errors()
    out = (ref.tv[uids].clone(), ref.tw[uids].clone(), ref.p.clone(),
           {k: v.clone() for k, v in ref.dense_tf_params().items()})
    del ref
    gc.collect()
    torch.cuda.empty_cache()
    return out


def n8_golden(synth, data, uids):
    """The fp32 PyTorch golden model (models/reference.py, reference semantics) on the global
    batch, over a COMPACT table of the touched ids (lazy Adam moves only touched rows, and the
    whole-table L2 term's gradient on a touched row is l2 * row either way): (v, w) of ``uids``,
    their initial values, and the dense parameters.  The MLP's GEMM operands are rounded to bf16
    as the native tower rounds them."""
    from hipfm.models.reference import GoldenDeepFM
    c = N8_SHAPE
    K, N = c["K"], c["N"]
    w0, v0 = _table_rows(uids, K)
    params = dict(n8_dense(synth))
    params["fm_w"], params["fm_v"] = w0.clone(), v0.clone()
    gold = GoldenDeepFM(uids.numel(), synth.F, K, c["layers"], c["keep"], sparse_update="lazy",
                        learning_rate=c["lr"], world_size=N, device=DEV, params=params, adam_epsilon=1e-2,
                        mlp_bf16=True)
    for ids, vals, lab in data:
        gold.train_step(torch.searchsorted(uids, ids.long().reshape(-1)).reshape(ids.shape), vals, lab)
    return gold.params["fm_v"], gold.params["fm_w"], v0, w0, gold


def _golden_close(got, gold, init, what):
    """Row updates within bf16-MLP noise of the fp32 golden update: 99 % of the elements within 5 %
    of the largest golden update, none beyond 25 % (the smoke test's criterion)."""
    scale = (gold - init).abs().max().item()
    err = (got - gold).abs()
    frac = (err <= 0.05 * scale).float().mean().item()
    assert scale > 0 and frac >= 0.99 and err.max().item() <= 0.25 * scale, \
        f"{what}: {frac:.4f} within 5% of the golden update scale {scale:.3e}, max err {err.max().item():.3e}"


def test_sharded_exchange_n8_criteo_1tb_shape():
    """The bench's multi-GPU step at its real shape, emulated on one GPU: N = 8 row-sharded ranks
    (Adam eps 1e-2 keeps the first update continuous in the gradient, so fp32 summation order
    cannot flip a near-zero gradient's sign; the exchange itself is what is checked)
    (882.8M-row table, 110M rows per rank), B = 16384 per rank, the capacity estimate bench.py
    uses, prefetched routing.  The 8 shards must reproduce ONE model trained on the global batch
    (131072) to 2e-5 on every touched row and on the dense parameters."""
    free, _ = torch.cuda.mem_get_info()
    if free < 245 * (1 << 30):
        pytest.skip(f"needs ~240 GB of free HBM (have {free / (1 << 30):.0f} GB)")
    synth, data, batches = n8_data()
    uids = torch.unique(torch.cat([d[0].reshape(-1) for d in data]).long())
    got_v, got_w, p_sh, d_sh = n8_sharded(synth, data, batches, uids)
    ref_v, ref_w, ref_p, d_ref = n8_single(synth, data, uids)
    dv = (got_v - ref_v).abs()
    badu = uids[dv.max(1).values > 2e-7]
    bad_samples = sorted({(s, r) for s, d in enumerate(data)
                          for r in torch.isin(d[0].long(), badu).any(1).nonzero().reshape(-1).tolist()})
    info = (f"bad samples (step, row): {bad_samples[:20]} ({len(bad_samples)}) "
            f"max|dv|={dv.max().item():.3e} rows>tol={int((dv.max(1).values > 2e-7).sum())}/{uids.numel()} "
            f"dense={(p_sh - ref_p).abs().max().item():.3e}")
    assert dv.max().item() <= 2e-5 * ref_v.abs().max().item(), info
    assert (got_w - ref_w).abs().max().item() <= 2e-5 * ref_w.abs().max().item()
    assert (p_sh - ref_p).abs().max().item() <= 2e-5 * ref_p.abs().max().item()
    # both native sides against the fp32 golden model (a bug shared by the sharded step and the
    # one-model step at B = 131072 -- chunked field sort + merge -- is invisible to the above)
    gold_v, gold_w, v0, w0, gold = n8_golden(synth, data, uids)
    d0 = n8_dense(synth)
    for nm, v, w, d in (("sharded", got_v, got_w, d_sh), ("one model", ref_v, ref_w, d_ref)):
        _golden_close(v, gold_v, v0, f"{nm} fm_v")
        _golden_close(w, gold_w, w0, f"{nm} fm_w")
        # the dense parameters too (MLP weights / biases, FM bias, output layer)
        for k, t in d.items():
            _golden_close(t.float().cpu(), gold.params[k].float().cpu(), d0[k].float().cpu(), f"{nm} {k}")


@pytest.mark.parametrize("N,C_slack", [(1, 1.3), (3, 1.3), (8, 1.3), (8, 0.5)])
def test_two_launch_routing_matches_segments_bucket(N, C_slack):
    """sh_route (2 launches) gives exactly the outputs of segments + sh_bucket (7 launches):
    1-based unique index per slot, owner buckets in id order with -1 padding, unique positions,
    bucket counts, the unique count; an overflowing bucket (capacity below the need) flags err
    the same way."""
    from hipfm.ops import kernels as KN
    synth = make_synth("criteo_1tb", seed=3)
    B = 4096 + 77
    ids = synth.batch(B, step=1, device=DEV, id_dtype=torch.int32)[0].reshape(-1)
    n = ids.numel()
    sk = torch.sort(ids)[0].contiguous()
    U = int(torch.unique(sk).numel())
    C = int(U / N * C_slack) // 64 * 64 + 64
    i32 = dict(dtype=torch.int32, device=DEV)
    temp = torch.zeros(KN.radix_temp_bytes(n), dtype=torch.uint8, device=DEV)
    out = []
    for two in (True, False):
        sid, ukeys, seg, num = (torch.zeros(n, **i32), torch.zeros(n, **i32), torch.zeros(n + 1, **i32),
                                torch.zeros(1, **i32))
        send, upos, cnt, err = (torch.full((N * C,), 7, **i32), torch.full((n,), 7, **i32),
                                torch.zeros(N, **i32), torch.zeros(1, **i32))
        if two:
            tcnt = torch.zeros(KN.sh_route_tiles(n) * (N + 1), **i32)
            KN.sh_route(sk, n, N, C, tcnt, sid, send, upos, cnt, num, err)
        else:
            flags = torch.zeros(n, **i32)
            KN.segments(sk, n, flags, sid, ukeys, seg, num, temp)
            KN.sh_bucket(ukeys, num, n, N, C, torch.zeros(KN.sh_count_blocks(n) * N, **i32), send, upos,
                         cnt, err)
        torch.cuda.synchronize()
        out.append((sid, send, upos[:U], cnt, num, err))
    for name, a, b in zip(["sid_incl", "send_ids", "upos", "send_cnt", "num_u", "err"], out[0], out[1]):
        assert torch.equal(a, b), name
    assert int(out[0][4].item()) == U
    assert (int(out[0][5].item()) != 0) == (C_slack < 1.0)


@pytest.mark.parametrize("sharded", [True, False])
def test_bf16_tables_through_the_exchanges(sharded):
    """Mixed-precision embeddings (config #5) on the multi-GPU paths: bf16 rows are served /
    updated by the owner (row-sharded) or updated on every replica (replicated); N = 2 emulated
    ranks track one bf16 model on the global batch to bf16 precision (stochastic rounding of
    values whose fp32 pre-images differ in the last bits may pick the other neighbour: 1 ulp)."""
    from hipfm.parallel.dist import exchange_capacity
    N, B = 2, 512
    synth = make_synth("criteo_kaggle", seed=8)
    F, K, layers, keep = synth.F, 8, [64, 32], [1.0, 1.0]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=4)
    okw = dict(adam_epsilon=1e-2, sparse_update="lazy", emb_dtype="bf16", device=DEV, init=False,
               field_ranges=synth.field_ranges())
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(3)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    cap = max(exchange_capacity((b[0] for b in batches[r]), N, sharded) for r in range(N))
    ref = NativeDeepFM(V, F, K, layers, keep, learning_rate=1e-3 * N, batch_size=N * B, **okw)
    ref.load_tf_params(params)
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, layers, keep, learning_rate=1e-3, batch_size=B,
                         comm=MeshComm(hub, r, capacity=cap, sharded=sharded), **okw)
        m.load_tf_params(params)
        models.append(m)
    _run_ranks(models, batches, prefetch=True)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
    uids = torch.unique(torch.cat([d[0].reshape(-1) for d in data]).long())
    if sharded:
        got = torch.empty(uids.numel(), K, device=DEV)
        for r, m in enumerate(models):
            sel = (uids % N) == r
            got[sel] = m.tv[uids[sel] // N].float()
    else:
        assert torch.equal(models[0].rec, models[1].rec)
        got = models[0].tv[uids].float()
    want = ref.tv[uids].float()
    # a row's fp32 pre-image differs in the last bits (rank-ordered vs one segmented sum), so a
    # stochastic rounding can pick the other bf16 neighbour; hot rows (every step) random-walk a few
    # such ulps over the steps
    d = (got - want).abs()
    assert (d <= want.abs() * 2.0 ** -7 + 1e-8).float().mean().item() > 0.99
    assert (d <= want.abs() * 2.0 ** -5 + 1e-6).all()
    assert (models[0].p - ref.p).abs().max().item() <= 1e-3 * ref.p.abs().max().item()


def test_sharded_eval_and_predict_unequal_shards():
    """Evaluation / predict on a row-sharded table at N = 3 with shards of unequal length (ranks
    with 3, 1 and 0 batches, as file-level sharding of va files or Pipe-mode evaluation gives):
    ranks run in lockstep (Estimator.lockstep_batches) and a rank whose shard is done joins each
    remaining forward with a dummy batch (join_forward).  No hang; the summed AUC histogram equals
    that of one unsharded model over every batch, and rank 0's predictions -- the other ranks only
    serving rows -- equal the unsharded model's."""
    from hipfm.ops.metrics import auc_from_hist
    synth = make_synth("criteo_kaggle", seed=4)
    F, K, layers, keep, B, N = synth.F, 8, [64, 32], [0.5, 0.5], 256, 3
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=7)
    data = [synth.batch(B - 32 * s, step=100 + s, device=DEV, id_dtype=torch.int32) for s in range(4)]
    shards = [[data[0], data[1], data[3]], [data[2]], []]
    ref = NativeDeepFM(V, F, K, layers, keep, batch_size=B, device=DEV, init=False,
                       field_ranges=synth.field_ranges())
    ref.load_tf_params(params)
    h_ref = torch.zeros(2, 201, dtype=torch.int64, device=DEV)
    for ids, vals, lab in data:
        ref.eval_batch(ids, vals, lab, h_ref)
    p_ref = [ref.predict(ids, vals) for ids, vals, _ in shards[0]]
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, layers, keep, batch_size=B, device=DEV, init=False, comm=MeshComm(hub, r),
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        assert m.forward_collective
        models.append(m)
    hists = [torch.zeros(2, 201, dtype=torch.int64, device=DEV) for _ in range(N)]
    preds = []
    steps = max(len(s) for s in shards)

    def fn(r):
        m = models[r]
        for k in range(steps):                      # evaluate: every rank, lockstep
            if k < len(shards[r]):
                ids, vals, lab = shards[r][k]
                m.eval_batch(ids, vals, lab, hists[r])
            else:
                m.join_forward()
        for k in range(len(shards[0])):             # predict: rank 0's batches only
            if r == 0:
                ids, vals, _ = shards[0][k]
                preds.append(m.predict(ids, vals))
            else:
                m.join_forward()
    _rank_threads(models, fn)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
    h = sum(hists)
    assert torch.equal(h, h_ref), (auc_from_hist(h.cpu()), auc_from_hist(h_ref.cpu()))
    assert len(preds) == len(p_ref)
    for a, b in zip(preds, p_ref):
        assert torch.equal(a, b)
