"""Row-sharded fixed-capacity exchange (parallel/sharded.py + csrc/kernels/shard.hip) with N > 1
ranks on ONE GPU: N model instances run in N threads, each on its own HIP stream, and the
all-to-all / all-reduce of the native RCCL engine are replaced by stream-ordered copies between
the instances (MeshEngine).  Every HIP kernel of the multi-GPU step runs exactly as on N GPUs
(bucketing by owner = id % N, serving, owner-side rank-ordered sums, row updates); only the
transport differs.  The sharded run must reproduce one model trained on the global batch."""
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


class MeshComm:
    def __init__(self, hub, rank, capacity=None):
        self.world_size, self.rank = hub.N, rank
        self.sharded = True
        self.force_exchange = False
        self.engine = MeshEngine(hub, rank)
        self.engine_dense = MeshEngine(hub, rank)
        self.engine_route = MeshEngine(hub, rank)
        self.capacity = capacity
        self.graph_safe = False

    @property
    def bytes_sent(self):
        return self.engine.bytes_sent


def _run_ranks(models, batches, prefetch=False):
    errs = []

    def body(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                bl = batches[r]
                for i, (ids, vals, lab) in enumerate(bl):
                    nxt = bl[i + 1][0] if (prefetch and i + 1 < len(bl)) else None
                    models[r].train_step(ids, vals, lab, next_ids=nxt)
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


@pytest.mark.parametrize("N,opt,update,prefetch", [(2, "Adam", "lazy", False), (3, "Adagrad", "lazy", True),
                                                   (4, "Adam", "tf1_dense", False), (4, "Adam", "lazy", True)])
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
