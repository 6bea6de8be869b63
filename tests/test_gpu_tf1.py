"""tf1_dense (TF1 non-lazy optimizer semantics) on one GPU: the split form -- batch rows updated in
the sparse kernel, every other row by a sweep on a concurrent graph branch (optim.hip
tf1_sweep_kernel) -- must equal the scatter + full-table sweep form bitwise, through eager steps,
captured multi-step graphs with prefetched sorts, discarded prefetches and the global sort."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
import hipfm.models.deepfm as dm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402

DEV = torch.device("cuda", 0)


def _pair(opt, K, V, ranges, B, l2=1e-3):
    kw = dict(optimizer=opt, sparse_update="tf1_dense", batch_size=B, device=DEV, seed=7,
              field_ranges=ranges, l2_reg=l2, adam_epsilon=1e-2)
    old = dm._TF1_SPLIT
    try:
        dm._TF1_SPLIT = True
        a = NativeDeepFM(V, len(ranges), K, [64, 32], [0.5, 0.5], **kw)
        dm._TF1_SPLIT = False
        b = NativeDeepFM(V, len(ranges), K, [64, 32], [0.5, 0.5], **kw)
    finally:
        dm._TF1_SPLIT = old
    assert a.tf1_split and not b.tf1_split
    return a, b


def _assert_same(a, b):
    torch.cuda.synchronize()
    assert torch.equal(a.tv, b.tv), (a.tv - b.tv).abs().max()
    assert torch.equal(a.tw, b.tw), (a.tw - b.tw).abs().max()
    for sa, sb in zip(a.sv, b.sv):
        assert torch.equal(sa, sb), (sa - sb).abs().max()
    assert torch.equal(a.p, b.p), (a.p - b.p).abs().max()
    assert int(a.step.item()) == int(b.step.item()) == int(a.sw_step.item())
    a.check_errors()


@pytest.mark.parametrize("opt,K,mode", [("Adam", 8, "merged"), ("Adam", 8, "branch"),
                                        ("Adagrad", 16, "merged"), ("Momentum", 4, "branch"),
                                        ("ftrl", 8, "merged"), ("GD", 8, "auto"),
                                        ("Adam", 32, "auto")])
def test_tf1_split_equals_scatter_sweep(opt, K, mode, monkeypatch):
    """merged: the sweep runs as extra workgroups of the sparse + wgfin launch; branch: as its own
    kernel on a graph branch concurrent with the whole step."""
    monkeypatch.setattr(dm, "_SWEEP_MODE", mode)
    synth = make_synth("criteo_kaggle")
    B = 2048
    a, b = _pair(opt, K, synth.feature_size, synth.field_ranges(), B)
    pool = [synth.batch(B, i, device=DEV, id_dtype=torch.int32) for i in range(6)]
    # eager steps, the first two with the next batch declared (prefetched sort + flags)
    for i in range(3):
        nxt = pool[i + 1][0] if i < 2 else None
        a.train_step(*pool[i], next_ids=nxt)
        b.train_step(*pool[i], next_ids=nxt)
    _assert_same(a, b)
    # a declared next batch that is NOT the one trained next: its flags must be cleared
    a.train_step(*pool[3], next_ids=pool[5][0])
    b.train_step(*pool[3], next_ids=pool[5][0])
    a.train_step(*pool[4])
    b.train_step(*pool[4])
    _assert_same(a, b)
    # captured multi-step graphs over a resident pool, replayed twice (prefetch chain)
    for _ in range(2):
        a.train_steps(pool, next_ids=pool[0][0])
        b.train_steps(pool, next_ids=pool[0][0])
    _assert_same(a, b)
    # single-step graph replays
    for i in range(4):
        a.train_step(*pool[i], use_graph=True, next_ids=pool[i + 1][0])
        b.train_step(*pool[i], use_graph=True, next_ids=pool[i + 1][0])
    _assert_same(a, b)
    # (auto: B = 2048 takes the branch for K <= 16, the merged sweep for K = 32)
    assert a._tf1_merged == (mode == "merged" or (mode == "auto" and K > 16))
    # every row moved (non-lazy semantics): rows never in a batch changed too
    seen = torch.zeros(a.R, dtype=torch.bool, device=DEV)
    for ids, _, _ in pool:
        seen[ids.reshape(-1).long()] = True
    if opt != "GD" or a.l2 > 0:
        a0, _ = _pair(opt, K, synth.feature_size, synth.field_ranges(), B)
        moved = (a0.tv != a.tv).any(dim=1)
        assert bool(moved[~seen].all())


def test_tf1_split_global_sort_and_restore():
    """No field ranges (global radix sort, inline each step) and a checkpoint round trip: the
    sweep's own step counter follows the restored global step."""
    synth = make_synth("total:4000", seed=3)
    B = 256
    old = dm._TF1_SPLIT
    try:
        kw = dict(optimizer="Adam", sparse_update="tf1_dense", batch_size=B, device=DEV, seed=3,
                  l2_reg=1e-3)
        dm._TF1_SPLIT = True
        a = NativeDeepFM(synth.feature_size, synth.F, 8, [32], [0.5], **kw)
        dm._TF1_SPLIT = False
        b = NativeDeepFM(synth.feature_size, synth.F, 8, [32], [0.5], **kw)
    finally:
        dm._TF1_SPLIT = old
    assert a.tf1_split and not b.tf1_split
    for i in range(3):
        ids, vals, lab = synth.batch(B, i, device=DEV, id_dtype=torch.int32)
        a.train_step(ids, vals, lab)
        b.train_step(ids, vals, lab)
    _assert_same(a, b)
    st = {k: v.clone() for k, v in a.state_dict_local().items()}
    for i in range(3, 5):
        ids, vals, lab = synth.batch(B, i, device=DEV, id_dtype=torch.int32)
        a.train_step(ids, vals, lab, use_graph=True)
    a.load_state_dict_local(st)
    assert int(a.sw_step.item()) == 3
    for i in range(3, 6):
        ids, vals, lab = synth.batch(B, i, device=DEV, id_dtype=torch.int32)
        a.train_step(ids, vals, lab, use_graph=True)
        b.train_step(ids, vals, lab)
    _assert_same(a, b)


def test_tf1_sweep_kernel_matches_torch():
    """The sweep alone against a plain fp32 PyTorch Adam step with g = l2 * w on unflagged rows."""
    R, K = 5000, 8
    rec = torch.zeros(R, 32, device=DEV)
    torch.manual_seed(0)
    rec[:, :K + 1] = torch.randn(R, K + 1, device=DEV)
    rec[:, K + 1] = torch.rand(R, device=DEV)            # w slot0 (m)
    rec[:, K + 2] = torch.rand(R, device=DEV) + 0.1      # w slot1 (v)
    rec[:, K + 4:2 * K + 4] = torch.randn(R, K, device=DEV) * 0.1
    rec[:, 2 * K + 4:3 * K + 4] = torch.rand(R, K, device=DEV) + 0.1
    flags = (torch.rand(R, device=DEV) < 0.3).to(torch.uint8)
    skip = flags.bool().clone()
    step = torch.tensor([4], dtype=torch.int64, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    lr, l2, b1, b2, eps = 1e-2, 1e-3, 0.9, 0.999, 1e-8
    h = KN.hyper(lr, l2, eps=eps)
    ref = rec.clone()
    KN.tf1_sweep(K, KN.OPT_IDS["Adam"], rec, flags, h, step, done, max_wg=7)
    torch.cuda.synchronize()
    t = 5
    lr_t = lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)

    def adam(p, m, v):
        g = l2 * p
        m2 = b1 * m + (1 - b1) * g
        v2 = b2 * v + (1 - b2) * g * g
        return p - lr_t * m2 / (v2.sqrt() + eps), m2, v2
    p, m, v = adam(ref[:, :K], ref[:, K + 4:2 * K + 4], ref[:, 2 * K + 4:3 * K + 4])
    pw, mw, vw = adam(ref[:, K], ref[:, K + 1], ref[:, K + 2])
    exp = ref.clone()
    exp[:, :K], exp[:, K + 4:2 * K + 4], exp[:, 2 * K + 4:3 * K + 4] = p, m, v
    exp[:, K], exp[:, K + 1], exp[:, K + 2] = pw, mw, vw
    exp[skip] = ref[skip]
    assert torch.allclose(rec, exp, rtol=1e-5, atol=1e-7), (rec - exp).abs().max()
    assert int(flags.sum().item()) == 0                 # flagged rows skipped and cleared
    assert int(step.item()) == 5 and int(done.item()) == 0
