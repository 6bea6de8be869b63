"""The tower's dX0 phase in a launch of its own (csrc/kernels/tower.hip tower_dx0_kernel,
HIPFM_DX0_SPLIT): dX0 from the stored dZ_0^T, the same MFMA chain in the same k order as the
fused tower's dX0 phase, so training is bit-identical with and without the split.  On run-sorted
steps the dX0 launch writes the slots' sorted gradient rows instead (the only sorted-row path at
K = 32; at K <= 16 the tower's own one is the oracle)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
import hipfm.models.deepfm as D  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("preset,K,B,update,multi", [("reference", 32, 1024, "lazy", True),
                                                     ("reference", 32, 1024, "tf1_dense", True),
                                                     ("reference", 8, 1024, "lazy", True),
                                                     ("criteo_kaggle", 16, 1024, "lazy", True),
                                                     ("criteo_kaggle", 8, 2048, "lazy", False),
                                                     ("criteo_kaggle", 16, 1000, "lazy", False)])
def test_dx0_split_trains_bitwise_like_the_fused_tower(monkeypatch, preset, K, B, update, multi):
    synth = make_synth(preset, seed=41)
    layers = [128, 64, 32]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=9)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(4)]
    out = []
    monkeypatch.setattr(D, "_L0_SPLIT", "0")      # (the layer-0 split reassociates: its own test)
    for split in ("1", "0"):
        monkeypatch.setattr(D, "_DX0_SPLIT", split)
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                         init=False, sparse_update=update, field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        if multi:
            for r in range(2):
                m.train_steps(pool[:2], next_ids=(pool[2][0], pool[3][0]))
                m.train_steps(pool[2:], next_ids=(pool[0][0], pool[1][0]))
        else:
            for s in range(8):
                ids, vals, lab = pool[s % 4]
                m.train_step(ids, vals, lab, use_graph=s % 2 == 0)
        torch.cuda.synchronize()
        m.check_errors()
        assert m.global_step() == 8
        if multi and split == "1":
            assert m.grow is not None and m._run_sort_ok(pool[:2])    # sorted rows from the dX0 launch
        out.append([m.tv.clone(), m.tw.clone(), m.p.clone()] + [s.clone() for s in m.sv if s.numel()] +
                   ([] if multi else [m.dX0.clone()]))
        del m
    for i, (x, y) in enumerate(zip(*out)):
        assert torch.equal(x, y), (i, (x.float() - y.float()).abs().max().item())
    assert multi or out[0][-1].abs().sum().item() > 0          # dX0 was written


@pytest.mark.parametrize("preset,K,B", [("reference", 32, 1024), ("criteo_kaggle", 8, 1024),
                                       ("criteo_kaggle", 16, 2000)])
def test_layer0_split_matches_the_fused_gather(monkeypatch, preset, K, B):
    """HIPFM_L0_SPLIT (tower.hip tower_l0s_kernel): the FM gather + layer 0 over ~8 field slices in
    a launch of their own, the tower summing the slices' fp32 partials in slice order.  The same
    function as the tower's own gather + layer-0 MFMA chain up to fp32 reassociation: one step's
    loss, predictions and gradients agree to rounding, and training stays close (Adam eps 1e-2
    keeps the update continuous in the gradient)."""
    synth = make_synth(preset, seed=43)
    layers = [128, 64, 32]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=10)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(4)]
    ev = synth.batch(700, step=99, device=DEV, id_dtype=torch.int32)
    res = []
    for l0 in ("auto", "0"):
        monkeypatch.setattr(D, "_L0_SPLIT", l0)
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                         init=False, sparse_update="lazy", field_ranges=synth.field_ranges(), adam_epsilon=1e-2)
        m.load_tf_params(params)
        assert (m.l0s > 1) == (l0 == "auto") and m.dx0_split
        g, _, UG = m.compute_grads(*pool[0])
        loss1 = m.loss_value(B)
        p1 = m.prob[:B].clone()
        for r in range(2):
            m.train_steps(pool[:2], next_ids=(pool[2][0], pool[3][0]))
            m.train_steps(pool[2:], next_ids=(pool[0][0], pool[1][0]))
        pred = m.predict(ev[0], ev[1])
        torch.cuda.synchronize()
        m.check_errors()
        res.append(dict(g=g.clone(), UG=UG.clone(), loss=loss1, p1=p1, tv=m.tv.clone(), tw=m.tw.clone(),
                        p=m.p.clone(), pred=pred.clone()))
        del m
    a, b = res
    assert abs(a["loss"] - b["loss"]) <= 1e-5
    assert (a["p1"] - b["p1"]).abs().max().item() <= 2e-5
    assert (a["g"] - b["g"]).abs().max().item() <= 1e-2 * b["g"].abs().max().item()
    assert (a["UG"] - b["UG"]).abs().max().item() <= 1e-2 * b["UG"].abs().max().item()
    for k in ("tv", "tw", "p"):
        d = (a[k] - b[k]).abs()
        scale = b[k].abs().max().item()
        assert (d <= 1e-3 * scale).float().mean().item() >= 0.999 and d.max().item() <= 2e-2 * scale, k
    assert (a["pred"] - b["pred"]).abs().max().item() <= 2e-3


@pytest.mark.parametrize("B", [4096, 1024])
def test_single_wide_hidden_layer_tower(monkeypatch, B):
    """One hidden layer of 256 (nl == 1): the tower's H region is then large enough that the dX0 /
    gradient-row wave tiles share the H_0 region, and with no dgrad chain only the barrier before
    the dX0 phase (tower.hip) keeps those tiles from overwriting H_0 while the head still reads it
    for the output-layer gradient.  Checked three ways: two runs are bitwise equal, the sorted
    gradient rows (HIPFM_GROW=1) train like the per-slot gather path (HIPFM_GROW=0), and one
    step's gradients match the per-layer kernels (B = 4096: the tower's own dX0 phase; 1024: the
    dX0 launch)."""
    synth = make_synth("criteo_kaggle", seed=47)
    K, layers = 8, [256]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=11)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(4)]
    res = {}
    for tag, grow, fused in (("a", "1", True), ("b", "1", True), ("nogrow", "0", True), ("layers", "1", False)):
        monkeypatch.setattr(D, "_GROW", grow)
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5], batch_size=B, device=DEV, init=False,
                         sparse_update="lazy", field_ranges=synth.field_ranges(), fused=fused)
        m.load_tf_params(params)
        assert m.fused == fused and (m.dx0_split == (B < 4096) or not fused)
        g, _, UG = m.compute_grads(*pool[0])
        out = dict(g=g.clone(), UG=UG.clone())
        if fused:
            assert (m.grow is not None) == (grow == "1") or not m._run_sort_ok(pool[:2])
            for r in range(2):
                m.train_steps(pool[:2], next_ids=(pool[2][0], pool[3][0]))
                m.train_steps(pool[2:], next_ids=(pool[0][0], pool[1][0]))
            torch.cuda.synchronize()
            m.check_errors()
            out.update(tv=m.tv.clone(), tw=m.tw.clone(), p=m.p.clone())
        res[tag] = out
        del m
    a, b, c, lay = res["a"], res["b"], res["nogrow"], res["layers"]
    for k in ("g", "UG", "tv", "tw", "p"):
        assert torch.equal(a[k], b[k]), k                        # deterministic (no LDS race)
    for k in ("tv", "tw", "p"):
        d = (a[k] - c[k]).abs().max().item()
        assert d <= 1e-5 * max(1.0, c[k].abs().max().item()), (k, d)
    scale = lay["g"].abs().max().item()
    assert (a["g"] - lay["g"]).abs().max().item() <= 1e-2 * scale + 1e-7
    assert (a["UG"] - lay["UG"]).abs().max().item() <= 1e-2 * lay["UG"].abs().max().item()
