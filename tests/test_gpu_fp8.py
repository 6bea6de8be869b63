"""fp8 deep tower (mlp_dtype=fp8, BASELINE config #5): OCP e4m3 forward GEMMs on
v_mfma_f32_16x16x32_fp8_fp8 with per-row / per-channel power-of-two scales, checked against
PyTorch's float8_e4m3fn conversion and the fp32 golden model."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import GoldenDeepFM, init_params  # noqa: E402

DEV = torch.device("cuda", 0)


def _pow2_scale(amax: torch.Tensor) -> torch.Tensor:
    _, e = torch.frexp(448.0 / amax)
    return torch.ldexp(torch.ones_like(amax), e - 1)


def test_w8_quant_matches_torch_e4m3():
    """Weight shadows: bytes equal torch's RNE float8_e4m3fn cast of W * q (OCP, not fnuz)."""
    synth = make_synth("total:3000", seed=1)
    layers = [128, 64]
    m = NativeDeepFM(synth.feature_size, synth.F, 8, layers, [1.0, 1.0], batch_size=256, device=DEV,
                     mlp_dtype="fp8", seed=3)
    g = torch.Generator(device=DEV).manual_seed(0)
    with torch.no_grad():
        m.p.copy_(torch.randn(m.P, generator=g, device=DEV) * 0.3)
    m.refresh_shadows()
    torch.cuda.synchronize()
    for i in range(len(layers)):
        s = m.dense_segs[f"Deep-part/mlp{i}/weights"]
        W = m.p[s.off: s.off + m.Np[i] * m.Kp[i]].view(m.Np[i], m.Kp[i])
        q = _pow2_scale(W.abs().amax(dim=1))
        ref = (W * q[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(m.W8[i], ref), i
        assert torch.equal(m.sW[i], 1.0 / q), i


def _pair(fp8_seed=5, layers=(128, 64, 32), keep=(1.0, 1.0, 1.0), B=1024):
    synth = make_synth("criteo_kaggle", seed=fp8_seed)
    F, K = synth.F, 8
    params = init_params(synth.feature_size, F, K, list(layers), False, seed=fp8_seed)
    mk = lambda dt: NativeDeepFM(synth.feature_size, F, K, list(layers), list(keep), batch_size=B,
                                 device=DEV, init=False, mlp_dtype=dt, sparse_update="lazy",
                                 learning_rate=1e-3)
    a, b = mk("fp8"), mk("bf16")
    a.load_tf_params(params)
    b.load_tf_params(params)
    return synth, params, a, b


def test_fp8_forward_close_to_fp32_golden():
    synth, params, a, b = _pair()
    gold = GoldenDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [1.0] * 3, params=params)
    # trained-scale embeddings: the glorot init of a 1M-row table is ~1e-3, so scale the
    # tables up to exercise the per-row scaling over a realistic range
    with torch.no_grad():
        for m in (a, b):
            m.tv.mul_(300.0)
        gold.params["fm_v"].mul_(300.0)
    ids, vals, _ = synth.batch(1024, step=1)
    pg = gold.predict(ids, vals).float()
    pa = a.predict(ids.to(DEV, torch.int32), vals.to(DEV)).cpu()
    pb = b.predict(ids.to(DEV, torch.int32), vals.to(DEV)).cpu()
    da, db = (pa - pg).abs(), (pb - pg).abs()
    assert not torch.equal(pa, pb)                       # the fp8 path really ran
    assert da.mean().item() < 4e-3 and da.max().item() < 3e-2, (da.mean().item(), da.max().item())
    assert db.mean().item() < 2e-3


def test_fp8_training_tracks_bf16():
    synth, params, a, b = _pair(keep=(0.5, 0.5, 0.5))
    la, lb = [], []
    for s in range(40):
        ids, vals, lab = synth.batch(1024, step=s, device=DEV, id_dtype=torch.int32)
        a.train_step(ids, vals, lab, use_graph=True)
        b.train_step(ids, vals, lab, use_graph=True)
        if s % 10 == 9:
            la.append(a.loss_value(1024))
            lb.append(b.loss_value(1024))
    torch.cuda.synchronize()
    assert la[-1] < la[0] and lb[-1] < lb[0]
    assert abs(la[-1] - lb[-1]) <= 0.03 * lb[-1], (la, lb)
    assert torch.isfinite(a.p).all() and torch.isfinite(a.tv).all()
