"""Native batch norm (csrc/kernels/bn.hip) vs the fp32 golden model (reference batch_norm_layer,
PS:288-292: after ReLU, before dropout, eps 1e-3, moving averages with decay)."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import GoldenDeepFM, init_params  # noqa: E402

DEV = "cuda"


def _mostly_close(a, b, atol, frac=0.98, hard=None):
    d = (a - b).abs()
    ok = (d <= atol).float().mean().item()
    assert ok >= frac, f"only {ok:.4f} of elements within {atol} (max {d.max().item():.3e})"
    if hard is not None:
        assert d.max().item() <= hard, d.max().item()


def _perturbed_params(V, F, K, layers, seed):
    """BN params away from the (1, 0) init so gamma/beta actually matter."""
    p = init_params(V, F, K, layers, True, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    for i, L in enumerate(layers):
        p[f"Deep-part/bn_{i}/gamma"] = 1.0 + 0.3 * torch.rand(L, generator=g)
        p[f"Deep-part/bn_{i}/beta"] = 0.1 * torch.randn(L, generator=g)
    return p


@pytest.mark.parametrize("B", [512, 500])     # 500: padded rows must not enter the statistics
def test_bn_gradients_match_golden(B):
    synth = make_synth("total:4000", seed=20)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.5, 0.75]
    V = synth.feature_size
    params = _perturbed_params(V, F, K, layers, 7)
    nat = NativeDeepFM(V, F, K, layers, keep, batch_size=B, device=DEV, init=False, batch_norm=True)
    nat.load_tf_params(params)
    gold = GoldenDeepFM(V, F, K, layers, keep, params=params, batch_norm=True)
    # the same model with bf16-rounded GEMM operands: BN divides by small batch stds, which
    # amplifies bf16 rounding (measured: up to ~9% of max|grad| vs fp32 on small-var columns),
    # so the tight check is against bf16-emulating autograd and the fp32 check is looser
    gold16 = GoldenDeepFM(V, F, K, layers, keep, params=params, batch_norm=True, mlp_bf16=True)
    ids, vals, labels = synth.batch(B, step=0)
    _, data, gg = gold.compute_grads(ids, vals, labels)
    _, _, gg16 = gold16.compute_grads(ids, vals, labels)
    g, uk, UG = nat.compute_grads(ids.to(DEV, torch.int32), vals.to(DEV), labels.to(DEV))
    torch.cuda.synchronize()
    assert abs(nat.loss_value(B) - float(data)) < 2e-3
    dense = nat.dense_tf_params(g)
    for k, v in dense.items():
        for ref, tol in ((gg16[k], 0.03), (gg[k], 0.15)):
            scale = ref.abs().max().item() + 1e-12
            err = (v - ref).abs().max().item()
            assert err <= tol * scale + 1e-6, (k, tol, err, scale)
    uk = uk.long().cpu()
    for ref, tol in ((gg16, 0.03), (gg, 0.1)):
        gv = ref["fm_v"][uk] - 1e-4 * params["fm_v"][uk]
        sv = gv.abs().max().item()
        assert (UG.cpu()[:, :K] - gv).abs().max().item() <= tol * sv, tol
    # moving statistics after one update (golden updated them inside compute_grads)
    tv = nat.tf_variables()
    for i in range(len(layers)):
        for n in ("moving_mean", "moving_variance"):
            k = f"Deep-part/bn_{i}/{n}"
            assert torch.allclose(tv[k], gold.params[k], atol=2e-2, rtol=2e-2), k


def test_bn_train_eval_match_golden():
    synth = make_synth("total:4000", seed=21)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.5, 0.75]
    V = synth.feature_size
    lr = 1e-3
    params = _perturbed_params(V, F, K, layers, 8)
    kw = dict(adam_epsilon=1e-2, batch_norm=True, batch_norm_decay=0.9)
    nat = NativeDeepFM(V, F, K, layers, keep, sparse_update="lazy", batch_size=256, device=DEV,
                       init=False, learning_rate=lr, **kw)
    nat.load_tf_params(params)
    gold = GoldenDeepFM(V, F, K, layers, keep, sparse_update="lazy", params=params, learning_rate=lr,
                        mlp_bf16=True, **kw)
    steps = 3
    for s in range(steps):
        ids, vals, labels = synth.batch(256, step=s)
        gold.train_step(ids, vals, labels)
        nat.train_step(ids.to(DEV, torch.int32), vals.to(DEV), labels.to(DEV))
    torch.cuda.synchronize()
    hard = 2.2 * lr * steps
    tw, tv = nat.sparse_tables_tf()
    _mostly_close(tv.cpu(), gold.params["fm_v"], 2e-4, hard=hard)
    for k, v in nat.dense_tf_params().items():
        _mostly_close(v, gold.params[k], 5e-4, frac=0.98, hard=hard + 1e-3)
    tfv = nat.tf_variables()
    for i in range(len(layers)):
        for n in ("moving_mean", "moving_variance"):
            k = f"Deep-part/bn_{i}/{n}"
            assert torch.allclose(tfv[k], gold.params[k], atol=3e-2, rtol=3e-2), k
    # eval forward uses the moving statistics (train_phase False branch, PS:291)
    ids, vals, labels = synth.batch(300, step=99)
    p_nat = nat.predict(ids.to(DEV, torch.int32), vals.to(DEV)).cpu()
    p_gold = gold.predict(ids, vals)
    assert torch.allclose(p_nat, p_gold, atol=1.5e-2)


def test_bn_graph_replay_and_tf_roundtrip():
    synth = make_synth("total:4000", seed=22)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.5, 0.5]
    V = synth.feature_size
    params = _perturbed_params(V, F, K, layers, 9)
    a = NativeDeepFM(V, F, K, layers, keep, batch_size=256, device=DEV, init=False, batch_norm=True)
    b = NativeDeepFM(V, F, K, layers, keep, batch_size=256, device=DEV, init=False, batch_norm=True)
    a.load_tf_params(params)
    b.load_tf_params(params)
    for s in range(4):
        ids, vals, labels = synth.batch(256, step=s, device=DEV, id_dtype=torch.int32)
        a.train_step(ids, vals, labels, use_graph=False)
        b.train_step(ids, vals, labels, use_graph=True)
    torch.cuda.synchronize()
    assert torch.equal(a.p, b.p) and torch.equal(a.bn_moving, b.bn_moving)
    c = NativeDeepFM(V, F, K, layers, keep, batch_size=256, device=DEV, init=False, batch_norm=True)
    c.load_tf_variables(a.tf_variables())
    assert torch.equal(c.p, a.p) and torch.equal(c.bn_moving, a.bn_moving)
    assert c.global_step() == 4
