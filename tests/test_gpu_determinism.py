"""Run-to-run determinism at full scale (B = 16384, 512 tower workgroups, two per CU), where a
VALU -> ds_bpermute hazard of packed-FP32 ops once made the gather-fused tower's FM logits wrong
for a random pair of samples per launch (ops/build.py NO_PACKED_F32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402

DEV = torch.device("cuda", 0)
B = 16384


def _model(synth, update="lazy"):
    return NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, seed=1234,
                        batch_size=B, device=DEV, field_ranges=synth.field_ranges(),
                        sparse_update=update)


def test_gather_tower_eval_is_exact_and_deterministic():
    synth = make_synth("criteo_kaggle", seed=2024)
    m = _model(synth)
    assert m.gather_fused
    ids, vals, _ = synth.batch(B, step=500_000, device=DEV, id_dtype=torch.int32)
    m.stage_batch(ids, vals, None)
    a = m._tower_args(B, train=False, with_labels=False, gather=m._fm_inputs(B, train=False))
    ys, ps = [], []
    for _ in range(10):
        m.y_fm.zero_()
        KN.tower(a, KE=m.K)
        torch.cuda.synchronize()
        ys.append(m.y_fm[:B].clone())
        ps.append(m.prob[:B].clone())
    for y, p in zip(ys[1:], ps[1:]):
        assert torch.equal(y, ys[0]) and torch.equal(p, ps[0])
    # the FM logit against float64 on the host (fm_bias + sum w x + pairwise interactions)
    idl = ids.long()
    v = m.tv[idl].double() * vals.double().unsqueeze(-1)
    w = m.tw[idl].double() * vals.double()
    fb = float(m.p[m.dense_segs["fm_bias"].off])
    ex = fb + w.sum(1) + 0.5 * (v.sum(1) ** 2 - (v * v).sum(1)).sum(1)
    assert float((ys[0].double() - ex).abs().max()) < 1e-6


@pytest.mark.parametrize("update", ["lazy", "tf1_dense"])
def test_training_is_bitwise_reproducible(update):
    synth = make_synth("criteo_kaggle", seed=2024)
    batches = [synth.batch(B, step=7_000 + i, device=DEV, id_dtype=torch.int32) for i in range(4)]
    ms = [_model(synth, update) for _ in range(2)]
    for mm in ms:
        for i, b in enumerate(batches[:2]):
            mm.train_step(*b, next_ids=batches[i + 1][0])
        mm.train_steps(batches[2:])              # captured multi-step graph
        if update == "tf1_dense":
            assert mm._tf1_merged                 # B = 16384: the merged sweep
    torch.cuda.synchronize()
    assert torch.equal(ms[0].rec, ms[1].rec)
    assert torch.equal(ms[0].p, ms[1].p)
