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
