"""Mixed-precision embeddings (BASELINE config #5): fm_v rows and their
optimizer slots stored bf16 with counter-based stochastic rounding, fm_w and all arithmetic fp32.
Checked against the fp32 model from the same initial values: the training trajectories agree to
bf16 precision, rounding is reproducible (bitwise run to run), and the row-sharded and
replicated exchanges carry bf16 tables too (N = 2 emulation vs the single-GPU bf16 model)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM, table_record_floats  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

DEV = torch.device("cuda", 0)


def test_record_sizes():
    assert table_record_floats(8, "Adam", bf16=True) * 4 == 64        # half the fp32 record
    assert table_record_floats(8, "Adam") * 4 == 128
    assert table_record_floats(32, "Adam", bf16=True) * 4 == 256      # Criteo-1TB K=32: 226 GB


@pytest.mark.parametrize("opt", ["Adam", "Adagrad"])
def test_bf16_rows_track_fp32_training(opt):
    synth = make_synth("criteo_kaggle", seed=11)
    F, K, layers, keep, B = synth.F, 8, [64, 32], [1.0, 1.0], 2048
    params = init_params(synth.feature_size, F, K, layers, False, seed=5)
    # eps / initial accumulator 1e-2: updates stay continuous in the gradient (with 1e-8 the first
    # steps are ~lr * sign(g), and bf16-level noise flips near-zero gradients by a full 2 lr)
    kw = dict(optimizer=opt, sparse_update="lazy", batch_size=B, device=DEV, init=False,
              field_ranges=synth.field_ranges(), learning_rate=1e-3, adam_epsilon=1e-2, adagrad_init=1e-2)
    a = NativeDeepFM(synth.feature_size, F, K, layers, keep, **kw)
    b = NativeDeepFM(synth.feature_size, F, K, layers, keep, emb_dtype="bf16", **kw)
    c = NativeDeepFM(synth.feature_size, F, K, layers, keep, emb_dtype="bf16", **kw)
    for m in (a, b, c):
        m.load_tf_params(params)
    assert b.tv.dtype == torch.bfloat16 and b.rec.shape[1] * 4 == 64
    batches = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(12)]
    la, lb = [], []
    for i, bt in enumerate(batches):
        nxt = batches[i + 1][0] if i + 1 < len(batches) else None
        a.train_step(*bt, next_ids=nxt)
        b.train_step(*bt, next_ids=nxt)
        c.train_step(*bt, use_graph=True, next_ids=nxt)
        la.append(a.loss_value(B))
        lb.append(b.loss_value(B))
    torch.cuda.synchronize()
    b.check_errors()
    # reproducible rounding: eager and graph-replayed runs are bitwise equal
    assert torch.equal(b.rec, c.rec) and torch.equal(b.p, c.p)
    for x, y in zip(la, lb):
        assert abs(x - y) < 2e-3 * max(1.0, abs(x)), (la, lb)
    ids = torch.unique(torch.cat([bt[0].reshape(-1) for bt in batches]).long())
    va, vb = a.tv[ids].float(), b.tv[ids].float()
    upd = (va - torch.as_tensor(params["fm_v"], device=DEV)[ids]).abs().max().item()
    # bf16 storage: ~|v| * 2^-8 per rounding (stochastic, so a random walk over the steps)
    err = (va - vb).abs()
    assert err.max().item() < 0.25 * upd + 3e-4 and err.mean().item() < 0.05 * upd + 3e-5
    # export view is fp32
    tfv = b.tf_variables()
    assert tfv["fm_v"].dtype == torch.float32 and tfv[f"fm_v/{b.SLOT_NAMES[opt][0]}"].dtype == torch.float32
