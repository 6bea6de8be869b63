"""Input safety on the native path (ids must satisfy id < V): a bad id in a batch
handed straight to the model (no loader check) never reads or writes out of bounds -- the global
slot sort and the tower's gather clamp it -- and the run raises a clear error instead of training
on: asynchronously after the next enqueue (poll_errors) and at the next host sync."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("bad", ["above", "negative"])
def test_out_of_vocabulary_id_flags_without_faulting(bad):
    synth = make_synth("total:20000", seed=3)
    B, F = 512, synth.F
    m = NativeDeepFM(synth.feature_size, F, 8, [32], [1.0], batch_size=B, device=DEV,
                     sparse_update="lazy")                   # no field ranges: global slot sort
    ids, vals, labels = (t.to(DEV) for t in synth.batch(B, step=0, id_dtype=torch.int32))
    m.train_step(ids, vals, labels)
    m.check_errors()                                          # a clean batch: no error
    before = m.rec.clone()
    ids2 = ids.clone()
    ids2[5, 7] = synth.feature_size + 11 if bad == "above" else -3
    m.train_step(ids2, vals, labels)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="outside \\[0, feature_size"):
        m.check_errors()
    assert torch.isfinite(m.rec).all() and m.rec.shape == before.shape
    # the asynchronous poll reports it too (first call starts the copy, a later one raises)
    m2 = NativeDeepFM(synth.feature_size, F, 8, [32], [1.0], batch_size=B, device=DEV,
                      sparse_update="lazy")
    m2.train_step(ids2, vals, labels)
    m2.poll_errors()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="feature_size"):
        m2.poll_errors()
