"""End-to-end on the native GPU path (HIP kernels): CLI train/eval/infer/export/resume, native
checkpoint round trip, TF-layout export parity with the golden model."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.cli import main  # noqa: E402
from hipfm.ckpt import tf_bundle as tb  # noqa: E402
from hipfm.ckpt.export import latest_export, load_servable  # noqa: E402
from hipfm.config import parse_flags  # noqa: E402
from hipfm.estimator import Estimator  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = tmp_path_factory.mktemp("gsyn")
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:50000", "--train_rows", "20000",
                           "--val_rows", "4000", "--test_rows", "500", "--files", "4"], cwd=REPO)
    return str(d)


def _flags(dataset, md, extra=()):
    return ["--training_data_dir", dataset, "--val_data_dir", dataset, "--model_dir", md,
            "--feature_size", "50000", "--field_size", "39", "--embedding_size", "8",
            "--batch_size", "512", "--deep_layers", "64,32", "--dropout", "0.9,0.9",
            "--learning_rate", "0.003", "--log_steps", "10", "--device", "cuda"] + list(extra)


def test_native_cli_train_eval_infer_export_resume(dataset, tmp_path):
    md, sd = str(tmp_path / "m"), str(tmp_path / "s")
    res = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "3",
                                    "--servable_model_dir", sd]))
    steps = 3 * (20000 // 512)
    assert res["global_step"] == steps and res["auc"] > 0.70, res
    ev = main(_flags(dataset, md, ["--task_type", "eval"]))
    assert ev["global_step"] == steps and abs(ev["auc"] - res["auc"]) < 1e-6
    inf = main(_flags(dataset, md, ["--task_type", "infer", "--pred_path", str(tmp_path / "p.txt")]))
    assert inf["rows"] == 500
    s = load_servable(latest_export(sd), device="cuda")
    s_cpu = load_servable(latest_export(sd))
    ids = torch.arange(39).repeat(8, 1)
    assert torch.allclose(s.predict(ids, torch.ones(8, 39)), s_cpu.predict(ids, torch.ones(8, 39)),
                          atol=1e-2)
    res2 = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "1"]))
    assert res2["global_step"] == steps + 20000 // 512


def test_native_tf_variables_roundtrip(tmp_path):
    cfg = parse_flags(["--feature_size", "3000", "--field_size", "39", "--embedding_size", "8",
                       "--deep_layers", "64,32", "--dropout", "1,1", "--batch_size", "256",
                       "--device", "cuda"])
    est = Estimator(cfg)
    ids = torch.randint(0, 3000, (256, 39))
    for _ in range(3):
        est.model.train_step(ids.cuda(), torch.rand(256, 39).cuda(), torch.ones(256).cuda())
    v = est.model.tf_variables()
    assert tuple(v["Deep-part/mlp0/weights"].shape) == (39 * 8, 64)
    assert int(v["global_step"]) == 3 and "fm_v/Adam_1" in v
    prefix = est.export_tf_checkpoint(str(tmp_path))
    back = tb.read_bundle(prefix)
    est2 = Estimator(cfg)
    est2.model.load_tf_variables({k: torch.from_numpy(a) for k, a in back.items()})
    assert torch.equal(est2.model.tv, est.model.tv) and torch.equal(est2.model.p, est.model.p)
    assert torch.equal(est2.model.sv[1], est.model.sv[1]) and est2.model.global_step() == 3


@pytest.mark.parametrize("update", ["tf1_dense", "lazy"])
def test_native_auc_parity_with_golden(update):
    """SURVEY §6 parity: the native HIP path and the golden PyTorch transcription of the
    reference's TF1 model (models/reference.py), trained from the same init on the same batches
    with the same seeds (dropout masks are a shared counter hash) for 240 steps, reach the same
    held-out AUC (|dAUC| <= 0.005) along loss curves that agree within 2% per 40-step window."""
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import GoldenDeepFM, init_params
    from hipfm.ops.metrics import auc_from_hist, hist_torch
    dev = torch.device("cuda", 0)
    synth = make_synth("total:60000", seed=31)
    F, K, layers, keep, B = synth.F, 8, [128, 64, 32], [0.5, 0.5, 0.5], 512
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=12)
    kw = dict(optimizer="Adam", sparse_update=update, learning_rate=1e-3, seed=77)
    nat = NativeDeepFM(V, F, K, layers, keep, batch_size=B, device=dev, init=False, **kw)
    nat.load_tf_params(params)
    gold = GoldenDeepFM(V, F, K, layers, keep, params=params, **kw)
    ln, lg = [], []
    for s in range(240):
        ids, vals, lab = synth.batch(B, step=s)
        gold.train_step(ids, vals, lab)
        lg.append(gold.last_loss)
        nat.train_step(ids.to(dev, torch.int32), vals.to(dev), lab.to(dev), use_graph=True)
        ln.append(nat.loss_value(B))
    for w in range(0, 240, 40):
        a, b = np.mean(ln[w:w + 40]), np.mean(lg[w:w + 40])
        assert abs(a - b) <= 0.02 * b, (w, a, b)
    assert np.mean(ln[-40:]) < np.mean(ln[:40]) - 0.02           # it actually learned
    hn = torch.zeros(2, 201, dtype=torch.int64, device=dev)
    hg = torch.zeros(2, 201, dtype=torch.int64)
    for s in range(16):
        ids, vals, lab = synth.batch(B, step=100000 + s)
        nat.eval_batch(ids.to(dev, torch.int32), vals.to(dev), lab.to(dev), hn)
        hg += hist_torch(gold.predict(ids, vals), lab)
    an, ag = auc_from_hist(hn.cpu()), auc_from_hist(hg)
    assert ag > 0.6 and abs(an - ag) <= 0.005, (an, ag)


def test_streamed_epochs_through_the_ring_train_like_the_cached_run(dataset, monkeypatch):
    """Streamed epochs (no HBM cache, e.g. a dataset over the cache budget) go through the staging
    ring as captured multi-step runs; they train bitwise like the cached run (epoch 0 streamed
    through the ring, later epochs replayed from the cache), with the per-field sort from
    --field_sizes from the first step on.  Both wire formats: compact (the 26 categorical fields'
    1.0 values never cross the link, sparse.hip expand_vals rebuilds them on the device) and full."""
    from hipfm.cli import _EpochView
    from hipfm.config import RunConfig
    from hipfm.data.pipeline import InputPipeline, discover_files
    files = discover_files(dataset, "tr")
    from hipfm.data.synthetic import make_synth
    sizes = ",".join(str(hi - lo) for lo, hi in make_synth("total:50000").field_ranges())
    out = []
    for cache, compact, gdec in ((False, "1", "0"), (False, "0", "0"), (False, "1", "1"), (True, "1", "1")):
        monkeypatch.setenv("HIPFM_WIRE_COMPACT", compact)
        monkeypatch.setenv("HIPFM_GPU_DECODE", gdec)
        cfg = RunConfig(feature_size=50000, field_size=39, embedding_size=8, batch_size=512,
                        deep_layers="64,32", dropout="0.9,0.9", device="cuda", log_steps=0,
                        watchdog_secs=0, graph_steps=8, num_threads=4, field_sizes=sizes)
        est = Estimator(cfg)
        pipe = InputPipeline(files, 39, 512, 1, cache=cache, device=est.device, id_dtype=torch.int32,
                             threads=4, seed=cfg.seed)
        for e in range(3):
            est.train(_EpochView(pipe, e))
        assert est.model.field_ranges is not None
        if not cache:
            # streamed batches landed in the pipeline's device ring (one copy each, issued by the
            # fill thread); runs of consecutive slots were trained in place, so the Estimator's
            # own copy-in staging ring was never needed
            assert pipe.cached_batches == 0 and pipe._ring is not None
            assert getattr(est, "_ring", None) is None
            per_row = pipe.h2d_bytes / ((20000 // 512) * 512)
            if gdec == "1":
                # GPU decode: the raw Example bytes + an offset per row crossed the link, the ring
                # slots hold the decoded plain layout
                assert not pipe._ring.compact and per_row > 39 * 4, per_row
            else:
                assert pipe._ring.compact == (compact == "1")
                # (the generator's values: 13 real-valued fields, 26 fields of 1.0)
                assert per_row == (39 * 4 + 4 + 13 * 4 if compact == "1" else 39 * 8 + 4), per_row
        torch.cuda.synchronize()
        out.append((est.model.p.clone(), est.model.rec.clone(), est.global_step))
    assert out[0][2] == out[1][2] == out[2][2] == out[3][2] == 3 * (20000 // 512)
    for a in out[1:]:
        assert torch.equal(out[0][0], a[0]) and torch.equal(out[0][1], a[1])
