"""The multi-rank step with real PROCESSES on the one GPU (HIPFM_SAME_DEVICE=1).

Each case launches N torchrun ranks of tests/mp_worker.py, all on device 0, exchanging through
the same-device engine (parallel/loopback.py, csrc/kernels/loopback.hip): every rank has its own
HIP context, caching allocator, streams and captured graphs, exactly as one process per GPU --
only the transport differs from RCCL.  The ranks' table shards and dense parameters must match
ONE model trained on the global batch (the in-process emulation's tolerance, tests/
test_gpu_shard.py), every rank must hold the same dense state and have issued the same collective
sequence, and the run modes must have captured graphs (the 8-GPU bench's first rung)."""
import os
import subprocess
import sys
import json

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)


def _free_port() -> int:
    import socket
    from hipfm.utils.net import free_port
    s = socket.socket()
    s.bind(("127.0.0.1", free_port()))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(N: int, cfg: dict, timeout: int = 240):
    env = dict(os.environ, HIPFM_SAME_DEVICE="1", HIPFM_LB_TIMEOUT_MS="60000", HSA_ENABLE_IPC_MODE_LEGACY="0",
               PYTHONUNBUFFERED="1")
    env.pop("HIPFM_XROWS", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={N}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "mp_worker.py"), json.dumps(cfg)]
    r = subprocess.run(cmd, env=env, cwd=REPO, timeout=timeout, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-6000:]
    return [torch.load(os.path.join(cfg["out"], f"rank{k}.pt"), weights_only=True) for k in range(N)]


def global_batch_model(N, B, steps, update, opt="Adam", lr=1e-3):
    synth = make_synth("criteo_kaggle", seed=4)
    F, K, layers, keep = synth.F, 8, [64, 32], [1.0, 1.0]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=7)
    ref = NativeDeepFM(V, F, K, layers, keep, optimizer=opt, sparse_update=update, learning_rate=lr * N,
                       batch_size=N * B, device=DEV, init=False, field_ranges=synth.field_ranges())
    ref.load_tf_params(params)
    for s in range(steps):
        ids, vals, lab = synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32)
        ref.train_step(ids, vals, lab)
    torch.cuda.synchronize()
    return ref


@pytest.mark.parametrize("N,sharded,update,mode", [
    (2, True, "lazy", "run"),            # the bench's first rung: run-level routing in a graph
    (4, True, "lazy", "run"),
    (2, True, "tf1_dense", "prefetch"),  # the CLI default update rule, per-step graphs + prefetch
    (3, True, "lazy", "eager"),
    (2, False, "lazy", "run"),           # replicated table (Horovod parity)
])
def test_processes_match_global_batch(tmp_path, N, sharded, update, mode):
    B, steps = 512, 3
    cfg = {"out": str(tmp_path), "sharded": sharded, "update": update, "mode": mode, "steps": steps, "B": B}
    outs = launch_ranks(N, cfg)
    ref = global_batch_model(N, B, steps, update)
    for o in outs:
        assert torch.equal(o["p"], outs[0]["p"])              # identical dense state on every rank
        assert torch.equal(o["trace"], outs[0]["trace"])      # identical collective sequence
        assert int(o["bytes_sent"]) > 0
        if mode != "eager":
            assert int(o["graphs"]) >= 1                      # the steps ran as captured graphs
    rtv, rtw, rp = ref.tv.float().cpu(), ref.tw.float().cpu(), ref.p.cpu()
    if sharded:
        full_v, full_w = torch.zeros_like(rtv), torch.zeros_like(rtw)
        for r, o in enumerate(outs):
            rows = full_v[r::N].shape[0]
            full_v[r::N] = o["tv"][:rows]
            full_w[r::N] = o["tw"][:rows]
    else:
        for o in outs:
            assert torch.equal(o["tv"], outs[0]["tv"]) and torch.equal(o["tw"], outs[0]["tw"])
        full_v, full_w = outs[0]["tv"], outs[0]["tw"]
    scale = rtv.abs().max().item()
    assert (full_v - rtv).abs().max().item() <= 2e-5 * scale
    assert (full_w - rtw).abs().max().item() <= 2e-5 * max(1.0, rtw.abs().max().item())
    assert (outs[0]["p"] - rp).abs().max().item() <= 2e-5 * rp.abs().max().item()


def test_launch_cli_two_ranks_train_eval_infer_export(tmp_path):
    """The reference user's flow with the launcher at N = 2 (mpirun -np / processes_per_host,
    NBHVD:87-92): train (epoch 0 streamed + cached, epoch 1 replayed from the HBM cache as graphs),
    eval, infer and export through ``python -m hipfm.launch --nproc_per_node 2 -m hipfm``, every
    rank a real process on the one GPU (row-sharded table, same-device engine)."""
    data = tmp_path / "data"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(data), "--preset", "total:50000", "--train_rows", "20000",
                           "--val_rows", "4000", "--test_rows", "500", "--files", "4"], cwd=REPO)
    md, sd, pred = tmp_path / "m", tmp_path / "s", tmp_path / "pred.txt"
    common = ["--training_data_dir", str(data), "--val_data_dir", str(data), "--model_dir", str(md),
              "--servable_model_dir", str(sd), "--pred_path", str(pred), "--feature_size", "50000",
              "--field_size", "39", "--embedding_size", "8", "--batch_size", "512", "--deep_layers", "64,32",
              "--dropout", "0.9,0.9", "--learning_rate", "0.003", "--log_steps", "10", "--device", "cuda",
              "--embedding_mode", "sharded"]
    env = dict(os.environ, HIPFM_SAME_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    for task, extra in (("train", ["--num_epochs", "2"]), ("eval", []), ("infer", []), ("export", [])):
        cmd = [sys.executable, "-m", "hipfm.launch", "--nproc_per_node", "2", "--master_port", str(_free_port()),
               "-m", "hipfm", "--task_type", task] + common + extra
        r = subprocess.run(cmd, env=env, cwd=REPO, timeout=300, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True)
        assert r.returncode == 0, f"{task}:\n" + r.stdout[-6000:]
    evals = [json.loads(line) for line in open(md / "metrics.jsonl") if '"eval"' in line]
    assert evals and evals[-1]["auc"] > 0.70, evals[-1:]
    steps = 2 * (20000 // 2 // 512)
    assert evals[-1]["global_step"] == steps, evals[-1]
    assert sum(1 for _ in open(pred)) == 500
    exports = [p for p in sd.iterdir() if p.is_dir()]
    assert exports and (exports[0] / "saved_model.pb").exists()
