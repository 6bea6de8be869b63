"""Host cost of one memoized multi-step graph replay (NativeDeepFM.train_steps) vs the GPU time
of the steps it launches (Kaggle shape, B = 16384, 20-step run): how much of a short timed
window is Python before the GPU gets work."""
import sys
import time
import torch
sys.path.insert(0, ".")
import hipfm  # noqa: F401,E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402

dev = torch.device("cuda", 0)
synth = make_synth("criteo_kaggle", seed=2024)
B, N = 16384, 20
m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, seed=1234, batch_size=B,
                 device=dev, field_ranges=synth.field_ranges(), sparse_update="lazy")
pool = [synth.batch(B, step=i, device=dev, id_dtype=torch.int32) for i in range(2 * N)]
for _ in range(3):
    m.train_steps(pool[:N], next_ids=pool[N][0])
    m.train_steps(pool[N:], next_ids=pool[0][0])
torch.cuda.synchronize()
host, gpu = [], []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    m.train_steps(pool[:N], next_ids=pool[N][0])
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.append((t1 - t0) * 1e6)
    gpu.append(e0.elapsed_time(e1) * 1e3)
    m.train_steps(pool[N:], next_ids=pool[0][0])
    torch.cuda.synchronize()
    print(f"train_steps host call {host[-1]:7.1f} us, events {gpu[-1]:8.1f} us, wall {(t2 - t0) * 1e6:8.1f} us",
          flush=True)
