"""Standalone timing of the tf1_dense split sweep (optim.hip tf1_sweep_kernel) on a
Criteo-Kaggle-sized record table: us per sweep and effective HBM rate vs workgroup count."""
import sys
import torch
sys.path.insert(0, ".")
import hipfm  # noqa: F401,E402
from hipfm.ops import kernels as KN  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 1338431
dev = torch.device("cuda", 0)
rec = torch.zeros(R, 32, device=dev)
rec[:, :9] = torch.randn(R, 9, device=dev) * 0.01
flags = torch.zeros(R, dtype=torch.uint8, device=dev)
step = torch.zeros(1, dtype=torch.int64, device=dev)
done = torch.zeros(1, dtype=torch.int32, device=dev)
h = KN.hyper(5e-4, 1e-4)
for wg in (64, 128, 256, 512, 1024, 2048, 8192):
    for _ in range(3):
        KN.tf1_sweep(8, 0, rec, flags, h, step, done, max_wg=wg)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        KN.tf1_sweep(8, 0, rec, flags, h, step, done, max_wg=wg)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    print(f"wg={wg:5d}  {us:7.1f} us/sweep  {2 * R * 128 / us / 1e6:5.2f} TB/s (128 B read + written per row)")

# reference point: a plain device copy of the same bytes (read + write), torch's copy kernel
src = torch.empty_like(rec)
for _ in range(3):
    rec.copy_(src)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    rec.copy_(src)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / 20
print(f"torch copy_ of the table: {us:7.1f} us  {2 * R * 128 / us / 1e6:5.2f} TB/s")
