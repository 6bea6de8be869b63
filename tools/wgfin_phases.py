"""Per-workgroup phase timestamps of the wgfin launch (tower.hip built with -DWGF_TIMING):
start, K loop done, slab published + arrival counted, end.  Experiment harness only."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hipfm  # noqa: F401
from hipfm.data.synthetic import make_synth
from hipfm.models.deepfm import NativeDeepFM
from hipfm.ops._lib import get_lib

dev = torch.device("cuda", 0)
synth = make_synth(os.environ.get("PRESET", "criteo_1tb"), seed=2024)
B = 16384
m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, l2_reg=1e-4, learning_rate=5e-4,
                 optimizer="Adam", sparse_update="lazy", seed=1234, batch_size=B, device=dev,
                 field_ranges=synth.field_ranges())
pool = [synth.batch(B, step=i, device=dev, id_dtype=torch.int32) for i in range(16)]
for _ in range(3):
    m.train_steps(pool, next_ids=pool[0][0])
torch.cuda.synchronize()
buf = np.zeros(2048 * 4, dtype=np.uint64)
lib = get_lib()
lib.hfm_wgfin_ts.argtypes = [C.c_void_p]
assert lib.hfm_wgfin_ts(buf.ctypes.data) == 0
n = m._wgfin_wgs + 1
t = buf[: n * 4].reshape(n, 4).astype(np.int64)
t0 = t[:, 0].min()
us = (t - t0) / 100.0          # wall clock: 100 MHz
tiles = us[:-1]
print(f"NS={m._wgfin_ns} tile WGs={n - 1}")
for name, col in (("start", tiles[:, 0]), ("kloop", tiles[:, 1] - tiles[:, 0]), ("publish", tiles[:, 2] - tiles[:, 1]),
                  ("tail", tiles[:, 3] - tiles[:, 2]), ("end", tiles[:, 3])):
    print(f"{name:8s} min {col.min():7.2f} med {np.median(col):7.2f} max {col.max():7.2f}")
print(f"head WG: start {us[-1, 0]:.2f} end {us[-1, 3]:.2f}")
last = tiles[:, 3] - tiles[:, 2] > 0.5
print(f"last arrivers: {int(last.sum())}, their tail med {np.median((tiles[:, 3] - tiles[:, 2])[last]) if last.any() else 0:.2f}")
