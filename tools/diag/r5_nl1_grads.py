"""compute_grads fused vs per-layer, per dense segment (diagnostic for the nl == 1 test)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hipfm  # noqa: F401
import hipfm.models.deepfm as D
from hipfm.data.synthetic import make_synth
from hipfm.models.deepfm import NativeDeepFM
from hipfm.models.reference import init_params

DEV = torch.device("cuda", 0)
synth = make_synth("criteo_kaggle", seed=47)
for layers, B in (([256], 4096), ([256], 1024), ([64, 32], 4096), ([16], 4096), ([256, 32], 4096)):
    params = init_params(synth.feature_size, synth.F, 8, layers, False, seed=11)
    batch = synth.batch(B, step=0, device=DEV, id_dtype=torch.int32)
    out = []
    for fused in (True, False):
        m = NativeDeepFM(synth.feature_size, synth.F, 8, layers, [0.5] * len(layers), batch_size=B, device=DEV,
                         init=False, sparse_update="lazy", field_ranges=synth.field_ranges(), fused=fused)
        m.load_tf_params(params)
        g, _, UG = m.compute_grads(*batch)
        torch.cuda.synchronize()
        out.append((g, UG, {k: (s.off, s.shape) for k, s in m.dense_segs.items()}, m._sp))
        del m
    (ga, ua, segs, sp), (gb, ub, _, _) = out
    print(layers, B, "plan:", sp)
    for k, (off, shape) in segs.items():
        n = int(torch.Size(shape).numel())
        a, b = ga[off:off + n], gb[off:off + n]
        print(f"  {k:32s} max|fused|={a.abs().max().item():.4g} max|layers|={b.abs().max().item():.4g} "
              f"max|diff|={(a - b).abs().max().item():.4g}")
    print("  UG max diff", (ua - ub).abs().max().item(), "scale", ub.abs().max().item())
