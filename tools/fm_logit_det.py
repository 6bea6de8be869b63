"""Gather-fused tower: per-sample FM logit (y_fm) across repeated launches vs an exact float64 host
value (the diagnosis of the packed-FP32 hazard, ops/build.py NO_PACKED_F32)."""
import sys
import torch
sys.path.insert(0, ".")
import hipfm  # noqa: F401,E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402

dev = torch.device("cuda", 0)
B = 16384
synth = make_synth("criteo_kaggle", seed=2024)
m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, seed=1234, batch_size=B,
                 device=dev, field_ranges=synth.field_ranges(), sparse_update="lazy")
ids, vals, _ = synth.batch(B, step=500_000, device=dev, id_dtype=torch.int32)
m.stage_batch(ids, vals, None)
torch.cuda.synchronize()
a = m._tower_args(B, train=False, with_labels=False, gather=m._fm_inputs(B, train=False))
ys = []
for r in range(8):
    m.y_fm.zero_()
    KN.tower(a, KE=m.K)
    torch.cuda.synchronize()
    ys.append(m.y_fm[:B].clone())
# exact FM logit
idl = ids.long()
v = m.tv[idl].double() * vals.double().unsqueeze(-1)        # [B, F, K]
w = m.tw[idl].double() * vals.double()
fb = float(m.p[m.dense_segs["fm_bias"].off])
ex = fb + w.sum(1) + 0.5 * (v.sum(1) ** 2 - (v * v).sum(1)).sum(1)
err = torch.stack([(y.double() - ex).abs() for y in ys])     # [runs, B]
ref = err.median(0).values
for r in range(8):
    bad = (ys[r] != ys[0]).nonzero().flatten().tolist()
    print(f"run {r}: differs from run 0 at {len(bad)} samples {bad[:6]}", flush=True)
    for b in bad[:3]:
        contrib = (w[b].abs()).tolist()
        print(f"   sample {b}: y0 {ys[0][b].item():.9g} yr {ys[r][b].item():.9g} exact {ex[b].item():.9g} "
              f"delta {ys[r][b].item() - ys[0][b].item():.3g}", flush=True)
        # does the delta match one field's w*x or v*x contribution?
        d = ys[r][b].item() - ys[0][b].item()
        fw = (w[b] - abs(d)).abs().argmin().item()
        print(f"     closest |w*x| field {fw}: {w[b][fw].item():.3g}", flush=True)
print("max |y - exact| (typical run):", float(ref.max()))
