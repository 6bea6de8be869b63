"""Diagnostics: per-column BN gradient error vs column statistics (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import hipfm  # noqa
from hipfm.data.synthetic import make_synth
from hipfm.models.deepfm import NativeDeepFM
from hipfm.models.reference import GoldenDeepFM, init_params

synth = make_synth("total:4000", seed=20)
F, K, layers, keep = synth.F, 8, [64, 32], [0.5, 0.75]
V = synth.feature_size
p = init_params(V, F, K, layers, True, seed=7)
g = torch.Generator().manual_seed(8)
for i, L in enumerate(layers):
    p[f"Deep-part/bn_{i}/gamma"] = 1.0 + 0.3 * torch.rand(L, generator=g)
    p[f"Deep-part/bn_{i}/beta"] = 0.1 * torch.randn(L, generator=g)
B = 512
for kp in ([0.5, 0.75], [1.0, 1.0]):
    nat = NativeDeepFM(V, F, K, layers, kp, batch_size=B, device="cuda", init=False, batch_norm=True)
    nat.load_tf_params(p)
    gold = GoldenDeepFM(V, F, K, layers, kp, params=p, batch_norm=True)
    ids, vals, labels = synth.batch(B, step=0)
    _, data, gg = gold.compute_grads(ids, vals, labels)
    gnat, _, _ = nat.compute_grads(ids.to("cuda", torch.int32), vals.to("cuda"), labels.to("cuda"))
    torch.cuda.synchronize()
    dense = nat.dense_tf_params(gnat)
    print("keep", kp, "loss", nat.loss_value(B), float(data))
    for k in dense:
        d = (dense[k] - gg[k]).abs()
        print(f"  {k:32s} maxerr {d.max().item():.3e} maxref {gg[k].abs().max().item():.3e}")
    d = (dense["Deep-part/mlp1/weights"] - gg["Deep-part/mlp1/weights"]).abs()
    print("  mlp1 per-out-col max err:", [f"{x:.1e}" for x in d.max(0).values.tolist()])
    print("  mlp1 per-in-row max err:", [f"{x:.1e}" for x in d.max(1).values.tolist()])
    # golden hidden stats
    with torch.no_grad():
        x = vals.reshape(-1, F).float()
        E = p["fm_v"][ids.reshape(-1, F).long()] * x.unsqueeze(-1)
        h = E.reshape(B, -1)
        r0 = torch.relu(h @ p["Deep-part/mlp0/weights"] + p["Deep-part/mlp0/biases"])
        print("  R0 col std min/max", r0.std(0).min().item(), r0.std(0).max().item(),
              "frac>0 min", (r0 > 0).float().mean(0).min().item())
    # compare native H0 / Ht0 consistency
    H0 = nat.H[0][:B].float().cpu()
    Ht0 = nat.Ht[0][:, :B].float().cpu().t()
    print("  H0 vs Ht0^T max diff", (H0 - Ht0).abs().max().item())
    dZ1 = nat.dZ[1][:B].float().cpu()
    dZt1 = nat.dZt[1][:, :B].float().cpu().t()
    print("  dZ1 vs dZt1^T max diff", (dZ1 - dZt1).abs().max().item())
    # recompute dW1 on host from native dZ1 and H0
    dW1 = (dZ1.t() @ H0)[:32, :64].t()
    print("  host dW1 from native tensors vs native dW1:", (dW1 - dense["Deep-part/mlp1/weights"]).abs().max().item(),
          " vs golden:", (dW1 - gg["Deep-part/mlp1/weights"]).abs().max().item())
    gold16 = GoldenDeepFM(V, F, K, layers, kp, params=p, batch_norm=True, mlp_bf16=True)
    _, _, gg16 = gold16.compute_grads(ids, vals, labels)
    for k in dense:
        d = (dense[k] - gg16[k]).abs()
        print(f"  vs bf16-golden {k:32s} maxerr {d.max().item():.3e} maxref {gg16[k].abs().max().item():.3e}")
