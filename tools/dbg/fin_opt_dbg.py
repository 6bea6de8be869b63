"""Debug: fused finalize+dense optimizer vs separate dense_opt, step by step (g and p)."""
import sys
import torch
sys.path.insert(0, ".")
import hipfm  # noqa
import hipfm.models.deepfm as D
from hipfm.data.synthetic import make_synth
from hipfm.models.deepfm import NativeDeepFM
from hipfm.models.reference import init_params

DEV = torch.device("cuda", 0)
synth = make_synth("criteo_kaggle", seed=5)
F, K, layers, B = synth.F, 8, [128, 64, 32], 1024
params = init_params(synth.feature_size, F, K, layers, False, seed=2)
ms = []
for fuse in (True, False):
    D._FUSE_FIN_OPT = fuse
    m = NativeDeepFM(synth.feature_size, F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                     init=False, optimizer="Adam", sparse_update="lazy", field_ranges=synth.field_ranges())
    m.load_tf_params(params)
    ms.append(m)
graph = sys.argv[1] == "1" if len(sys.argv) > 1 else True
for s in range(4):
    ids, vals, lab = synth.batch(B, step=s, device=DEV, id_dtype=torch.int32)
    for m, fuse in zip(ms, (True, False)):
        D._FUSE_FIN_OPT = fuse
        m.train_step(ids, vals, lab, use_graph=graph)
    torch.cuda.synchronize()
    a, b = ms
    for nm in ("g", "p", "tv", "dX0"):
        x, y = getattr(a, nm).float(), getattr(b, nm).float()
        bad = (x != y).nonzero().flatten()
        print(f"graph={graph} step {s} {nm}: ndiff {bad.numel()} max {(x - y).abs().max().item():.3e} first {bad[:6].tolist()}", flush=True)
    print("fin_opt", a._fin_opt_step, b._fin_opt_step, "step", a.step.item(), b.step.item())
