"""Compare the fused sparse backward fed by tower slot records (gslot) with the dX0 gathers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
fr = len(sys.argv) > 3 and sys.argv[3] == "fr"
synth = make_synth("criteo_kaggle", seed=3)
F, K, layers = synth.F, 8, [128, 64, 32]
params = init_params(synth.feature_size, F, K, layers, False, seed=1)
dev = torch.device("cuda", 0)
ms = []
for gs in (True, False):
    m = NativeDeepFM(synth.feature_size, F, K, layers, [0.5] * 3, batch_size=B, device=dev, init=False,
                     sparse_update="lazy", field_ranges=synth.field_ranges() if fr else None)
    m.load_tf_params(params)
    if not gs:
        m._gslot_mode = lambda: False
    for s in range(3):
        ids, vals, lab = synth.batch(B, step=s, device=dev, id_dtype=torch.int32)
        m.train_step(ids, vals, lab, use_graph=graph)
    torch.cuda.synchronize()
    ms.append(m)
a, b = ms
print("gslot", a._gslot_step, "ref", b._gslot_step)
for name, x, y in (("tv", a.tv, b.tv), ("tw", a.tw, b.tw), ("p", a.p, b.p)):
    d = (x - y).abs().max().item()
    print(name, "maxdiff", d, "scale", y.abs().max().item())
print("loss", a.loss_value(B), b.loss_value(B))
