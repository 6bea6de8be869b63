"""Determinism check of the predict path: graph-replayed predictions vs eager predict for every
request batch, several rounds (a mismatch means a race in the forward-only tower)."""
import sys
import torch
sys.path.insert(0, ".")
import hipfm  # noqa: F401,E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402

dev = torch.device("cuda", 0)
preset = sys.argv[1] if len(sys.argv) > 1 else "criteo_1tb"
synth = make_synth(preset, seed=2024)
B, P, G = 16384, 32, 16
m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5] * 3, seed=1234, batch_size=B,
                 device=dev, field_ranges=synth.field_ranges(), sparse_update="lazy")
reqs = [synth.batch(B, step=500_000 + i, device=dev, id_dtype=torch.int32) for i in range(P)]
out = torch.zeros(P, B, device=dev)


def serve(lo, hi):
    for i in range(lo, hi):
        m.stage_batch(reqs[i][0], reqs[i][1], None)
        m.predict_enqueue(B, with_labels=False)
        out[i].copy_(m.prob[:B])


serve(0, G)
torch.cuda.synchronize()
graphs = []
for g0 in range(0, P, G):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        serve(g0, g0 + G)
    graphs.append(g)
eager = torch.stack([m.predict(r[0], r[1]) for r in reqs])
e2 = torch.stack([m.predict(r[0], r[1]) for r in reqs])
print("eager vs eager: batches differing", int(((eager - e2).abs().amax(1) > 0).sum()))
for rnd in range(5):
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    d = (out - eager).abs()
    bad = (d.amax(1) > 0).nonzero().flatten().tolist()
    print(f"round {rnd}: batches differing {len(bad)} {bad[:8]} max {d.max().item():.3g} "
          f"elements {(d > 0).sum().item()}")
