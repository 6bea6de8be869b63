"""Run-to-run determinism check at bench batch size (1 GPU): two models from the same init train
the same resident batches with multi-step graphs; every parameter / slot tensor and the eval
forward must be bitwise equal.  usage: python tools/det_check.py [preset] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "criteo_kaggle"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    mode = sys.argv[3] if len(sys.argv) > 3 else "graph"      # graph | eager | eager_nosort
    dev = torch.device("cuda", 0)
    synth = make_synth(preset, seed=2024)
    B = 16384
    pool = [synth.batch(B, step=i, device=dev, id_dtype=torch.int32) for i in range(16)]
    states = []
    for run in range(2):
        m = NativeDeepFM(synth.feature_size, synth.F, 8, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4,
                         learning_rate=5e-4, optimizer="Adam", sparse_update="lazy", seed=1234,
                         batch_size=B, device=dev, field_ranges=synth.field_ranges())
        if mode == "graph":
            for s in range(0, steps, 16):
                m.train_steps(pool, next_ids=pool[0][0])
        else:
            for s in range(steps):
                nxt = pool[(s + 1) % 16][0] if mode == "eager" else None
                m.train_step(*pool[s % 16], next_ids=nxt)
        torch.cuda.synchronize()
        m.check_errors()
        ev = m.predict(*pool[3][:2])
        S1 = m.S.clone()
        for _ in range(3):
            ev2 = m.predict(*pool[3][:2])
            if not torch.equal(ev, ev2):
                bad = (ev != ev2).nonzero().reshape(-1)[:8].tolist()
                print(f"run {run}: predict differs on the SAME model: {int((ev != ev2).sum())} samples "
                      f"{bad}, max {float((ev - ev2).abs().max()):.3e}; S equal: {torch.equal(S1, m.S)}")
        st = {k: v.detach().clone() for k, v in m.state_dict_local().items()}
        if ev is not None:
            st["__pred"] = ev.detach().clone()
        states.append(st)
        del m
        torch.cuda.empty_cache()
    bad = []
    for k in states[0]:
        a, b = states[0][k], states[1][k]
        if not torch.equal(a, b):
            d = (a.float() - b.float()).abs()
            bad.append((k, int((d > 0).sum()), float(d.max())))
    print("deterministic" if not bad else f"DIFFERS: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
