"""Diagnostic: N emulated row-sharded ranks on one GPU (tests/test_gpu_shard.py MeshEngine) vs
one model on the global batch; prints the max errors.  Knobs come from the environment, so a
shell loop can bisect execution variants:  python tools/diag/shard_emul_check.py N B preset steps"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import hipfm  # noqa: E402,F401
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402
from hipfm.parallel.sharded import estimate_capacity  # noqa: E402
from test_gpu_shard import MeshComm, _Hub, _fill_tables, _run_ranks  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    N, B = int(sys.argv[1]), int(sys.argv[2])
    preset = sys.argv[3] if len(sys.argv) > 3 else "criteo_kaggle"
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    prefetch = os.environ.get("DIAG_PREFETCH", "1") == "1"
    fr = os.environ.get("DIAG_FIELD_RANGES", "1") == "1"
    synth = make_synth(preset, seed=2024)
    F, K, layers, keep = synth.F, 8, [128, 64, 32], [1.0, 1.0, 1.0]
    V = synth.feature_size
    fill = V > (1 << 24)                  # huge tables: hashed init on the GPU (no host tables)
    params = init_params(V, F, K, layers, False, seed=11, tables=not fill)
    okw = dict(adam_epsilon=1e-2, optimizer="Adam", sparse_update="lazy", device=DEV, init=False,
               field_ranges=synth.field_ranges() if fr else None)
    data = [synth.batch(N * B, step=s, device=DEV, id_dtype=torch.int32) for s in range(steps)]
    batches = [[(ids[r * B:(r + 1) * B].contiguous(), vals[r * B:(r + 1) * B].contiguous(),
                 lab[r * B:(r + 1) * B].contiguous()) for ids, vals, lab in data] for r in range(N)]
    cap = max(estimate_capacity((batches[r][s][0] for s in range(steps)), N) for r in range(N))
    hub = _Hub(N)
    models = []
    for r in range(N):
        m = NativeDeepFM(V, F, K, layers, keep, learning_rate=5e-4, batch_size=B,
                         comm=MeshComm(hub, r, capacity=cap), **okw)
        m.load_tf_params(params)
        if fill:
            _fill_tables(m, N, r)
        models.append(m)
    _run_ranks(models, batches, prefetch)
    torch.cuda.synchronize()
    for m in models:
        m.check_errors()
    uids = torch.unique(torch.cat([d[0].reshape(-1) for d in data]).long())
    got = torch.empty(uids.numel(), K, device=DEV)
    for r, m in enumerate(models):
        sel = (uids % N) == r
        got[sel] = m.tv[uids[sel] // N]
    p_sh = models[0].p.clone()
    del models, hub
    torch.cuda.empty_cache()
    ref = NativeDeepFM(V, F, K, layers, keep, learning_rate=5e-4 * N, batch_size=N * B, **okw)
    ref.load_tf_params(params)
    if fill:
        _fill_tables(ref, 1, 0)
    v0 = ref.tv[uids].clone()
    for ids, vals, lab in data:
        ref.train_step(ids, vals, lab)
    torch.cuda.synchronize()
    rv = ref.tv[uids]
    d = (got - rv).abs()
    upd = (rv - v0).abs()
    bad = (d > 1e-2 * upd.max()).any(1).nonzero().reshape(-1)
    print(f"N={N} B={B} prefetch={prefetch} field_ranges={fr} cap={cap} max|dv|={d.max().item():.3e} "
          f"max|update|={upd.max().item():.3e} bad_rows={bad.numel()}/{uids.numel()} "
          f"dense={(p_sh - ref.p).abs().max().item():.3e}", flush=True)
    if bad.numel():
        ids0 = uids[bad[:8]].tolist()
        print("bad ids:", ids0, "owner:", [x % N for x in ids0], "err:", d[bad[:8]].max(1).values.tolist(),
              "upd:", upd[bad[:8]].max(1).values.tolist())
        cnt = torch.cat([d[0].reshape(-1) for d in data]).long()
        print("occurrences:", [int((cnt == x).sum()) for x in ids0])


if __name__ == "__main__":
    main()
