"""Randomized check of the executor's host-side plan state (models/runner.py: prefetched sorts and
routing sets, tf1_dense flag sets, the run memo, captured graphs): random sequences of
train_step (eager or graph, with 0 / 1 / 2 declared upcoming batches), train_steps (run-level
sort / routing, with or without a lookahead), predict, eval_batch, reset_plan_state and a state
load, each followed by a BITWISE comparison with a reference model that trains the same batches
as plain eager single steps.  A declared upcoming batch that is then not stepped (a dropped
prefetch), a served-ahead set left behind by a replayed run, stale stamps after a load -- the
round-3 stale-state bugs -- all surface here as a parameter mismatch."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402

B = 512
P = 5            # resident pool
SEQS = 67        # random sequences per mode (~200 over the three modes)
OPS = 8          # operations per sequence


@pytest.fixture(scope="module")
def group():
    if not dist.is_initialized():
        from hipfm.utils.net import free_port
        s = socket.socket()
        s.bind(("127.0.0.1", free_port()))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield


def _same(a, b, what):
    torch.cuda.synchronize()
    for n, x, y in (("p", a.p, b.p), ("rec", a.rec, b.rec), ("step", a.step, b.step)):
        if not torch.equal(x, y):
            d = (x.double() - y.double()).abs().max().item()
            pytest.fail(f"{what}: {n} differs (max {d:.3e})")


@pytest.mark.parametrize("mode,update", [("local", "lazy"), ("local", "tf1_dense"), ("sharded", "lazy")])
def test_random_op_sequences_match_eager_steps(group, mode, update):
    from hipfm.parallel.dist import Comm
    synth = make_synth("total:6000", seed=31)
    F, K, layers, keep = synth.F, 8, [64, 32], [0.8, 0.8]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=4)
    pool = [synth.batch(B, step=s, device="cuda", id_dtype=torch.int32) for s in range(P)]

    def make(comm):
        m = NativeDeepFM(V, F, K, layers, keep, sparse_update=update, batch_size=B, device="cuda",
                         init=False, comm=comm, field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        return m

    comm = Comm(sharded=True, force_exchange=True) if mode == "sharded" else None
    rng = random.Random(7 if update == "lazy" else 8)
    a, ref = make(comm), make(Comm(sharded=True, force_exchange=True) if comm is not None else None)
    log = []
    for seq in range(SEQS):
        for op_i in range(OPS):
            op = rng.choices(["step", "steps", "predict", "eval", "reset", "load"], [4, 3, 1, 1, 1, 1])[0]
            nxt_kind = rng.choice(["none", "one", "two"])
            nxt = None
            if nxt_kind != "none":
                j, k = rng.randrange(P), rng.randrange(P)
                nxt = pool[j][0] if nxt_kind == "one" else (pool[j][0], pool[k][0])
            if op == "step":
                i = rng.randrange(P)
                g = rng.random() < 0.7
                log.append(f"step({i}, graph={g}, next={nxt_kind})")
                a.train_step(*pool[i], use_graph=g, next_ids=nxt)
                ref.train_step(*pool[i], use_graph=False)
            elif op == "steps":
                i0, n = rng.randrange(P), rng.randint(2, 4)
                run = [pool[(i0 + t) % P] for t in range(n)]
                log.append(f"steps({i0}..+{n}, next={nxt_kind})")
                a.train_steps(run, next_ids=nxt)
                for b in run:
                    ref.train_step(*b, use_graph=False)
            elif op == "predict":
                i = rng.randrange(P)
                log.append(f"predict({i})")
                pa, pr = a.predict(pool[i][0], pool[i][1]), ref.predict(pool[i][0], pool[i][1])
                torch.cuda.synchronize()
                assert torch.equal(pa, pr), f"predict differs after {log}"
            elif op == "eval":
                i = rng.randrange(P)
                log.append(f"eval({i})")
                ha = torch.zeros(2, 201, dtype=torch.int64, device="cuda")
                hr = torch.zeros_like(ha)
                a.eval_batch(*pool[i], ha)
                ref.eval_batch(*pool[i], hr)
                torch.cuda.synchronize()
                assert torch.equal(ha, hr), f"eval histogram differs after {log}"
            elif op == "reset":
                log.append("reset")
                a.reset_plan_state()
            else:
                log.append("load")
                a.load_state_dict_local(ref.state_dict_local())
            _same(a, ref, f"after {log}")
        a.check_errors()
        ref.check_errors()
