"""Process launcher: one process per GPU (replaces ``mpirun`` + Horovod launch).

The reference's Horovod job is started by SageMaker with ``mpirun`` and
``processes_per_host`` (NBHVD:87-92); here:

  python -m hipfm.launch --nproc_per_node 8 -m hipfm --task_type train ...
  python -m hipfm.launch --nproc_per_node 8 bench.py --gpus 8

Every child gets torchrun-style ``RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
MASTER_ADDR / MASTER_PORT`` and initialises RCCL through ``torch.distributed`` (TCPStore
rendezvous, no MPI).  Multi-host: ``--nnodes/--node_rank`` or SageMaker's ``SM_HOSTS`` /
``SM_CURRENT_HOST`` / ``SM_NUM_GPUS``, or a parameter-server ``TF_CONFIG``.  If any rank fails, the others are terminated (Horovod's
"one rank died -> job shut down" behaviour, DOC p.22) and the failing exit code is returned.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time


def _sagemaker_defaults():
    hosts = os.environ.get("SM_HOSTS")
    if not hosts:
        return None
    try:
        hosts = json.loads(hosts)
    except ValueError:
        hosts = hosts.split(",")
    cur = os.environ.get("SM_CURRENT_HOST", hosts[0])
    return {"nnodes": len(hosts), "node_rank": hosts.index(cur) if cur in hosts else 0,
            "master_addr": hosts[0], "nproc": int(os.environ.get("SM_NUM_GPUS", "0") or 0)}


def _tf_config_defaults():
    """Map a parameter-server ``TF_CONFIG`` (reference C26, PS:414-428: cluster
    {chief|master, worker, ps}, task {type, index}) onto this launcher's node layout: every
    chief/master/worker host becomes a training node (synchronous data parallel over RCCL);
    ``ps`` and ``evaluator`` tasks have no role here (the embedding table lives in GPU HBM)
    and exit 0, so a PS-style launch configuration still starts the right processes."""
    raw = os.environ.get("TF_CONFIG")
    if not raw:
        return None
    try:
        tc = json.loads(raw)
    except ValueError:
        return None
    cluster, task = tc.get("cluster", {}), tc.get("task", {})
    nodes = []
    for role in ("chief", "master", "worker"):
        nodes += [(role, i, h) for i, h in enumerate(cluster.get(role, []))]
    if not nodes:
        return None
    ttype, tidx = task.get("type", "worker"), int(task.get("index", 0))
    if ttype in ("ps", "evaluator"):
        return {"idle_role": ttype}
    rank = next((k for k, (r, i, _) in enumerate(nodes) if r == ttype and i == tidx), 0)
    return {"nnodes": len(nodes), "node_rank": rank, "master_addr": nodes[0][2].split(":")[0]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="hipfm.launch")
    ap.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=0)
    ap.add_argument("--nnodes", type=int, default=0)
    ap.add_argument("--node_rank", "--node-rank", type=int, default=-1)
    ap.add_argument("--master_addr", "--master-addr", default="")
    ap.add_argument("--master_port", "--master-port", type=int, default=29517)
    argv = list(sys.argv[1:] if argv is None else argv)
    # launcher options come first; the target starts at "-m <module>" or the first positional
    cut = len(argv)
    i = 0
    while i < len(argv):
        tok = argv[i]
        if tok == "-m" or not tok.startswith("-"):
            cut = i
            break
        i += 1 if "=" in tok else 2
    own, target = argv[:cut], argv[cut:]
    a = ap.parse_args(own)
    a.module, a.script, a.args = None, None, []
    if target and target[0] == "-m":
        if len(target) < 2:
            ap.error("-m needs a module name")
        a.module, a.args = target[1], target[2:]
    elif target:
        a.script, a.args = target[0], target[1:]
    sm = _sagemaker_defaults() or _tf_config_defaults() or {}
    if "idle_role" in sm:
        print(f"[hipfm.launch] TF_CONFIG task type {sm['idle_role']!r} has no role in hipfm "
              "(no parameter servers: the table is sharded over GPU HBM); exiting", flush=True)
        return 0
    nnodes = a.nnodes or sm.get("nnodes", 1)
    node_rank = a.node_rank if a.node_rank >= 0 else sm.get("node_rank", 0)
    master = a.master_addr or sm.get("master_addr", "127.0.0.1")
    nproc = a.nproc_per_node or sm.get("nproc") or 0
    if nproc <= 0:
        try:
            import torch
            nproc = max(1, torch.cuda.device_count())
        except Exception:  # noqa: BLE001
            nproc = 1
    world = nnodes * nproc
    if a.module:
        cmd_tail = ["-m", a.module] + ([a.script] if a.script else []) + a.args
    else:
        if not a.script:
            ap.error("a script or -m module is required")
        cmd_tail = [a.script] + a.args
    procs = []
    for lr in range(nproc):
        env = dict(os.environ)
        env.update(RANK=str(node_rank * nproc + lr), LOCAL_RANK=str(lr), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=master, MASTER_PORT=str(a.master_port),
                   GROUP_RANK=str(node_rank))
        if env.get("HIPFM_SAME_DEVICE") == "1":        # one-GPU rehearsal: a CU slice per rank
            from .parallel.dist import same_device_env
            env.update(same_device_env(lr, nproc))
        procs.append(subprocess.Popen([sys.executable] + cmd_tail, env=env))
    rc = 0
    try:
        alive = set(range(nproc))
        while alive:
            for i in list(alive):
                r = procs[i].poll()
                if r is None:
                    continue
                alive.discard(i)
                if r != 0 and rc == 0:
                    rc = r
                    for j in alive:                      # one rank failed: stop the job
                        procs[j].send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        rc = 130
    return rc


if __name__ == "__main__":
    sys.exit(main())
