"""Per-kernel launch floor: N tiny dependent kernels captured in one HIP graph (and eager).

  python tools/bench_launch.py            # prints us/kernel for graph replay and eager launch
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import hipfm  # noqa: F401
    from hipfm.ops import kernels as KN
    dev = torch.device("cuda")
    x = torch.zeros(1, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    N = 200
    res = {}
    for name, fn in (("torch_add", lambda: x.add_(1.0)), ("hipfm_step_inc", lambda: KN.step_inc(step))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / N * 1e6
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                for _ in range(N):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / (reps * N) * 1e6
        res[name] = (eager, graph)
        print(f"{name:16s} eager {eager:6.2f} us/kernel   graph {graph:6.2f} us/kernel "
              f"(env HIP_FORCE_DEV_KERNARG={os.environ.get('HIP_FORCE_DEV_KERNARG', '')})", flush=True)


def xstream():
    """Cost of graph branches: per iteration, a tiny kernel on the main stream, optionally a
    tiny kernel on a side stream forked from main (joined back at once, joined next iteration,
    or never joined until the end), then another main kernel."""
    import hipfm  # noqa: F401
    from hipfm.ops import kernels as KN
    dev = torch.device("cuda")
    a = torch.zeros(1, dtype=torch.int64, device=dev)
    b = torch.zeros(1, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream()
    N = 100

    def body(mode):
        main = torch.cuda.current_stream()
        for _ in range(N):
            KN.step_inc(a)
            if mode != "none":
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    KN.step_inc(b)
                if mode == "join":
                    main.wait_stream(side)
            KN.step_inc(a)
        if mode != "none":
            main.wait_stream(side)

    for mode in ("none", "join", "fork_only"):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                body(mode)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / (reps * N) * 1e6
        print(f"xstream {mode:10s}: {us:6.2f} us per iteration (2 main kernels [+ 1 side])", flush=True)


if __name__ == "__main__":
    if "--xstream" in sys.argv:
        xstream()
    else:
        main()
