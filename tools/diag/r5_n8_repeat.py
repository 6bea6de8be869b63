"""Round-5 diagnostic: is the n8 sharded emulation or its one-model oracle nondeterministic?
Runs each side twice in ONE process (the second run on a warm caching allocator) and reports
bitwise equality and the distance between the sides."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
if os.environ.get("R5_GUARD"):     # guard zones around every device allocation (tools/guard_alloc)
    _ga = torch.cuda.memory.CUDAPluggableAllocator(
        os.path.join(REPO, "tools", "guard_alloc", "libguard_alloc.so"), "hfm_guard_malloc", "hfm_guard_free")
    torch.cuda.memory.change_current_allocator(_ga)
import hipfm  # noqa: E402,F401
import hipfm.models.deepfm as D  # noqa: E402
D._XROWS = os.environ.get("R5_XROWS", "fp32")
import test_gpu_shard as T  # noqa: E402


def diff(a, b):
    return max((x - y).abs().max().item() for x, y in zip(a, b))


synth, data, batches = T.n8_data()
uids = torch.unique(torch.cat([d[0].reshape(-1) for d in data]).long())
order = sys.argv[1] if len(sys.argv) > 1 else "ssrr"
POISON = int(os.environ.get("R5_POISON", "255"))


def poison():
    """Fill (almost) all free HBM with a byte pattern through the caching allocator and free it
    again: later allocations are carved from these segments, so any read past a buffer's end
    (inside its 512-B rounding or into a neighbour's free block) sees the pattern, not zeros."""
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    sizes, left = [], free - (6 << 30)
    for sz in (112 << 30, 40 << 30, 16 << 30, 16 << 30, 8 << 30, 8 << 30, 4 << 30, 4 << 30, 2 << 30,
               2 << 30, 1 << 30, 1 << 30, 256 << 20, 256 << 20, 64 << 20, 64 << 20, 16 << 20, 4 << 20):
        if sz <= left:
            sizes.append(sz)
            left -= sz
    keep = []
    for sz in sizes:
        t = torch.empty(sz, dtype=torch.uint8, device="cuda")
        t.fill_(POISON)
        keep.append(t)
    torch.cuda.synchronize()
    print(f"poisoned {sum(sizes) / (1 << 30):.0f} GB with byte {POISON:#x}", flush=True)
    del keep


res = {}
for i, c in enumerate(order):
    if c == "p":
        poison()
        continue
    if c == "k":            # advance torch's stream pool by one stream (shifts the HW-queue mapping)
        _ks = torch.cuda.Stream()
        continue
    t = time.time()
    res[i] = T.n8_sharded(synth, data, batches, uids) if c == "s" else T.n8_single(synth, data, uids)
    print(f"run {i} ({'sharded' if c == 's' else 'single'}) {time.time() - t:.1f}s", flush=True)
if os.environ.get("R5_SAVE"):
    torch.save([t.cpu() for t in res[min(res)]], os.environ["R5_SAVE"])
if os.environ.get("R5_CMP"):
    ref = torch.load(os.environ["R5_CMP"], weights_only=True)
    for i in res:
        got = [t.cpu() for t in res[i]]
        print(f"{order[i]}{i} vs saved: " + " ".join(
            f"max|d|={(a - b).abs().max().item():.3e} nan={int(torch.isnan(a).sum())}" for a, b in zip(got, ref)),
            flush=True)
for i in res:
    for j in res:
        if j <= i:
            continue
        print(f"{order[i]}{i} vs {order[j]}{j}: max|dv|={diff(res[i][:1], res[j][:1]):.3e} "
              f"max|dw|={diff(res[i][1:2], res[j][1:2]):.3e} dense={diff(res[i][2:], res[j][2:]):.3e} "
              f"bitwise={all(torch.equal(x, y) for x, y in zip(res[i], res[j]))}", flush=True)
