"""Does a pool stream run while the launching (default) stream is busy?  (fresh process)"""
import threading
import time

import torch

x = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()


def probe(tag, in_thread, n=4, warm=False):
    res = []
    if warm:
        torch.cuda.synchronize()
    torch.cuda._sleep(500_000_000)                   # the default stream: busy ~0.2 s

    def body(i):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            y = x + i                                # tiny kernel (+ allocation)
        time.sleep(0.02)
        res.append((i, s.query(), s.stream_id))
        del y
    if in_thread:
        th = [threading.Thread(target=body, args=(i,)) for i in range(n)]
        [t.start() for t in th]
        [t.join() for t in th]
    else:
        for i in range(n):
            body(i)
    busy = not torch.cuda.current_stream().query()
    torch.cuda.synchronize()
    print(tag, "default still busy:", busy, "pool streams done early:", sorted(res), flush=True)


probe("main-thread cold", False)
probe("main-thread warm", False)
probe("threads", True)
probe("threads again", True)
