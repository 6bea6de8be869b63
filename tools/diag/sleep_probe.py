import time, torch
torch.cuda.init(); x = torch.zeros(1, device="cuda"); torch.cuda.synchronize()
for c in (1_000_000, 100_000_000, 600_000_000):
    t = time.time(); torch.cuda._sleep(c); q = torch.cuda.current_stream().query(); torch.cuda.synchronize()
    print(c, f"{time.time() - t:.4f}s pending_after_enqueue={not q}")
