import time, torch, numpy as np
d = torch.device("cuda:0")
for mb in (8, 64, 256):
    a = np.random.randint(0, 255, size=mb << 20, dtype=np.uint8)
    t = torch.from_numpy(a)
    g = torch.empty(mb << 20, dtype=torch.uint8, device=d)
    for i in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter(); g.copy_(t); torch.cuda.synchronize(); dt = time.perf_counter() - t0
    p = t.pin_memory()
    for i in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter(); g.copy_(p, non_blocking=True); torch.cuda.synchronize(); dt2 = time.perf_counter() - t0
    print("%d MB pageable %.2f GB/s pinned %.2f GB/s" % (mb, (mb << 20) / dt / 1e9, (mb << 20) / dt2 / 1e9), flush=True)
