#!/usr/bin/env python3
# raw PCIe copy rates between pinned host memory and HBM (the e2e ceiling)
import time, torch
n = 512 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def rate(f, reps=10):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return reps * n / (time.perf_counter() - t) / 1e9
h2 = torch.empty(n, dtype=torch.uint8).pin_memory(); d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
print("h2d GB/s", round(rate(lambda: d.copy_(h, non_blocking=True)), 1))
print("d2h GB/s", round(rate(lambda: h.copy_(d, non_blocking=True)), 1))
def both():
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
print("h2d+d2h concurrent GB/s each", round(rate(both), 1))
