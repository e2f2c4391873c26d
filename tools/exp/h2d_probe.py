"""Pure PCIe copy rates with pinned host memory (tools only): H2D in 64/256 MB chunks over two
streams, D2H one copy."""
import time, torch
n = 1_500_000_000
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h.fill_(1)
d = torch.empty(n, dtype=torch.uint8, device='cuda')
d.copy_(h, non_blocking=True); torch.cuda.synchronize()  # warm
for chunk in (64 << 20, 256 << 20, 64 << 20):
    torch.cuda.synchronize()
    s = [torch.cuda.Stream() for _ in range(2)]
    t0 = time.perf_counter()
    for k, o in enumerate(range(0, n, chunk)):
        with torch.cuda.stream(s[k & 1]):
            d[o:o + chunk].copy_(h[o:o + chunk], non_blocking=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"H2D pinned chunk {chunk>>20} MB: {n/el/1e9:.1f} GB/s", flush=True)
r = torch.empty(n // 10, dtype=torch.uint8, pin_memory=True)
torch.cuda.synchronize(); t0 = time.perf_counter()
r.copy_(d[: n // 10], non_blocking=True); torch.cuda.synchronize()
print(f"D2H pinned: {n/10/(time.perf_counter()-t0)/1e9:.1f} GB/s")
