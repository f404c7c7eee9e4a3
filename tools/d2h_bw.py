"""D2H bandwidth ceiling on the box (profiling): a 96 MB device buffer into pinned host
memory, whole and in 8 / 16 / 32 MB chunks, and into pageable memory."""
import time, torch
n = 96 << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d.fill_(1)
for pin in (True, False):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=pin)
    for chunk in (n, 8 << 20, 16 << 20, 32 << 20):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            for o in range(0, n, chunk):
                h[o:o + chunk].copy_(d[o:o + chunk], non_blocking=pin)
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 5
        print("pinned" if pin else "pageable", "chunk %d MB" % (chunk >> 20), "%.1f GB/s" % (n / dt / 1e9), flush=True)
