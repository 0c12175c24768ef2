"""H2D / D2H rate against transfer size, pinned and pageable host memory
(why C2's 12.9 MB H2D ran at 35 GB/s and C3's 144 MB at 55):
python tools/h2d_sweep.py  -> one line per (direction, memory, size): median of 9 copies"""
import time
import numpy as np
import torch

dev = torch.device("cuda:0")
torch.cuda.init()
sizes = [1 << 20, 4 << 20, 13 << 20, 32 << 20, 64 << 20, 144 << 20]
s = torch.cuda.Stream()
for mem in ("pinned", "pageable"):
    for n in sizes:
        h = torch.empty(n, dtype=torch.uint8, pin_memory=(mem == "pinned"))
        h.fill_(7)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        for direction in ("h2d", "d2h"):
            ts = []
            for _ in range(9):
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                with torch.cuda.stream(s):
                    e0.record(s)
                    if direction == "h2d":
                        d.copy_(h, non_blocking=True)
                    else:
                        h.copy_(d, non_blocking=True)
                    e1.record(s)
                s.synchronize()
                wall = time.perf_counter() - t0
                ts.append((e0.elapsed_time(e1) / 1e3, wall))
            ev = float(np.median([t[0] for t in ts]))
            wl = float(np.median([t[1] for t in ts]))
            print(f"{direction} {mem:8s} {n / 1e6:7.1f} MB  events {n / ev / 1e9:6.1f} GB/s ({ev * 1e6:8.1f} us)  "
                  f"wall {n / wl / 1e9:6.1f} GB/s ({wl * 1e6:8.1f} us)", flush=True)
