#!/usr/bin/env python3
"""Host-to-device copy bandwidth from pinned memory: one copy vs the same bytes split over 2 / 4
streams (PCIe-inclusive path).  Usage: python tools/h2d_bw.py [GB]"""
import sys
import time

import torch

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.33
n = int(gb * (1 << 30)) // 8
src = torch.empty(n, dtype=torch.int64, pin_memory=True)
src.fill_(1)
dst = torch.empty(n, dtype=torch.int64, device="cuda:0")
for parts in (1, 2, 4, 8):
    streams = [torch.cuda.Stream() for _ in range(parts)]
    cuts = [n * i // parts for i in range(parts + 1)]
    best = 1e9
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for s, a, b in zip(streams, cuts[:-1], cuts[1:]):
            with torch.cuda.stream(s):
                dst[a:b].copy_(src[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{parts} stream(s): {n * 8 / best / 1e9:.1f} GB/s ({best * 1e3:.1f} ms for {n * 8 / 1e9:.2f} GB)", flush=True)
