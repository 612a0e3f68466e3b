#!/usr/bin/env python3
"""Occupancy of the device timeline from a rocprofv3 --kernel-trace CSV: over the middle part of the
run (default: the dispatches between 30% and 90% of the trace's time span, i.e. inside the timed
steps), the fraction of wall time with any kernel running, with a hashing kernel (row / Merkle
Tip5) running, and with only latency-bound kernels running; the time-weighted number of
concurrent kernels; each kernel's covered time (union of its dispatches).
Usage: python tools/trace_util.py DIR_OR_CSV [t0_frac t1_frac]"""
import csv
import glob
import os
import sys

src = sys.argv[1]
f = src if src.endswith(".csv") else glob.glob(f"{src}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Kind"] == "KERNEL_DISPATCH"]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("nhip::", "").split("(")[0])
      for r in rows]
t_lo, t_hi = min(s for s, _, _ in iv), max(e for _, e, _ in iv)
a = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
b = float(sys.argv[3]) if len(sys.argv) > 3 else 0.9
W0, W1 = t_lo + a * (t_hi - t_lo), t_lo + b * (t_hi - t_lo)
HASH = ("k_hash_rows", "k_mp_hash")
ev = []
for s, e, n in iv:
    s, e = max(s, W0), min(e, W1)
    if e > s:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
ev.sort(key=lambda x: (x[0], x[1]))
active = {}
last = W0
busy = hashing = only_lat = conc = 0.0
cover = {}
for t, d, n in ev:
    dt = t - last
    if dt > 0 and active:
        busy += dt
        conc += dt * sum(active.values())
        if any(k.split("<")[0].replace("void ", "") in HASH or k.startswith(HASH) for k in active):
            hashing += dt
        else:
            only_lat += dt
        for k in active:
            cover[k] = cover.get(k, 0.0) + dt
    last = t
    active[n] = active.get(n, 0) + d
    if active[n] == 0:
        del active[n]
span = W1 - W0
print(f"{os.path.basename(f)}: window {span / 1e6:.2f} ms ({a:.0%}-{b:.0%} of the trace)")
print(f"  busy {busy / span:.3f}  hashing kernel running {hashing / span:.3f}  only latency-bound kernels {only_lat / span:.3f}"
      f"  mean concurrent kernels {conc / max(busy, 1):.2f}")
for k, v in sorted(cover.items(), key=lambda x: -x[1]):
    print(f"  {k[:40]:40s} covers {v / span:.3f}")
