#!/usr/bin/env python3
"""Device occupancy of bench.py's timed region from a rocprofv3 --kernel-trace CSV: the region is
taken as the dispatches from the (warmup + 1)-th k_decode to the last k_verdicts (run bench.py with
--iso-steps 0 --group-batches 0 and no other legs).  Prints the region span, the time with any
kernel / a Tip5 hashing kernel running, and per 10% slice of the region the hashing coverage and
the kernels running: where a short run's fill and drain lose time.
Usage: python tools/region_util.py DIR_OR_CSV WARMUP"""
import csv
import glob
import sys

src = sys.argv[1]
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
f = src if src.endswith(".csv") else glob.glob(f"{src}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("nhip::", "").split("(")[0].split("<")[0].replace("void ", ""))
            for r in rows)
dec = [s for s, _, n in iv if n.startswith("k_decode")]
ver = [e for _, e, n in iv if n.startswith("k_verdicts")]
W0, W1 = dec[warm], max(ver)
HASH = ("k_hash_rows", "k_mp_hash")


def cover(names, a, b):
    segs = sorted((max(s, a), min(e, b)) for s, e, n in iv if e > a and s < b and any(n.startswith(x) for x in names))
    tot, cur_s, cur_e = 0, None, None
    for s, e in segs:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


span = W1 - W0
print(f"steps after warmup: {len(dec) - warm}, region {span / 1e6:.3f} ms")
print(f"any kernel {cover(('k_',), W0, W1) / span:.3f}, hashing {cover(HASH, W0, W1) / span:.3f}, "
      f"merkle {cover(('k_mp_hash',), W0, W1) / span:.3f}, rows {cover(('k_hash_rows',), W0, W1) / span:.3f}, "
      f"sponge {cover(('k_fs_replay',), W0, W1) / span:.3f}")
for k in range(10):
    a, b = W0 + span * k / 10, W0 + span * (k + 1) / 10
    names = {}
    for s, e, n in iv:
        if e > a and s < b:
            names[n] = names.get(n, 0) + min(e, b) - max(s, a)
    top = sorted(names.items(), key=lambda x: -x[1])[:5]
    print(f"{k * 10:3d}-{k * 10 + 10:3d}%  hash {cover(HASH, a, b) / (b - a):.2f}  " +
          "  ".join(f"{n} {v / (b - a):.2f}" for n, v in top))
