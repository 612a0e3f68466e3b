#!/usr/bin/env python3
"""Per-dispatch timeline of the last batch step from a rocprofv3 --kernel-trace CSV.
Usage: python tools/timeline.py DIR   (finds *kernel_trace.csv under DIR)"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at k_fs_replay_wide; take the last one
starts = [i for i, r in enumerate(rows) if "k_fs_replay_wide" in r["Kernel_Name"]]
i0 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
step = [r for r in rows[i0 - 2:] if "k_mtree" not in r["Kernel_Name"]]
for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].replace("nhip::", "").split("(")[0][:28]
    print(f"{name:28s} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3s} {s / 1e6:8.3f} -> {e / 1e6:8.3f}  {(e - s) / 1e6:7.3f} ms  grid {r.get('Grid_Size', '')}")
