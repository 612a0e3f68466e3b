#!/usr/bin/env python3
"""Summarize a tools/profile_round.sh output directory into a markdown table.
Usage: python tools/summarize_profile.py gpurun_out/prof_TAG > profiles/TAG/SUMMARY.md"""
import collections
import csv
import glob
import json
import os
import sys


def kname(full):
    full = full.replace("(anonymous namespace)::", "")
    return full.split("(")[0]

d = sys.argv[1]
print(f"# rocprofv3 summary: {os.path.basename(d)}\n")
stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
if stats:
    print("## Kernel trace (--kernel-trace --stats)\n")
    print("| kernel | calls | avg ms | min ms | max ms | % |")
    print("|---|---|---|---|---|---|")
    for r in csv.DictReader(open(stats[0])):
        name = kname(r["Name"])
        print(f"| {name} | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | {float(r['MinNs'])/1e6:.3f} | "
              f"{float(r['MaxNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
if stats:
    tot_ns, calls = 0.0, 0
    for r in csv.DictReader(open(stats[0])):
        if kname(r["Name"]).endswith(("k_mp_hash", "k_mp_hash_wide")):
            tot_ns += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    if calls:
        print(f"\nMerkle hash launches (k_mp_hash + k_mp_hash_wide): {calls} calls, average "
              f"{tot_ns / calls / 1e6:.3f} ms per launch")
bench = os.path.join(d, "bench_trace.json")
if os.path.exists(bench):
    b = json.load(open(bench))
    print(f"\nbench (under profiler): value {b['value']:.4g} {b['unit']}, kernel avg {b['roofline']['kernel_avg_ms']:.3f} ms\n")
print("## PMC (separate passes, per dispatch, averaged over dispatches of each kernel)\n")
print("| kernel | counter | dispatches | mean per dispatch |")
print("|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"| {k} | {c} | {len(v)} | {sum(v)/len(v):.6g} |")
