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
b = json.load(open(bench)) if os.path.exists(bench) else None
trace = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
if trace and b and b.get("roofline_isolated"):
    # bench.py runs the timed steps (steps in flight), then 5 steps one at a time: split the Merkle
    # hash launches in time order into those two groups, each to compare with its bench figure
    rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
    mh = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
          if kname(r["Kernel_Name"]).endswith(("k_mp_hash", "k_mp_hash_wide"))]
    per_step = int(round(b["roofline"]["launches_per_step"]))
    iso = 5 * per_step
    timed = b["steps"] * per_step
    if len(mh) >= iso + timed:
        t, i = mh[-iso - timed:-iso], mh[-iso:]
        print(f"\nMerkle hash launches of the timed steps (2 in flight): {len(t)} calls, average "
              f"{sum(t) / len(t) / 1e6:.3f} ms; bench: {b['roofline']['kernel_avg_ms']:.3f} ms")
        print(f"Merkle hash launches of the isolated steps: {len(i)} calls, average {sum(i) / len(i) / 1e6:.3f} ms; "
              f"bench: {b['roofline_isolated']['kernel_avg_ms']:.3f} ms")
if b:
    print(f"\nbench (under profiler): value {b['value']:.4g} {b['unit']}, {b['ms_per_step']:.3f} ms per step, "
          f"kernel avg {b['roofline']['kernel_avg_ms']:.3f} ms\n")
print("## PMC (separate passes, per dispatch, averaged over dispatches of each kernel)\n")
print("| kernel | counter | dispatches | mean per dispatch |")
print("|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"| {k} | {c} | {len(v)} | {sum(v)/len(v):.6g} |")
