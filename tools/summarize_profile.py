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
if trace and b and b.get("roofline"):
    # the timed steps are the last steps x launches_per_step hash launches of the run (bench.py runs
    # warmup, then the timed steps; --stream-batches 0 --paths-log2 0 for the profiled command)
    rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
    mh = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
          if kname(r["Kernel_Name"]).endswith(("k_mp_hash", "k_mp_hash_wide"))]
    rf = b["roofline"]
    per_step = int(round(rf["launches_per_step"]))
    timed = b["steps"] * per_step
    iso = 5 * per_step if b.get("roofline_isolated") else 0
    if iso and len(mh) >= iso:
        i_ = mh[-iso:]
        ri = b["roofline_isolated"]
        avg_i = sum(i_) / len(i_) / 1e6
        print(f"\nMerkle hash launches of the isolated steps: {len(i_)} calls, trace average {avg_i:.4f} ms; bench "
              f"{ri['kernel_avg_ms']:.4f} ms ({(ri['kernel_avg_ms'] / avg_i - 1) * 100:+.1f}%); frac from the trace "
              f"{ri['perms_per_launch'] * ri['valu_ops_per_perm'] / (avg_i / 1e3) / (ri['peak'] * 1e12):.4f}, bench {ri['frac']:.4f}")
    if len(mh) >= timed + iso:
        t = mh[len(mh) - iso - timed:len(mh) - iso]
        avg_ms = sum(t) / len(t) / 1e6
        frac = rf["perms_per_launch"] * rf["valu_ops_per_perm"] / (avg_ms / 1e3) / (rf["peak"] * 1e12)
        print(f"\nMerkle hash launches of the timed steps: {len(t)} calls, trace average {avg_ms:.4f} ms; "
              f"bench kernel_avg_ms (in-kernel clocks) {rf['kernel_avg_ms']:.4f} ms "
              f"({(rf['kernel_avg_ms'] / avg_ms - 1) * 100:+.1f}%), HIP-event span / launches "
              f"{rf.get('kernel_avg_ms_events', float('nan')):.4f} ms")
        print(f"roofline frac from the trace: {rf['perms_per_launch']:.0f} perms/launch x {rf['valu_ops_per_perm']} / "
              f"{avg_ms:.4f} ms / {rf['peak']:.1f} T = {frac:.4f}; bench frac {rf['frac']:.4f}")
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
