#!/usr/bin/env python3
"""Summarize a tools/profile_round.sh output directory into a markdown table.
Usage: python tools/summarize_profile.py gpurun_out/prof_TAG [iso] > profiles/TAG/SUMMARY.md

Default: the trace of in-flight steps only (trace/, bench_trace.json, bench --iso-steps 0: every
Merkle hash dispatch in trace_kernel_stats.csv belongs to a step with two in flight, so its average
is the bench roofline's kernel_avg_ms) and the PMC passes.  "iso": the second trace (trace_iso/,
bench_trace_iso.json) with the one-at-a-time steps after the timed region."""
import collections
import csv
import glob
import json
import os
import sys

MERKLE = ("k_mp_hash", "k_mp_hash_wide", "k_mp_hash_tail", "k_mp_climb")


def kname(full):
    full = full.replace("(anonymous namespace)::", "")
    full = full.split("(")[0]
    # template instances (k_mp_hash<6>, k_mp_hash<7>) count as their kernel for the Merkle roofline
    return full.split("<")[0] if full.split("<")[0].endswith(MERKLE) else full


def frac_of(rf, avg_ms):
    return rf["perms_per_launch"] * rf["valu_ops_per_perm"] / (avg_ms / 1e3) / (rf["peak"] * 1e12)


d = sys.argv[1]
iso_mode = len(sys.argv) > 2 and sys.argv[2] == "iso"
tdir = os.path.join(d, "trace_iso" if iso_mode else "trace")
bench = os.path.join(d, "bench_trace_iso.json" if iso_mode else "bench_trace.json")
b = json.load(open(bench)) if os.path.exists(bench) else None
if iso_mode:
    print("\n## Second trace: the same command with the one-at-a-time steps (bench --iso-steps 5)\n")
else:
    print(f"# rocprofv3 summary: {os.path.basename(d)}\n")
stats = glob.glob(os.path.join(tdir, "*kernel_stats.csv"))
if stats and not iso_mode:
    print("## Kernel trace (--kernel-trace --stats; in-flight steps only: bench --iso-steps 0)\n")
    print("| kernel | calls | avg ms | min ms | max ms | % |")
    print("|---|---|---|---|---|---|")
    for r in csv.DictReader(open(stats[0])):
        print(f"| {kname(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | {float(r['MinNs'])/1e6:.3f} | "
              f"{float(r['MaxNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
if stats and b and b.get("roofline"):
    tot_ns, calls = 0.0, 0
    for r in csv.DictReader(open(stats[0])):
        if kname(r["Name"]).endswith(MERKLE):
            tot_ns += float(r["TotalDurationNs"])
            calls += int(r["Calls"])
    if calls:
        avg = tot_ns / calls / 1e6
        rf = b["roofline"]
        print(f"\nMerkle hash launches in trace_kernel_stats.csv (every dispatch of the run): {calls} calls, "
              f"average {avg:.4f} ms per launch; roofline frac from it: {rf['perms_per_launch']:.0f} perms/launch "
              f"x {rf['valu_ops_per_perm']} / {avg:.4f} ms / {rf['peak']:.1f} T = {frac_of(rf, avg):.4f}; "
              f"bench kernel_avg_ms {rf['kernel_avg_ms']:.4f} ms, frac {rf['frac']:.4f}")
trace = glob.glob(os.path.join(tdir, "*kernel_trace.csv"))
if trace and b and b.get("roofline"):
    # bench.py runs warmup, then the timed steps, then (iso_steps > 0) the one-at-a-time steps;
    # --stream-batches 0 --paths-log2 0 for the profiled command
    rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
    mh = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if kname(r["Kernel_Name"]).endswith(MERKLE)]
    # round 4: with isolated steps, `roofline` is theirs and `roofline.inflight` the timed steps'
    # (round 3 lines: `roofline` timed, `roofline_isolated`)
    if "inflight" in b["roofline"]:
        ri, rf = b["roofline"], dict(b["roofline"], **b["roofline"]["inflight"])
    else:
        ri, rf = b.get("roofline_isolated"), b["roofline"]
    per_step = int(round(rf["launches_per_step"]))
    # round 5: roofline.inflight is a pass of `pass_steps` in-flight steps right after the timed
    # region (which runs without per-dispatch timestamps), before the isolated steps
    timed = rf.get("pass_steps", b["steps"]) * per_step
    iso = b.get("iso_steps", 5) * per_step if ri else 0
    if iso and len(mh) >= iso:
        i_ = mh[-iso:]
        avg_i = sum(i_) / len(i_) / 1e6
        print(f"\nMerkle hash launches of the isolated steps: {len(i_)} calls, trace average {avg_i:.4f} ms; bench "
              f"{ri['kernel_avg_ms']:.4f} ms ({(ri['kernel_avg_ms'] / avg_i - 1) * 100:+.1f}%)")
        print(f"isolated roofline frac from the trace: {frac_of(ri, avg_i):.4f}; bench frac {ri['frac']:.4f}")
    if len(mh) >= timed + iso:
        t = mh[len(mh) - iso - timed:len(mh) - iso]
        avg_ms = sum(t) / len(t) / 1e6
        print(f"\nMerkle hash launches of the in-flight steps (the timing pass after the timed region; before round 5 the timed steps): {len(t)} calls, trace average {avg_ms:.4f} ms; "
              f"bench kernel_avg_ms (HIP start/stop events per launch) {rf['kernel_avg_ms']:.4f} ms "
              f"({(rf['kernel_avg_ms'] / avg_ms - 1) * 100:+.1f}%), HIP-event span / launches "
              f"{rf.get('kernel_avg_ms_events', float('nan')):.4f} ms")
        print(f"roofline frac from the trace: {rf['perms_per_launch']:.0f} perms/launch x {rf['valu_ops_per_perm']} / "
              f"{avg_ms:.4f} ms / {rf['peak']:.1f} T = {frac_of(rf, avg_ms):.4f}; bench frac {rf['frac']:.4f}")
if b:
    print(f"\nbench (under profiler): value {b['value']:.4g} {b['unit']}, {b['ms_per_step']:.3f} ms per step, "
          f"kernel avg {b['roofline']['kernel_avg_ms']:.3f} ms\n")
if not iso_mode:
    print("## PMC (separate passes, per dispatch, averaged over dispatches of each kernel)\n")
    print("| kernel | counter | dispatches | mean per dispatch |")
    print("|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            print(f"| {k} | {c} | {len(v)} | {sum(v)/len(v):.6g} |")
