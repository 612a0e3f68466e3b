#!/usr/bin/env python3
"""bench.py — batched STARK verification on MI355X (BASELINE.json metric: STARK proofs verified/s
+ Tip5 permutations/s vs the VALU roofline).

Workload (default, BASELINE config 4, the north-star workload): 4,096 transaction proofs with log2
padded heights drawn uniformly (seed 0xC4) from the ProofCollection member mix {16, 10, 11, 12, 12,
11, 9, 9}, 1% with one flipped MainRows word (must reject), LPT-sharded over the ranks by estimated
Tip5 cost, Stark::default() parameters (security 160, expansion 4, 80 collinearity checks, 379 main /
88 aux columns, 4 quotient segments).  The proofs are the accepting synthetic proofs of
tests/golden/c3_pool.npz (made by tests/golden/make_bench_pool.py), each stored separately in HBM.

One step = whole verification of the rank's batch from its raw proof words in HBM: the proof-stream
decode on the device (k_decode: ProofStream::try_from + the dequeue order of Stark::verify, every
step again), Fiat-Shamir replay, row hashing, Merkle multiproofs, OOD AIR evaluation, FRI, DEEP, the
verdict copy back (nhip_batch_launch / nhip_batch_wait) and, for N > 1, the verdict exchange: configs
4 / 5 one all-gather per step of [batch verdict byte, per-proof verdict bytes] over the host (gloo:
the verdicts are host bytes; the batch verdict is the MIN of the leading bytes; block validation
needs every transaction's verdict: SURVEY.md §8e), posted without waiting and completed three steps
later, the last ones inside the timed region (shard.VerdictExchange); config 3 one all-reduce(MIN)
of the batch verdict per step.  After the timed region ONE RCCL all-reduce over xGMI carries the
job's verdict AND and the max over ranks of the region's time (an RCCL communicator alive during
the region costs a 512-proof rank ~6%: DESIGN.md §6).  Steps are pipelined as a node verifying a stream
of batches runs them (--inflight; 8 from 1,024 proofs per GPU, 10 below, 20 on one stream each up to
64 proofs): resident copies rotate, step k+1 is launched before step k is waited on, so one step's
latency-bound phases overlap the other's VALU-bound hashing; every timed step is launched and waited
inside the timed region.  The copies' streams need more than HIP's default 4 hardware queues per
process, so GPU_MAX_HW_QUEUES is raised here before HIP starts (to streams x in-flight + 2, at least
8, at most 22: past that a process collapses); the library's nhip_init provisions 8 when the
variable is unset.
The default timed region is 200 steps (~2 s of sustained load).

Defaults (round 4): the AIR is the synthetic constraints bloated to triton-air's size class
(--air triton-size, ~21.7k nodes: the OOD work timed is at least the reference's), and the proof /
claim words are given as twenty-first's in-memory Montgomery words (--input-form montgomery: the
form the Rust drop-in hands over without a copy; converted on the host before anything is timed).

Beside `value` (HBM-resident input, the contract):
  roofline: the dominant kernel, the per-level Merkle hash launches (k_mp_hash), as Tip5 VALU
    lane-ops/s against the gfx950 VALU peak, from its launches in steps run one at a time right
    after the timed region (the kernel's own rate: launches x average <= step time).
    roofline.inflight: the same launches in the timed region's shape (R steps in flight, up to 50
    steps) run again right after it, where launches of the steps in flight overlap each other and
    the other kernels (labelled, not the kernel's rate).  The kernel timing (per-dispatch begin / end
    timestamps, nhip_batch_set_launch_timing) is on in these two passes only: the timed region runs
    the product's configuration, without it (it costs a 512-proof share ~4.5%; the pass's own rate
    stands beside the timed region's in roofline.inflight).
  pcie_inclusive: the same batch arriving from host memory (pinned, DMA'd per refill, two batches
    alternating) with the host-to-device link's measured ceiling; never `value`.
  group_stream: the same batches through the in-process multi-GPU form neptune-core uses
    (nhip_group_stream over every GPU of the job from rank 0, from pinned host memory).
  tip5_paths: the config-2 Tip5 path microbench.
  cpu_baseline: the C restatement of the verifier (oracle/stark_oracle.c), one proof per host thread,
    over a bounded sample of this batch's proofs (the reference, Rust triton-vm, cannot be built here).
  hw_queues_4 (opt-in, --hwq4-steps): the same workload in a child process at HIP's default 4
    hardware queues (never under a profiler: the child would be started from a process whose GPU
    the profiler's library has already initialised).
  config1_latency: BASELINE config 1's single-proof latency (log2-21 substitute): GPU resident and
    from host memory, beside the C restatement on ONE host thread.
  roofline.traffic / valu_issue / hbm.pmc_*: from the committed rocprofv3 PMC passes of
    profiles/LATEST, attached only when profiles/<tag>/LIB_SHA256 is the hash of the library this run
    loaded; every fraction of a ceiling is asserted <= 1.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config {3,4,5}]
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
ISO_STEPS = 5
sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))

P = (1 << 64) - (1 << 32) + 1
POOL = os.path.join(ROOT, "tests", "golden", "c3_pool.npz")
COLLECTION_HEIGHTS = [16, 10, 11, 12, 12, 11, 9, 9]
# Algorithmic VALU work of one Tip5 permutation in 32-bit VALU lane-ops: a fixed analytic count of
# a minimal implementation: per round S-box 64 + x^7 672 + MDS 512+160 + ARK 96.
TIP5_VALU_OPS_PER_PERM = 5 * 1504
# VALU instructions a hash_pair permutation needs in the kernel's form (round 0 without the constant
# capacity's x^7 and MDS terms, the last round's 5 digest outputs only: DESIGN.md §3)
PAIR_HASH_VALU_OPS = 6070
# gfx950: 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz (wave64 VALU issues over 2 cycles on SIMD-32)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# MI355X_MICROARCH.md, HBM [CDNA4]: FETCH_SIZE is in KiB and on gfx950 counts half the bytes of a
# coalesced read (128-B requests tallied at 64 B): doubled; WRITE_SIZE reads true bytes
FETCH_CORRECTION = {"FETCH_SIZE": 2.0, "WRITE_SIZE": 1.0}


# the library neptune_hip loads (NHIP_LIB selects a variant for A/B runs): the one whose hash keys
# the committed profiles and is reported in config.lib_sha256
LIB_PATH = os.environ.get("NHIP_LIB") or os.path.join(ROOT, "neptune-core_amd", "neptune_hip", "libneptune_hip.so")


def lib_sha256(path: str = LIB_PATH) -> str:
    import hashlib
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


WORKLOAD = {"air": "triton-size", "input_form": "montgomery"}  # set by main() from the arguments


def latest_profile(config: int, proofs: int):
    """profiles/LATEST = '<tag> <config> <proofs per GPU> [<air> <input form>]': the committed
    rocprofv3 PMC passes and the workload they were taken on (none for another config, per-GPU batch
    size, AIR or input form: the PMC figures are per step of that workload; a line without the last
    two fields is the synthetic AIR, canonical input).  The passes count only for the library they
    were taken with: profiles/<tag>/LIB_SHA256 must equal the hash of the library this run loads,
    else the counters belong to another binary and are not attached."""
    try:
        parts = open(os.path.join(ROOT, "profiles", "LATEST")).read().split()
    except OSError:
        return None
    tag, cfg = parts[0], int(parts[1]) if len(parts) > 1 else 3
    n = int(parts[2]) if len(parts) > 2 else None
    air = parts[3] if len(parts) > 3 else "synthetic"
    form = parts[4] if len(parts) > 4 else "canonical"
    if cfg != config or n not in (None, proofs) or (air, form) != (WORKLOAD["air"], WORKLOAD["input_form"]):
        return None
    try:
        want = open(os.path.join(ROOT, "profiles", tag, "LIB_SHA256")).read().split()[0]
    except (OSError, IndexError):
        return None
    return tag if want == lib_sha256() else None


def pmc_traffic(kernel: str, config: int, proofs: int):
    """HBM bytes per launch of `kernel` from the latest committed rocprofv3 PMC passes
    (profiles/LATEST -> profiles/<tag>/pmc_{fetch,write}_counter_collection.csv), raw
    (FETCH_SIZE + WRITE_SIZE) x 1024; None when absent."""
    import csv
    tag = latest_profile(config, proofs)
    if tag is None:
        return None, None
    try:
        tot = 0.0
        for part, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            vals = [float(r["Counter_Value"]) for r in
                    csv.DictReader(open(os.path.join(ROOT, "profiles", tag, f"pmc_{part}_counter_collection.csv")))
                    if kernel in r["Kernel_Name"] and r["Counter_Name"] == ctr]
            tot += sum(vals) / len(vals) * 1024 * FETCH_CORRECTION.get(ctr, 1.0)
        return tot, tag
    except (OSError, ZeroDivisionError, KeyError):
        return None, None


def pmc_valu_per_step(config: int, proofs: int):
    """Wave-level VALU instructions one config-3 step issues, from the latest committed PMC pass
    (profiles/<LATEST>/pmc_valu_counter_collection.csv: SQ_INSTS_VALU summed over a step's
    dispatches, microbench kernels excluded; steps = k_hash_rows dispatches); None when absent."""
    import csv
    tag = latest_profile(config, proofs)
    if tag is None:
        return None, None
    try:
        tot, steps = 0.0, 0
        for r in csv.DictReader(open(os.path.join(ROOT, "profiles", tag, "pmc_valu_counter_collection.csv"))):
            k = r["Kernel_Name"]
            if r["Counter_Name"] != "SQ_INSTS_VALU" or "mtree" in k or "rocclr" in k:
                continue
            tot += float(r["Counter_Value"])
            steps += "k_hash_rows" in k
        return (tot / steps, tag) if steps else (None, None)
    except (OSError, KeyError):
        return None, None


def pmc_mp_valu_per_launch(config: int, proofs: int):
    """Wave-level VALU instructions of the Merkle level hash launches (k_mp_hash*, the roofline's
    kernel) per step, from the latest committed PMC pass; None when absent."""
    import csv
    tag = latest_profile(config, proofs)
    if tag is None:
        return None, None
    try:
        tot, steps = 0.0, 0
        for r in csv.DictReader(open(os.path.join(ROOT, "profiles", tag, "pmc_valu_counter_collection.csv"))):
            k = r["Kernel_Name"]
            if r["Counter_Name"] != "SQ_INSTS_VALU":
                continue
            if "k_mp_hash" in k or "k_mp_climb" in k:
                tot += float(r["Counter_Value"])
            steps += "k_hash_rows" in k
        return (tot / steps, tag) if steps else (None, None)
    except (OSError, KeyError):
        return None, None


def pmc_rows_valu_per_launch(config: int, proofs: int):
    """Wave-level VALU instructions of one row-hashing launch (k_hash_rows, one per step) from the
    latest committed PMC pass; None when absent."""
    import csv
    tag = latest_profile(config, proofs)
    if tag is None:
        return None, None
    try:
        tot, n = 0.0, 0
        for r in csv.DictReader(open(os.path.join(ROOT, "profiles", tag, "pmc_valu_counter_collection.csv"))):
            if r["Counter_Name"] == "SQ_INSTS_VALU" and "k_hash_rows" in r["Kernel_Name"]:
                tot += float(r["Counter_Value"])
                n += 1
        return (tot / n, tag) if n else (None, None)
    except (OSError, KeyError):
        return None, None


def under_profiler() -> bool:
    """rocprofv3 runs this process with its tool library preloaded (it initialises the GPU before
    bench.py starts): no child process may then be started from here."""
    pre = os.environ.get("LD_PRELOAD", "") + os.environ.get("HSA_TOOLS_LIB", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def pmc_bytes_per_step(config: int, proofs: int):
    """HBM bytes (raw FETCH_SIZE + WRITE_SIZE, x 1024) one config-3 step moves, summed over the step's
    dispatches in the latest committed PMC passes (microbench and runtime copy kernels excluded;
    steps = k_hash_rows dispatches); None when absent."""
    import csv
    tag = latest_profile(config, proofs)
    if tag is None:
        return None, None
    try:
        tot, steps = 0.0, 0
        for part, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            n_rows = 0
            for r in csv.DictReader(open(os.path.join(ROOT, "profiles", tag, f"pmc_{part}_counter_collection.csv"))):
                k = r["Kernel_Name"]
                if r["Counter_Name"] != ctr or "mtree" in k or "rocclr" in k:
                    continue
                tot += float(r["Counter_Value"]) * 1024 * FETCH_CORRECTION.get(ctr, 1.0)
                n_rows += "k_hash_rows" in k
            steps = n_rows
        return (tot / steps, tag) if steps else (None, None)
    except (OSError, KeyError):
        return None, None


def _assert_fracs(obj, path="res"):
    """Every fraction of a ceiling in the result line is <= 1: a larger one means mismatched inputs
    (counters of another binary, a wrong launch count), never a faster kernel."""
    if isinstance(obj, dict):
        for k, v in obj.items():
            if (k == "frac" or k.endswith("_frac")) and isinstance(v, (int, float)):
                assert 0.0 <= v <= 1.0, f"{path}.{k} = {v} is not a fraction of its ceiling"
            _assert_fracs(v, f"{path}.{k}")


HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md; 6.29 TB/s measured copy)

# measured gfx950 issue ceiling for this instruction mix: ~1 wave64 VALU instruction per 4 clocks
# per SIMD (tools/valu_microbench.hip)
VALU_ISSUE_CEILING = 256 * 4 * 2.4e9 / 4
# the fastest class measured (v_mov / v_add / logic: 1.4-1.7 wave64 instructions per CU-clock)
VALU_ISSUE_MAX = 256 * 1.7 * 2.4e9


# ------------------------------------------------------------------ config 3 batch
def load_pool():
    z = np.load(POOL)  # plain arrays, allow_pickle=False
    meta = json.loads(bytes(z["meta"]).decode())
    pool = {}
    for h in meta["heights"]:
        c = meta["claims"][str(h)]
        pool[h] = {"claim": (c["digest"], c["version"], c["input"], c["output"]),
                   "proof": z[f"proof_{h}"], "main_rows": meta["main_rows"][str(h)]}
    return z["air"], pool


def make_batch(pool, collections: int, corrupt_frac: float, seed: int):
    """(claims, proofs, expected verdicts): collections x 8 members, corrupt_frac of the collections
    with one flipped word in one member's MainRows payload."""
    rng = np.random.default_rng(seed)
    n_bad = int(round(collections * corrupt_frac))
    bad = set(rng.choice(collections, size=n_bad, replace=False).tolist()) if n_bad else set()
    claims, proofs, expect = [], [], []
    for c in range(collections):
        victim = int(rng.integers(0, len(COLLECTION_HEIGHTS))) if c in bad else -1
        for m, h in enumerate(COLLECTION_HEIGHTS):
            e = pool[h]
            proof = e["proof"]
            ok = True
            if m == victim:
                proof = proof.copy()
                lo, hi = e["main_rows"]
                pos = int(rng.integers(lo, hi))
                proof[pos] = np.uint64((int(proof[pos]) + 1) % P)
                ok = False
            claims.append(e["claim"])
            proofs.append(proof)
            expect.append(ok)
    return claims, proofs, np.array(expect, dtype=bool)


# exchanges posted before the oldest is completed (shard.VerdictExchange ring; 2 = complete the
# previous step's right after posting this one's)
EXCHANGE_DEPTH = 4


def kernel_timing(batches, on: bool = True):
    """Per-dispatch timestamps on the Merkle hash and row launches (nhip_batch_set_launch_timing),
    for the kernel-timing passes only: every batch runs without them otherwise, as the product's
    batches do (they cost a 512-proof share ~4.5% of its rate)."""
    for b in batches:
        if hasattr(b.ctx.lib, "nhip_batch_set_launch_timing"):  # older libraries (NHIP_LIB A/B) always time
            b.set_launch_timing(on)


def pipelined(batches, steps: int, inflight: int, expect):
    """`steps` launches over resident `batches` (round robin), at most `inflight` in flight, each
    wait followed at once by the next launch; returns (seconds, every verdict vector == expect)."""
    ok = True
    q, launched = [], 0
    t = time.perf_counter()
    for i in range(min(inflight, steps, len(batches))):
        batches[i].launch()
        q.append(i)
        launched += 1
    while q:
        i = q.pop(0)
        v, _ = batches[i].wait()
        if launched < steps:
            batches[i].launch()
            q.append(i)
            launched += 1
        ok = ok and bool((np.asarray(v, dtype=bool) == expect).all())
    return time.perf_counter() - t, ok


# resident one-stream batches (<= SINGLE_STREAM_MAX_PROOFS) replay their launches from a HIP graph
# (nhip_batch_set_graph): config 5's 64 / 8 proofs +3.5% / +5% at 20 in flight; a two-stream batch's
# graph measured slower (512 proofs -12%: profiles/r06/ab_graphs.txt), so those launch directly

# batches of at most this many proofs run every phase on one stream (nhip_batch_set_streams) at
# twice the depth: config 5's 8 / 64 proofs +17% / +13%; config 4's 512-4,096 lose 10-23% that way
# (profiles/r05z/ab/single_stream_ab_r05l.txt)
SINGLE_STREAM_MAX_PROOFS = 64


# targets the line reports itself against (`meets_target`): the N = 8 rank's 512-proof share of config 4
# at >= 0.92 of the 4,096-proof per-proof rate, config 5's 8-proof share at >= 40k proofs/s
SHARE_TARGET = 0.92
CONFIG5_SHARE_TARGET = 40000.0


def streams_for(n: int) -> int:
    return 1 if n <= SINGLE_STREAM_MAX_PROOFS else 2


def default_inflight(n: int, multi_rank: bool = False) -> int:
    """Steps in flight for an n-proof batch per GPU: 8 from 1,024 proofs, 10 below (9 for a rank
    whose per-step exchange runs on RCCL, NHIP_DIST_BACKEND=nccl: its process then also holds
    torch's and RCCL's streams during the timed region, see hw_queues_wanted; `multi_rank` means
    that case; the default host exchange holds none).
    The N = 1 / 2 / 4 / 8 shares of config 4; config 5's 8-64 proofs: 10 vs 8 in flight +10-11%,
    profiles/r03s.  Round 4, the driver's command (20 timed steps after 5 warm-up steps;
    `gpurun_out/ab_r04q`): 4,096 proofs 461.6-462.0k at 8 in flight vs 453.7-455.9k at 2; 512 proofs
    393.7-396.4k at 10, 367.6-377.9k at 6, 340.4-345.5k at 4; 200 steps: 4,096 at 8 461.5-463.7k vs
    450.1-451.6k at 2 (`ab_r04n`, `ab_r04o`).  (Before the library made a batch's streams, events
    and pinned readback at its preparation, a resident batch whose first launch fell inside the
    timed region stalled the others: with 5 warm-up steps, 512 proofs ran at 91-93k with 10 in
    flight.)  More in flight would need more than the 22 hardware queues below."""
    if n >= 1024:
        return 8
    if streams_for(n) == 1:  # one stream per batch: twice the depth in the same hardware queues
        return 18 if multi_rank else 20
    return 9 if multi_rank else 10


def hw_queues_wanted(inflight: int, multi_rank: bool, streams: int = 2) -> int:
    """GPU_MAX_HW_QUEUES for R steps in flight: R resident batches x 2 streams + the context stream
    need their own hardware queues (streams sharing a queue serialize; the GPU boxes export HIP's
    default of 4); with several ranks two more for torch's stream and RCCL's, so that no batch stream
    queues behind a collective waiting for the other ranks.  At least 8, at most 22: a process whose
    streams occupy more than ~22 hardware queues collapses (round 5, `profiles/r05z/ab/
    hw_queue_budget_r05.txt`: 11 steps in flight = 23 queues in use, 512 proofs 82k instead of
    406-416k; one rank of the multi-rank path at 512 proofs, 10 in flight with 24 queues 173-178k,
    22 queues 367-372k, 9 in flight 377-380k)."""
    return min(22, max(8, streams * inflight + 2 + (2 if multi_rank else 0)))


def load_pool4():
    """The 256 distinct accepting proofs config 4 draws from (oracle/pool4.py: the 5 committed full
    proofs of c3_pool.npz + 251 sparse-prover proofs, distinct claims and seeds, every one verified
    by both oracles, with its oracle transcript), built once per machine outside the timed region."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pool4  # test-data generator (proof construction only)
    return pool4.load()


def pool4_from_c3(pool):
    """A pool in load_pool4()'s form holding only the 5 committed c3 proofs (CPU tests: the real
    pool takes a minute of proving)."""
    hs = sorted(pool)
    return {"heights": hs, "proofs": [pool[h]["proof"] for h in hs], "claims": [pool[h]["claim"] for h in hs],
            "main_rows": [pool[h]["main_rows"] for h in hs]}


def make_config4(pool4, total: int, corrupt_frac: float, world: int, rank: int):
    """BASELINE config 4: `total` transaction proofs with log2 padded heights drawn uniformly from
    the ProofCollection member mix (seed 0xC4); the k-th proof of height h is distinct pool proof
    k mod (pool proofs of height h), so the 256 distinct proofs (oracle/pool4.py) each appear
    total / 256 times.  corrupt_frac of them get one flipped MainRows word.  LPT-sharded over the
    ranks by estimated Tip5 cost (neptune_hip.shard.lpt_shard).  Returns this rank's (claims,
    proofs, expect, pool index per proof), the shard assignment every rank agrees on, and the
    expected verdict of every proof of the job."""
    from neptune_hip import shard
    rng = np.random.default_rng(0xC4)
    hs = rng.choice(COLLECTION_HEIGHTS, size=total)
    bad = set(rng.choice(total, size=int(round(total * corrupt_frac)), replace=False).tolist())
    cost = [10_000 + 600 * int(h) for h in hs]  # ~ Tip5 permutations per proof of that height
    by_h = {}
    for j, h in enumerate(pool4["heights"]):
        by_h.setdefault(int(h), []).append(j)
    seen = {}
    src = []
    for i in range(total):
        h = int(hs[i])
        k = seen.get(h, 0)
        seen[h] = k + 1
        src.append(by_h[h][k % len(by_h[h])])
    mine = shard.lpt_shard(cost, world)[rank]
    claims, proofs, expect, srcs = [], [], [], []
    for i in mine:
        j = src[i]
        proof = pool4["proofs"][j]
        if i in bad:
            proof = proof.copy()
            lo, hi = pool4["main_rows"][j]
            pos = lo + (i * 7919) % (hi - lo)
            proof[pos] = np.uint64((int(proof[pos]) + 1) % P)
        claims.append(pool4["claims"][j])
        proofs.append(proof)
        expect.append(i not in bad)
        srcs.append(j)
    expect_all = np.array([i not in bad for i in range(total)], dtype=bool)
    return claims, proofs, np.array(expect, dtype=bool), srcs, shard.lpt_shard(cost, world), expect_all


def make_config5(air_words, total: int, log2_ph: int, world: int, rank: int):
    """BASELINE config 5: `total` proofs at log2 padded height `log2_ph` (seed 0xC5 + i; constant-
    codeword synthetic prover, oracle/stark_prover_const.py), contiguous shards over the ranks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import stark_prover_const as K  # test-data generator (proof construction only)
    import stark_ref as S
    import tip5_ref as T
    from neptune_hip import shard
    T.use_c_backend()
    params = S.StarkParams()
    _, recipe = S.synth_air(params, seed=1)
    air = S.AirCircuit.from_words([int(w) for w in air_words])
    claims, proofs = [], []
    for i in shard.contiguous_shard(total, world, rank):
        claim = ([0xC5, i, 0, 0, 0], 0, [i], [])
        proof, _ = K.prove(params, air, recipe, claim, log2_ph, seed=0xC5 + i)
        claims.append(claim)
        proofs.append(np.asarray(proof, dtype=np.uint64))
    shards = [list(shard.contiguous_shard(total, world, r)) for r in range(world)]
    return claims, proofs, np.ones(len(proofs), dtype=bool), shards, np.ones(total, dtype=bool)


# ------------------------------------------------------------------ CPU baseline (oracle)
def cpu_baseline(air_words, claims, proofs, expect, target_s: float, threads: int):
    """The C restatement of the verifier (oracle/stark_oracle.c), one proof per host thread, over a
    bounded prefix of the batch (whole collections, so the padded-height mix is the batch's)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as C  # oracle: CPU baseline leg only
    import stark_ref as S
    params = S.StarkParams()
    m0 = min(len(proofs), 8 * threads)
    a0 = C.stark_batch_args(air_words, params, claims[:m0], proofs[:m0])
    C.stark_verify_args(a0, threads)  # cold (thread heaps, clocks): untimed
    t = time.perf_counter()
    C.stark_verify_args(a0, threads)
    dt = time.perf_counter() - t
    m = min(len(proofs), max(m0, int(m0 * target_s / max(dt, 1e-6)) // 8 * 8))
    # whole passes over the sample until ~target_s (a 2,048-proof batch is ~1.5 s on 16 cores);
    # the proofs are marshaled into the C call's flat arrays once, outside the timed passes (as the
    # GPU's value starts with the proof words resident)
    passes = max(1, int(target_s / max(dt * m / m0, 1e-6)))
    am = C.stark_batch_args(air_words, params, claims[:m], proofs[:m])
    t = time.perf_counter()
    for _ in range(passes):
        v = C.stark_verify_args(am, threads)
        assert [bool(x) for x in v] == list(expect[:m]), "CPU baseline verdicts disagree with the expected verdicts"
    dt = time.perf_counter() - t
    return {"value": passes * m / dt, "unit": "proofs/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over the first {m} of this batch's {len(proofs)} proofs ({m // 8} whole "
                      f"collections), C restatement of the verifier (oracle/stark_oracle.c, Tip5 "
                      f"oracle/tip5_oracle.c), {threads} threads, {dt:.1f} s"}


# ------------------------------------------------------------------ config 1: single-proof latency
def config1_case(air_words):
    """BASELINE config 1 substitute (the reference's SingleProof is unavailable
    offline): one SingleProof-shaped proof at log2 padded height 21 (FRI domain 2^24, 15 FRI
    rounds), the claim of single_proof.rs:295-304 (input = a 5-word kernel MAST hash reversed,
    output empty; synthetic program digest, seed 0xC1).  tests/golden/config1.npz, made by the
    sparse synthetic prover (tests/golden/make_config1.py): every FRI codeword non-zero, a
    non-empty last polynomial (the constant-codeword proof used before folded zeros).  Returns
    (claim, proof, oracle samples, oracle FRI indices)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "config1.npz"))
    m = json.loads(bytes(z["meta"]).decode())
    claim = (m["digest"], m["version"], m["input"], m["output"])
    samples = [tuple(int(c) for c in x) for x in z["samples"]]
    return claim, np.asarray(z["proof"], dtype=np.uint64), samples, [int(i) for i in z["indices"]]


def config1_latency(ctx, gair, stark, air_words, cpu_seconds: float, reps: int = 50):
    """Single-proof latency on the config-1 substitute: the GPU (one proof resident in HBM, launch to
    verdict; and from host memory through nhip_verify_batch) beside the C restatement on ONE host
    thread (config 1's CPU baseline is the restatement, 1 thread).  Medians."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as C  # oracle: CPU baseline leg only
    import neptune_hip.stark as NS
    import stark_ref as S
    claim, proof, samples, indices = config1_case(air_words)
    dcl, dpr = device_form([claim], [proof], stark.input_form == 1)
    ncl, dproof = NS.Claim(*dcl[0]), dpr[0]
    b = NS.Batch(ctx, gair, stark, [ncl], [dproof])
    for _ in range(5):
        v, _ = b.run()
    xs, idx, fail = b.transcript(0)
    transcript_ok = fail == 0 and xs == samples and idx == indices
    res_ms = []
    for _ in range(reps):
        t = time.perf_counter()
        v, _ = b.run()
        res_ms.append((time.perf_counter() - t) * 1e3)
    ok = bool(v[0]) and transcript_ok
    b.close()
    host_ms = []
    for _ in range(max(5, reps // 5)):
        t = time.perf_counter()
        ok = NS.verify_batch(ctx, gair, stark, [(ncl, dproof)]) == [True] and ok
        host_ms.append((time.perf_counter() - t) * 1e3)
    args = C.stark_batch_args(air_words, S.StarkParams(), [claim], [proof])
    ok = bool(C.stark_verify_args(args, 1)[0]) and ok  # warm, and the oracle's verdict
    cpu_ms = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < cpu_seconds or len(cpu_ms) < 3:
        t = time.perf_counter()
        C.stark_verify_args(args, 1)
        cpu_ms.append((time.perf_counter() - t) * 1e3)
    gpu = float(np.median(res_ms))
    cpu = float(np.median(cpu_ms))
    return {"workload": "BASELINE config 1 substitute: one SingleProof-shaped proof, log2 padded height 21 "
                        "(FRI domain 2^24, 15 FRI rounds), seed 0xC1, Stark::default()",
            "proof": "tests/golden/config1.npz (sparse synthetic prover: non-zero FRI codewords, last polynomial "
                     "of degree 122)",
            "proof_words": int(proof.size), "verdict_accept": ok, "transcript_equals_oracle": transcript_ok,
            "gpu_resident_ms": gpu, "gpu_from_host_ms": float(np.median(host_ms)),
            "cpu_ms": cpu, "cpu_threads": 1, "cpu_kind": "port", "cpu_runs": len(cpu_ms),
            "gpu_speedup": cpu / gpu,
            "measured": f"medians: {reps} resident runs (launch to verdicts back), {len(host_ms)} nhip_verify_batch "
                        f"calls from host memory, {len(cpu_ms)} single-thread runs of the C restatement "
                        f"(oracle/stark_oracle.c)"}


def config5_leg(ctx, gair, stark, proofs_n: int = 64, steps: int = 200, inflight: int = None):
    """BASELINE config 5 beside the headline: `proofs_n` proofs at log2 padded height 23 (FRI domain
    2^26, 16 folding rounds) on one GPU.  The proof is tests/golden/deep_fri.npz's height-23 case
    (the sparse synthetic prover: every FRI codeword non-zero, a non-empty last polynomial), its
    words copied once per proof; `inflight` resident batches (default: the bench's depth for that
    batch size, 20 for <= 64 proofs on one stream each), `steps` steps after 3 warm-up steps (200: a
    stream of tiny batches in its steady state; 20 steps at 20 in flight would time one pipeline fill,
    the host enqueueing 20 batches back to back while the first ones run).
    Beside the rate: one batch alone (phase split; the sequential Fiat-Shamir sponge replay's share
    of that batch's device time) and proof 0's transcript against the oracle's, stored with the
    fixture."""
    import neptune_hip.stark as NS
    inflight = inflight or default_inflight(proofs_n)
    z = np.load(os.path.join(ROOT, "tests", "golden", "deep_fri.npz"))
    meta = json.loads(bytes(z["meta"]).decode())["cases"]["23"]
    claim = (meta["digest"], meta["version"], meta["input"], meta["output"])
    proof = z["proof_23"]
    samples = [tuple(int(c) for c in x) for x in z["samples_23"]]
    indices = [int(i) for i in z["indices_23"]]
    dcl, dpr = device_form([claim], [proof], stark.input_form == 1)
    ncl = [NS.Claim(*dcl[0])] * proofs_n
    prs = [np.array(dpr[0], dtype=np.uint64, copy=True) for _ in range(proofs_n)]
    nstreams = int(os.environ.get("NHIP_BENCH_C5_STREAMS", "0")) or streams_for(proofs_n)  # A/B: 2 = two streams
    ring = [NS.Batch(ctx, gair, stark, ncl, prs).set_streams(nstreams) for _ in range(inflight)]
    ok = True
    # alone: phase split (a direct launch) and the transcript; then every batch replays its graph
    v, _ = ring[0].run()
    alone = ring[0].stats()
    xs, idx, fail = ring[0].transcript(0)
    transcript_ok = fail == 0 and xs == samples and idx == indices
    ok = ok and bool(np.asarray(v, dtype=bool).all()) and transcript_ok
    for b in ring:
        b.set_graph(nstreams == 1)

    def region(k):
        nonlocal ok
        inflight_q = []
        for i in range(min(inflight, k)):
            ring[i].launch()
            inflight_q.append(i)
        launched = len(inflight_q)
        while inflight_q:
            i = inflight_q.pop(0)
            vv, _ = ring[i].wait()
            ok = ok and bool(np.asarray(vv, dtype=bool).all())
            if launched < k:
                ring[i].launch()
                inflight_q.append(i)
                launched += 1

    region(3)
    ctx.synchronize()
    t = time.perf_counter()
    region(steps)
    ctx.synchronize()
    dt = time.perf_counter() - t
    for b in ring:
        b.close()
    dev = max(alone["ms_device_total"], 1e-9)
    return {"workload": f"BASELINE config 5: {proofs_n} proofs at log2 padded height 23 (FRI domain 2^26, 16 FRI "
                        f"rounds), one GPU, Stark::default()",
            "proof": "tests/golden/deep_fri.npz height 23 (sparse synthetic prover: non-zero FRI codewords)",
            "proof_words": int(proof.size), "value": proofs_n * steps / dt, "unit": "proofs/s",
            "ms_per_step": dt / steps * 1e3, "steps": steps, "inflight": inflight,
            "streams_per_batch": nstreams,
            "alone_ms": {k[3:]: round(alone[k], 4) for k in ("ms_device_decode", "ms_fiat_shamir", "ms_row_hash",
                                                               "ms_merkle", "ms_ood_air", "ms_fri", "ms_deep",
                                                               "ms_device_total")},
            "sponge_replay_share": alone["ms_fiat_shamir"] / dev,
            "transcript_equals_oracle": transcript_ok, "verdicts_correct": ok}


def _pcts(ms):
    a = np.sort(np.asarray(ms, dtype=np.float64))
    if not a.size:
        return {}
    return {"p50": float(a[a.size // 2]), "p90": float(a[int(a.size * 0.9)]), "p99": float(a[int(a.size * 0.99)]),
            "max": float(a[-1])}


def queue_leg(ctx, gair, stark, claims, proofs, expect, callers: int = 64, rounds: int = 16,
              open_rates=(5000, 10000, 20000), open_seconds: float = 1.5):
    """The per-proof call of many concurrent tasks (verifier.rs:60-63 from peer_loop.rs:1342's
    mempool admission, one tokio task per peer transaction) through the coalescing queue
    (nhip_queue_verify), one proof per call:
      * closed loop: `callers` threads each verify one proof at a time, `rounds` calls each, beside
        the same calls serialized one proof per nhip_verify_batch;
      * open loop: Poisson arrivals at each of `open_rates` proofs/s for `open_seconds` (256 caller
        threads, each taking every 256th arrival at its scheduled time; a call that starts late counts
        its lateness as queueing delay), achieved rate and latency.
    Latency percentiles as the library measures them (nhip_queue_latencies: the caller's arrival in
    nhip_queue_verify -> its verdicts delivered) and, for the closed loop, also as this Python caller
    sees them (around the ctypes call: adds GIL hand-over, which the library's figure excludes)."""
    import threading
    import neptune_hip.stark as NS
    from neptune_hip.stark import _Marshal
    n = len(proofs)
    ncl = [NS.Claim(*c) for c in claims]
    NS.verify_batch(ctx, gair, stark, [(ncl[0], proofs[0])])
    m_ser = 32
    t = time.perf_counter()
    ser_ok = all(NS.verify_batch(ctx, gair, stark, [(ncl[i], proofs[i])])[0] == bool(expect[i]) for i in range(m_ser))
    rate_ser = m_ser / (time.perf_counter() - t)
    calls = [((j * 37) % n) for j in range(callers * rounds)]
    marsh = [_Marshal([ncl[i]], [proofs[i]]) for i in calls]
    lat = [0.0] * len(calls)
    ok = [True]
    old_switch = sys.getswitchinterval()
    sys.setswitchinterval(1e-4)  # 64-256 Python threads: hand the GIL over quickly after each C call
    try:
        with NS.Queue(ctx, gair, stark, max_wait_us=200) as q:
            q.verify(ncl[0], proofs[0])
            # warm-up burst: every caller once at the same time, so the queue's second batch slot and
            # its grown device buffers exist before the timed loop (a node's queue is warm after its
            # first few batches; allocating them synchronizes the device)
            warm = [threading.Thread(target=q.verify, args=(ncl[i % n], proofs[i % n])) for i in range(callers)]
            for th in warm:
                th.start()
            for th in warm:
                th.join()
            q.profile(reset=True)
            q.latencies_ms(reset=True)
            barrier = threading.Barrier(callers + 1)

            def worker(w):
                v = np.zeros(1, dtype=np.uint8)
                barrier.wait()
                for r in range(rounds):
                    j = w * rounds + r
                    mm = marsh[j]
                    t0 = time.perf_counter()
                    rc = ctx.lib.nhip_queue_verify(q.handle, mm.claims, mm.proofs, 1, v.ctypes.data)
                    lat[j] = time.perf_counter() - t0
                    if rc != 0 or bool(v[0]) != bool(expect[calls[j]]):
                        ok[0] = False

            ths = [threading.Thread(target=worker, args=(w,)) for w in range(callers)]
            for th in ths:
                th.start()
            barrier.wait()
            t = time.perf_counter()
            for th in ths:
                th.join()
            dt = time.perf_counter() - t
            prof = q.profile(reset=True)
            lib_lat = q.latencies_ms(reset=True)
            # open loop
            open_legs = []
            rng = np.random.default_rng(0x0E)
            workers = 256
            for rate in open_rates:
                k = max(workers, int(rate * open_seconds))
                arrivals = np.cumsum(rng.exponential(1.0 / rate, size=k))
                late = [0.0] * workers
                okw = [True] * workers
                bar = threading.Barrier(workers + 1)
                t_base = [0.0]

                def oworker(w, arrivals=arrivals, late=late, okw=okw, bar=bar, t_base=t_base):
                    v = np.zeros(1, dtype=np.uint8)
                    bar.wait()
                    for j in range(w, len(arrivals), workers):
                        due = t_base[0] + arrivals[j]
                        now = time.perf_counter()
                        if now < due:
                            time.sleep(due - now)
                        else:
                            late[w] = max(late[w], now - due)
                        mm = marsh[j % len(marsh)]
                        rc = ctx.lib.nhip_queue_verify(q.handle, mm.claims, mm.proofs, 1, v.ctypes.data)
                        if rc != 0 or bool(v[0]) != bool(expect[calls[j % len(marsh)]]):
                            okw[w] = False

                ths = [threading.Thread(target=oworker, args=(w,)) for w in range(workers)]
                for th in ths:
                    th.start()
                t_base[0] = time.perf_counter() + 0.01
                bar.wait()
                for th in ths:
                    th.join()
                span = time.perf_counter() - t_base[0]
                pr = q.profile(reset=True)
                ll = q.latencies_ms(reset=True)
                ok[0] = ok[0] and all(okw)
                open_legs.append({"offered": rate, "achieved": k / span, "proofs": k,
                                  "latency_ms": _pcts(ll), "max_start_lateness_ms": max(late) * 1e3,
                                  "proofs_per_batch": pr.get("proofs", 0) / max(pr.get("batches", 1), 1),
                                  "device_ms_per_batch": pr.get("ms_device", 0.0) / max(pr.get("batches", 1), 1),
                                  "window_ms_per_batch": pr.get("ms_window", 0.0) / max(pr.get("batches", 1), 1)})
    finally:
        sys.setswitchinterval(old_switch)
    nb = max(prof.get("batches", 1), 1)
    return {"callers": callers, "calls": len(calls), "value": len(calls) / dt, "unit": "proofs/s",
            "serialized_one_proof_calls": rate_ser, "vs_serialized": len(calls) / dt / rate_ser,
            "latency_ms": _pcts(lib_lat), "latency_ms_python_caller": _pcts(np.asarray(lat) * 1e3),
            # without each caller's first call (the 64 callers released at once by the barrier)
            "latency_ms_python_caller_after_first": _pcts(np.asarray([x for j, x in enumerate(lat) if j % rounds])
                                                          * 1e3),
            "proofs_per_batch": prof.get("proofs", 0) / nb, "batches": prof.get("batches", 0),
            "per_batch_ms": {k: prof.get(k, 0.0) / nb for k in ("ms_window", "ms_stage", "ms_upload", "ms_launch",
                                                                 "ms_device", "ms_wait", "ms_turnaround")},
            "open_loop": open_legs,
            "verdicts_correct": ok[0] and ser_ok,
            "measured": f"{callers} threads x {rounds} closed-loop nhip_queue_verify calls of one proof (max wait 200 us), "
                        f"beside {m_ser} one-proof nhip_verify_batch calls in a row; open loop: Poisson arrivals at "
                        f"{list(open_rates)} proofs/s for {open_seconds} s each; latency_ms from nhip_queue_latencies"}


# ------------------------------------------------------------------ config 2 Tip5 path microbench
def tip5_paths(ctx, log2_leaves: int, steps: int):
    """2^log2_leaves depth-log2_leaves Merkle authentication paths (pow.rs:162-180), 1% corrupted;
    Tip5 perms/s of k_mtree_verify and its VALU roofline fraction."""
    rng = np.random.default_rng(0xC2)
    n = 1 << log2_leaves
    depth = log2_leaves
    leafs = rng.integers(0, P, size=(n, 5), dtype=np.uint64)
    d_leafs = ctx.upload(leafs)
    d_nodes = ctx.alloc(n * 40)
    ctx.mtree_build_dev(d_leafs, n, d_nodes)
    nodes = d_nodes.download(np.uint64, (n, 5))
    idx = rng.permutation(n).astype(np.int64)
    paths = np.empty((n, depth, 5), dtype=np.uint64)
    paths[:, 0] = leafs[idx ^ 1]
    running = idx + n
    for k in range(1, depth):
        running >>= 1
        paths[:, k] = nodes[running ^ 1]
    elements = leafs[idx].copy()
    expect = np.ones(n, dtype=np.uint8)
    bad = rng.choice(n, size=n // 100, replace=False)
    elements[bad, 0] = (elements[bad, 0] + np.uint64(1)) % np.uint64(P)
    expect[bad] = 0
    d = {k: ctx.upload(v) for k, v in (("root", nodes[1]), ("idx", idx.astype(np.uint64)), ("el", elements),
                                       ("paths", paths))}
    d_v = ctx.alloc(n)
    ctx.mtree_verify_dev(d["root"], 1, d["idx"], d["el"], d["paths"], depth, n, d_v)
    ctx.synchronize()
    ctx.timing_read(reset=True)
    ctx.timing(True)
    for _ in range(steps):
        ctx.mtree_verify_dev(d["root"], 1, d["idx"], d["el"], d["paths"], depth, n, d_v)
    ctx.timing(False)
    ctx.synchronize()
    kern_ms, launches = ctx.timing_read(reset=True)
    ok = bool((d_v.download(np.uint8, (n,)) == expect).all())
    for b in list(d.values()) + [d_leafs, d_nodes, d_v]:
        b.free()
    avg_s = kern_ms / max(launches, 1) / 1e3
    perms_s = n * depth / avg_s
    return {"workload": f"BASELINE config 2: 2^{log2_leaves} depth-{depth} Merkle auth paths, 1% corrupted",
            "kernel": "k_mtree_verify", "kernel_avg_ms": avg_s * 1e3, "perms_per_s": perms_s,
            "valu_frac": perms_s * TIP5_VALU_OPS_PER_PERM / VALU_PEAK_LANE_OPS, "verdicts_correct": ok}


# ------------------------------------------------------------------ proofs arriving in host memory
def pcie_stream(ctx, gair, stark, claims, proofs, expect, batches: int, dist=None, total_proofs=None):
    """The PCIe-inclusive rate (never `value`): the same batch arriving from host memory, as a node
    receiving proofs would feed the verifier.  The proofs sit in pinned host memory on the GPU's NUMA
    node (nhip_host_alloc_near), so each refill is a DMA straight from it; two batches alternate
    refill / launch / wait, so each upload overlaps the other batch's device run.  Beside it the raw
    host-to-device rate of one copy of the same bytes: the link's measured ceiling.
    With several ranks (`dist`) every rank streams its own shard to its own GPU at the same time
    (each from memory on its GPU's node), between two barriers: the multi-process node rate over
    `total_proofs`, its time the slowest rank's; the raw ceiling is measured by all ranks at once."""
    import neptune_hip.stark as NS
    # With several ranks every barrier below is reached by every rank whatever happens on its own GPU:
    # a rank whose work raised skips the rest of its work (its error goes in the result) but still
    # meets the others at each barrier, so one rank's fault cannot leave the others waiting.
    st_ = {"err": None}

    def guarded(fn):
        if st_["err"] is None:
            try:
                fn()
            except Exception as e:  # noqa: BLE001 -- reported in the leg, never the headline
                st_["err"] = e

    def barrier():
        if dist is not None:
            dist.barrier()

    v_ = {}

    def setup():
        v_["pinned"] = NS.PinnedProofs(proofs, near=ctx)  # the receive path: pinned, on the GPU's NUMA node
        v_["ncl"] = [NS.Claim(*c) for c in claims]
        v_["nbytes"] = sum(len(p) for p in proofs) * 8
        ctx.synchronize()

    def raw_dma():  # raw DMA of the proof bytes, pinned -> device (best of 3)
        dbuf = ctx.alloc(v_["nbytes"])
        v_["raw"] = []
        for _ in range(3):
            t = time.perf_counter()
            dbuf.upload(v_["pinned"].flat)
            v_["raw"].append(v_["nbytes"] / (time.perf_counter() - t))
        dbuf.free()

    def prepare():
        v_["a"] = NS.Batch(ctx, gair, stark, v_["ncl"], v_["pinned"].views)
        v_["b"] = NS.Batch(ctx, gair, stark, v_["ncl"], v_["pinned"].views)
        v_["a"].run()
        # the C arrays, built once (a node's receive loop fills them in place)
        v_["m"] = NS.marshal(v_["ncl"], v_["pinned"].views)
        ctx.synchronize()

    def stream():
        ok = True
        cur, nxt = v_["a"], v_["b"]
        cur.refill(None, marshalled=v_["m"])
        cur.launch()
        for _ in range(batches - 1):
            nxt.refill(None, marshalled=v_["m"])
            v, _ = cur.wait()
            ok = ok and bool((np.asarray(v, dtype=bool) == expect).all())
            nxt.launch()
            cur, nxt = nxt, cur
        v, _ = cur.wait()
        v_["ok"] = ok and bool((np.asarray(v, dtype=bool) == expect).all())

    guarded(setup)
    barrier()
    guarded(raw_dma)
    guarded(prepare)
    barrier()
    t = time.perf_counter()
    guarded(stream)
    barrier()  # the slowest rank's end
    dt = time.perf_counter() - t
    st = {}

    def teardown():
        st.update(v_["a"].stats())

    guarded(teardown)
    for k in ("a", "b", "pinned"):
        if k in v_:
            try:
                v_[k].close()
            except Exception:  # noqa: BLE001
                pass
    if st_["err"] is not None:
        return {"error": repr(st_["err"])[:300], "verdicts_correct": None,
                "measured": "the leg raised on this rank (the headline is unaffected)"}
    nbytes = v_["nbytes"]
    h2d = nbytes * batches / dt
    peak = max(v_["raw"])
    return {"value": (total_proofs or len(proofs)) * batches / dt, "unit": "proofs/s", "batches": batches,
            "ranks": 1 if dist is None else dist.get_world_size(),
            "proof_bytes_per_batch": nbytes, "h2d_GBps": h2d / 1e9, "h2d_peak_GBps": peak / 1e9,
            "frac_of_h2d_peak": h2d / peak, "bound": "pcie (host-to-device DMA)",
            "refill_ms": {"host_stage": st["ms_decode"], "upload_wait": st["ms_upload"]},
            "verdicts_correct": v_["ok"],
            "measured": f"{batches} batches from pinned host memory on the GPU's node, 2 alternating (refill overlaps "
                        f"the other's run)" + ("" if dist is None else
                                               f"; every rank its own shard to its own GPU at once, h2d figures "
                                               f"rank 0's")}


def device_form(claims, proofs, mont: bool):
    """(claims, proofs) in the input form the library is given: unchanged, or as twenty-first's
    Montgomery words (each distinct proof array converted once: config 4 reuses 256 pool proofs)."""
    if not mont:
        return claims, proofs
    from neptune_hip.stark import to_montgomery
    seen = {}

    def conv(p):
        k = id(p)
        if k not in seen:
            seen[k] = (p, to_montgomery(p))
        return seen[k][1]

    def words(v):
        return [int(x) for x in to_montgomery(list(v))] if len(v) else []

    return [(words(c[0]), c[1], words(c[2]), words(c[3])) for c in claims], [conv(p) for p in proofs]


def group_stream(devices, air_words, stark, claims, proofs, expect, batches: int, pageable: bool = False):
    """The in-process multi-GPU form neptune-core runs: ONE process driving every GPU through
    nhip_group_stream (GpuNode::verify_stream in the Rust crate).  The job's whole batch is submitted
    `batches` times from host memory; each member's share of batch k is uploaded while its share of
    batch k - 1 runs, the members in parallel.  Two warm submissions first (each member's two device
    batches are allocated on first use).
    pageable=False: the proofs in per-member pinned arenas (nhip_arena_ingest_spans, once, outside
    the timed region: each proof in pinned memory on its member GPU's NUMA node, the members' shares
    adjacent), submitted with nhip_group_stream_submit_placed, so every member DMAs its own share as
    it lies (the verify_arenas form of the Rust crate).  pageable=True: every proof in its own
    ordinary allocation, as the Rust drop-in hands `proof.0.as_ptr()` of each `Vec` over
    (rust/neptune-hip/src/lib.rs marshal): the library copies the words into each member's pinned
    staging on copy threads bound to that GPU's NUMA node, then DMAs them."""
    import neptune_hip.stark as NS
    ncl = [NS.Claim(*c) for c in claims]
    gair = NS.Air([int(w) for w in air_words])
    want = [bool(x) for x in expect]
    ok = True
    nbytes = sum(len(p) for p in proofs) * 8
    arena = None
    with NS.Group(list(devices)) as g, NS.GroupStream(g, gair, stark) as st:
        if pageable:
            # distinct allocations: config 4 reuses 256 pool proofs, which would stay cache-resident
            src = [np.array(p, dtype=np.uint64, copy=True) for p in proofs]
            m = NS.marshal(ncl, src)

            def submit():
                return st.submit_marshalled(m)
        else:
            flat = np.concatenate([np.asarray(p, dtype=np.uint64) for p in proofs])
            offs = np.concatenate([[0], np.cumsum([len(p) for p in proofs])[:-1]]) * 8
            arena = NS.Arena(g, nbytes // len(devices) + (64 << 20))
            placed = arena.ingest_spans(flat.view(np.uint8), list(zip(offs.tolist(), [len(p) for p in proofs])))
            del flat
            cm = NS.marshal(ncl, [[] for _ in ncl])

            def submit():
                return st.submit_placed(cm, placed)
        for _ in range(2):
            submit()
        ok = st.finish()[0] == want
        st0 = st.stats()
        t = time.perf_counter()
        for _ in range(batches):
            r = submit()
            ok = ok and (r is None or r[0] == want)
        ok = ok and st.finish()[0] == want
        dt = time.perf_counter() - t
        st1 = st.stats()
        numa = g.numa()
        arenas = [arena.member_info(i) for i in range(len(devices))] if arena is not None else None
        if arena is not None:
            arena.close()
    d = {k: (st1[k] - st0[k]) / batches for k in ("ms_stage", "ms_upload", "ms_device")}
    out = {"value": len(proofs) * batches / dt, "unit": "proofs/s", "gpus": len(devices), "batches": batches,
           "proofs_per_batch": len(proofs), "h2d_GBps": nbytes * batches / dt / 1e9,
           "per_batch_ms": {"wall": dt / batches * 1e3, "stage_sum_members": d["ms_stage"],
                            "upload_wait_sum_members": d["ms_upload"], "device_sum_members": d["ms_device"]},
           "verdicts_correct": ok,
           "source": "pageable (one allocation per proof)" if pageable else
           "per-member pinned arenas on each GPU's NUMA node (nhip_arena, submit_placed)",
           "numa": [{"device": d["device"], "node": d["node"], "cpus": len(d["cpus"])} for d in numa],
           "numa_binding": os.environ.get("NHIP_NUMA", "1") != "0",
           "measured": f"{batches} submissions of the whole batch from "
                       f"{'pageable' if pageable else 'per-member pinned'} host memory through "
                       f"nhip_group_stream over devices {list(devices)} (one process)"}
    if arenas is not None:
        out["arena_pages_node"] = [a["page_node"] for a in arenas]
        out["arena_share_words"] = [a["used_words"] for a in arenas]
    return out


def tx_stream(proofs, seed: int = 0x7E):
    """The job's proofs as a peer would send them: back-to-back bincode TransferTransactions
    (protocol/peer/transfer_transaction.rs:31-47), each a synthetic TransactionKernel (one of 16,
    oracle/bincode_ref.py's encoder) and the SingleProof variant holding the proof's words as
    8-byte little-endian canonical values.  Test-data construction, outside every timed region."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import random
    import bincode_ref as B  # test-data encoder (the kernel bytes) only
    g = random.Random(seed)
    heads = []
    for _ in range(16):
        b = B.encode_transfer_transaction({"kernel": B.random_kernel(g, 1, 2, 1), "kind": B.TT_SINGLE_PROOF,
                                           "proof": []})
        heads.append(np.frombuffer(b[:-8], dtype=np.uint8))  # without the proof's length prefix
    sizes = [heads[i % 16].size + 8 + 8 * len(p) for i, p in enumerate(proofs)]
    buf = np.empty(sum(sizes), dtype=np.uint8)
    pos = 0
    for i, p in enumerate(proofs):
        h = heads[i % 16]
        buf[pos:pos + h.size] = h
        pos += h.size
        buf[pos:pos + 8] = np.frombuffer(np.uint64(len(p)).astype("<u8").tobytes(), dtype=np.uint8)
        pos += 8
        w = np.asarray(p, dtype="<u8").view(np.uint8)
        buf[pos:pos + w.size] = w
        pos += w.size
    return buf


def node_from_bytes(devices, air_words, claims, proofs, expect, batches: int, stream=None):
    """The whole node, bytes to verdicts: the job's proofs arrive as wire bytes (tx_stream: 4,096
    TransferTransactions in ordinary host memory), and each batch is decoded straight into
    per-member pinned arenas on the GPUs' NUMA nodes (nhip_arena_ingest_txs: scan, place on the
    least-loaded member, 8-byte LE words -> field elements with streaming stores on copy threads
    bound to that node) and submitted with nhip_group_stream_submit_placed (every member DMAs its
    share as it lies; its previous share's verdicts come back).  Two arena sets: a decode thread fills
    batch k + 1 while batch k uploads.  Decode, upload, device and verdicts are all inside the timed
    region; the claims are the bench's (synthetic proofs prove synthetic claims: a node derives a
    SingleProof claim from the kernel's MAST hash, verifier.single_proof_claim)."""
    import queue as pyqueue
    import threading
    import neptune_hip.stark as NS
    if stream is None:
        stream = tx_stream(proofs)
    ncl = [NS.Claim(*c) for c in claims]
    cm = NS.marshal(ncl, [[] for _ in ncl])
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()  # wire words are canonical values
    want = [bool(x) for x in expect]
    n = len(proofs)
    nbytes = sum(len(p) for p in proofs) * 8
    per_member = nbytes // len(devices) + max(len(p) for p in proofs) * 8 + (64 << 20)
    ok = [True]
    timing = {"decode_ms": [], "submit_ms": []}
    with NS.Group(list(devices)) as g, NS.GroupStream(g, gair, stark) as st:
        arenas = [NS.Arena(g, per_member), NS.Arena(g, per_member)]
        free = threading.Semaphore(2)
        ready = pyqueue.Queue()

        def decode(k):
            free.acquire()  # this set's previous batch has been submitted (its words are on the GPUs)
            a = arenas[k % 2]
            a.reset()
            t = time.perf_counter()
            pl, ntx, used = a.ingest_txs(stream, proof_cap=n)
            timing["decode_ms"].append((time.perf_counter() - t) * 1e3)
            if pl.n != n or ntx != n or used != stream.size:
                ok[0] = False
            return pl

        def producer(total):
            try:
                for k in range(total):
                    ready.put(decode(k))
            except Exception as e:  # noqa: BLE001 - surfaces on the consumer side
                ready.put(e)

        def run(total):
            th = threading.Thread(target=producer, args=(total,))
            th.start()
            for _ in range(total):
                pl = ready.get()
                if isinstance(pl, Exception):
                    raise pl
                t = time.perf_counter()
                r = st.submit_placed(cm, pl)
                timing["submit_ms"].append((time.perf_counter() - t) * 1e3)
                free.release()
                ok[0] = ok[0] and (r is None or r[0] == want)
            ok[0] = ok[0] and st.finish()[0] == want
            th.join()

        run(2)  # warm: device batches allocated, arena pages touched
        timing["decode_ms"].clear()
        timing["submit_ms"].clear()
        st0 = st.stats()
        t0 = time.perf_counter()
        run(batches)
        dt = time.perf_counter() - t0
        st1 = st.stats()
        pages = [arenas[0].member_info(i)["page_node"] for i in range(len(devices))]
        for a in arenas:
            a.close()
    d = {k: (st1[k] - st0[k]) / batches for k in ("ms_stage", "ms_upload", "ms_device")}
    return {"value": n * batches / dt, "unit": "proofs/s", "gpus": len(devices), "batches": batches,
            "proofs_per_batch": n, "wire_bytes_per_batch": int(stream.size), "proof_bytes_per_batch": nbytes,
            "h2d_GBps": nbytes * batches / dt / 1e9,
            "per_batch_ms": {"wall": dt / batches * 1e3, "decode": float(np.median(timing["decode_ms"])),
                             "submit": float(np.median(timing["submit_ms"])),
                             "upload_wait_sum_members": d["ms_upload"], "device_sum_members": d["ms_device"]},
            "arena_pages_node": pages, "verdicts_correct": ok[0],
            "path": "wire bytes (bincode TransferTransactions) -> nhip_arena_ingest_txs into per-member pinned "
                    "arenas -> nhip_group_stream_submit_placed -> verdicts",
            "measured": f"{batches} batches of {n} proofs, decode of batch k + 1 overlapping the upload of batch k "
                        f"(two arena sets), over devices {list(devices)} from one process"}


def launch_plan(gpus: int, env, argv, n_visible=None, port: int = 29500) -> dict:
    """How `bench.py --gpus N` runs (a pure function of its inputs; tests/test_bench_launch.py):
      * WORLD_SIZE set (the driver's `torch.distributed.run ... bench.py --gpus N`, or any launcher):
        this process is one rank; WORLD_SIZE must equal N, else an error (exit 2), so a run can never
        report a different GPU count than it was asked for;
      * N = 1 and no WORLD_SIZE: run here;
      * N > 1 and no WORLD_SIZE: relaunch as N ranks, one per GPU, under torch.distributed.run on this
        node (rendezvous on 127.0.0.1), with the same arguments; this process only waits for the
        child (nothing here has touched the GPU yet) and exits with its code.  N above the visible
        GPU count (n_visible, when known) is an error.
    Returns {"action": "run" | "relaunch" | "error", "world": N, "cmd": [...] (relaunch),
    "message": ... (error)}."""
    if gpus < 1:
        return {"action": "error", "world": gpus, "message": f"--gpus {gpus}: at least 1"}
    ws = env.get("WORLD_SIZE")
    if ws not in (None, ""):
        if int(ws) != gpus:
            return {"action": "error", "world": int(ws),
                    "message": f"WORLD_SIZE={ws} but --gpus {gpus}: launch one rank per GPU (--nproc-per-node {gpus})"}
        return {"action": "run", "world": gpus}
    if gpus == 1:
        return {"action": "run", "world": 1}
    if n_visible is not None and n_visible < gpus:
        return {"action": "error", "world": gpus, "message": f"--gpus {gpus} but {n_visible} GPU(s) visible"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return {"action": "relaunch", "world": gpus, "cmd": cmd}


def _visible_gpus():
    """GPUs this process could use, counted without initialising HIP (torch.cuda.device_count does
    not on this image); None when unknown."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return None


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default timed region: 200 config-4 steps, ~2 s of full VALU load (the clock settles under
    # sustained load on this power-bound integer pipeline)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=4, choices=(3, 4, 5),
                    help="4 (default, the north-star workload): 4,096 mixed transaction proofs over all ranks, "
                         "LPT-sharded, strong scaling; 3: 256 ProofCollections (2,048 proofs) per GPU, weak "
                         "scaling; 5: 64 proofs at log2 padded height 23 over all ranks, strong scaling")
    ap.add_argument("--proofs", type=int, default=None, help="config 4 / 5 total proofs (4096 / 64)")
    ap.add_argument("--log2-height", type=int, default=23, help="config 5 padded height")
    ap.add_argument("--collections", type=int, default=256)
    ap.add_argument("--corrupt-frac", type=float, default=0.05)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--air", default="triton-size", choices=("synthetic", "triton-size"),
                    help="AIR circuit: the same constraints bloated to triton-air's size class (default; ~21.7k "
                         "nodes, stark_ref.bloat_air: identically-zero extra terms, so the same proofs verify) or the "
                         "pool's synthetic AIR (505 constraints, 3,151 nodes)")
    ap.add_argument("--input-form", default="montgomery", choices=("montgomery", "canonical"),
                    help="how the proof / claim words reach the library: twenty-first's in-memory Montgomery "
                         "words (default: what the Rust drop-in hands over, Proof.0 as it lies) or canonical values")
    ap.add_argument("--group-batches", type=int, default=16,
                    help="group_stream leg: submissions of the job's batch through nhip_group_stream over every GPU "
                         "of the job from rank 0 (0 = skip)")
    ap.add_argument("--iso-steps", type=int, default=ISO_STEPS,
                    help="steps run one at a time after the timed region for roofline_isolated (0 = none: a "
                         "profiled run's kernel statistics then hold only in-flight steps)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--hwq4-steps", type=int, default=0,
                    help="N = 1, opt-in: also run the workload in a child process at HIP's default 4 hardware "
                         "queues (GPU_MAX_HW_QUEUES=4) and report it as hw_queues_4; never under a profiler")
    ap.add_argument("--config1-seconds", type=float, default=8.0,
                    help="config-1 single-proof latency leg: CPU-restatement time budget (0 = skip the leg)")
    ap.add_argument("--paths-log2", type=int, default=20, help="config-2 microbench size (0 = skip)")
    ap.add_argument("--product-steps", type=int, default=20,
                    help="steps of the product-depth leg (2 in flight) after the timed region (0 = skip)")
    ap.add_argument("--share-steps", type=int, default=100,
                    help="config 4 at N = 1: timed steps of the N = 8 rank's 512-proof share (0 = skip); 100: the "
                         "stream's steady state (at 20 steps the 10-deep pipeline's fill and drain are half the "
                         "region: profiles/r06/share_shapes_20steps.txt vs _100steps.txt)")
    ap.add_argument("--queue-callers", type=int, default=64,
                    help="queue leg at N = 1: concurrent single-proof callers through nhip_queue (0 = skip)")
    ap.add_argument("--no-rank-path", dest="rank_path", action="store_false",
                    help="skip share_n8.rank_path (the share size through the multi-rank path in a child)")
    ap.add_argument("--config5-inflight", type=int, default=None,
                    help="steps in flight of the config-5 leg (default: the bench's depth for its size)")
    ap.add_argument("--config5-proofs", type=int, default=64,
                    help="config-5 leg at N = 1: proofs at log2 padded height 23 (0 = skip)")
    ap.add_argument("--node-batches", type=int, default=32,
                    help="node leg (config 4): batches of wire bytes decoded into per-GPU pinned arenas and "
                         "verified through nhip_group_stream_submit_placed from rank 0 (0 = skip)")
    ap.add_argument("--stream-batches", type=int, default=6,
                    help="PCIe-inclusive leg: batches streamed from pinned host memory (0 = skip)")
    ap.add_argument("--shuffle", action="store_true",
                    help="config 4, one rank: verify the batch in a random order instead of the LPT order (heights "
                         "mixed within every wave: the order a node's batch arrives in)")
    ap.add_argument("--inflight", type=int, default=None, choices=tuple(range(1, 17)),
                    help="R > 1: R resident copies of the batch in rotation, up to R steps in flight (step k+1 is "
                         "launched before step k is waited on, so its row hashing fills step k's latency-bound "
                         "phases). Default: 2 for >= 4,096 proofs per GPU, 8 below (profiles/r03j)")
    args = ap.parse_args()

    plan = launch_plan(args.gpus, os.environ, sys.argv[1:],
                       n_visible=_visible_gpus() if args.gpus > 1 and not os.environ.get("WORLD_SIZE") else None,
                       port=_free_port())
    if plan["action"] == "error":
        log(f"bench.py: {plan['message']}")
        return 2
    if plan["action"] == "relaunch":
        import subprocess
        log(f"bench.py: {args.gpus} GPUs requested without a launcher: running {args.gpus} ranks under "
            f"torch.distributed.run")
        return subprocess.call(plan["cmd"])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    WORKLOAD.update(air=args.air, input_form=args.input_form)
    if under_profiler():
        args.hwq4_steps = 0  # no child process from a process the profiler has attached to the GPU
    air_words, pool = load_pool()
    sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
    shards = expect_all = None  # configs 4 / 5: per-proof verdicts are all-gathered every step
    if args.config == 3:
        claims, proofs, expect = make_batch(pool, args.collections, args.corrupt_frac, 0xC3 + rank)
        total = world * len(proofs)
    elif args.config == 4:
        total = args.proofs or 4096
        t = time.time()
        pool4 = load_pool4()
        log(f"[rank {rank}] config-4 pool: {len(pool4['proofs'])} distinct proofs ({time.time() - t:.1f}s)")
        air_words = pool4["air"]
        claims, proofs, expect, _, shards, expect_all = make_config4(pool4, total, 0.01, world, rank)
        if args.shuffle and world == 1:
            order = np.random.default_rng(0x5F).permutation(len(proofs))
            claims = [claims[i] for i in order]
            proofs = [proofs[i] for i in order]
            expect = expect[order]
    else:
        total = args.proofs or 64
        claims, proofs, expect, shards, expect_all = make_config5(air_words, total, args.log2_height, world, rank)
    if args.air == "triton-size":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import stark_ref as S  # AIR descriptor construction only (test-data generator)
        air_words = np.asarray(S.bloat_air(S.AirCircuit.from_words([int(w) for w in air_words]), 24000).to_words(),
                               dtype=np.uint64)
    n = len(proofs)
    # NHIP_BENCH_FORCE_DIST=1 (rehearsal on one GPU): one rank through the multi-rank path (process
    # group, per-step verdict exchange, its hardware-queue budget), as each rank of an N-GPU run
    multi = world > 1 or os.environ.get("NHIP_BENCH_FORCE_DIST") == "1"
    # torch's and RCCL's streams live in the process during the timed region only when the per-step
    # exchange runs on RCCL (NHIP_DIST_BACKEND=nccl); the default host exchange adds none
    gpu_exchange = multi and os.environ.get("NHIP_DIST_BACKEND", "gloo") == "nccl"
    R = args.inflight or default_inflight(n, gpu_exchange)
    # before anything initialises HIP (nothing above has)
    want_q = hw_queues_wanted(R, gpu_exchange, streams_for(n))
    if world == 1 and args.config == 4 and total == 4096 and args.share_steps > 0:
        # the share_n8 leg runs the N = 8 rank's 512-proof share at its own depth in this process
        want_q = max(want_q, hw_queues_wanted(default_inflight(total // 8), False))
    if world == 1 and args.config5_proofs > 0:  # the config-5 leg at its own depth
        want_q = max(want_q, hw_queues_wanted(default_inflight(args.config5_proofs), False,
                                              streams_for(args.config5_proofs)))
    if os.environ.get("NHIP_BENCH_HWQ"):  # A/B runs: exactly this many
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ["NHIP_BENCH_HWQ"]
    elif int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < want_q:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)
    hwq4 = None
    if world == 1 and args.hwq4_steps > 0 and not os.environ.get("NHIP_BENCH_HWQ"):
        # a child process, started before this one touches the GPU: the same workload with every
        # stream on HIP's default 4 hardware queues (the library's own provisioning is overridden)
        import subprocess
        cmd = [sys.executable, os.path.abspath(__file__), "--config", str(args.config), "--steps", str(args.hwq4_steps),
               "--warmup", str(min(args.warmup, 10)), "--no-cpu", "--paths-log2", "0", "--stream-batches", "0",
               "--config1-seconds", "0", "--iso-steps", "0", "--hwq4-steps", "0", "--air", args.air,
               "--input-form", args.input_form, "--group-batches", "0"]
        if args.proofs:
            cmd += ["--proofs", str(args.proofs)]
        if args.inflight:
            cmd += ["--inflight", str(args.inflight)]
        env = dict(os.environ, NHIP_BENCH_HWQ="4")
        t = time.time()
        out = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=600, check=True)
        h = json.loads(out.stdout.decode().strip().splitlines()[-1])
        hwq4 = {"value": h["value"], "ms_per_step": h["ms_per_step"], "steps": h["steps"],
                "gpu_max_hw_queues": h["config"]["gpu_max_hw_queues"], "verdicts_correct": h["verdicts_correct"],
                "measured": "child process before this one initialised HIP, same workload, NHIP_BENCH_HWQ=4"}
        log(f"[hwq4] {h['value']:.0f} proofs/s at 4 hardware queues ({time.time() - t:.1f}s)")
    rank_path = None
    if (world == 1 and args.config == 4 and total == 4096 and args.share_steps > 0 and args.rank_path
            and not os.environ.get("NHIP_BENCH_FORCE_DIST")):
        # the N = 8 rank's share size through the multi-rank path itself (process group, host
        # exchange, one RCCL all-reduce after the region) at world size 1: a child under
        # torch.distributed.run, started before this process touches the GPU
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
               "--gpus", "1", "--proofs", str(total // 8), "--steps", str(args.share_steps), "--warmup",
               str(args.warmup), "--no-cpu", "--paths-log2", "0", "--stream-batches", "0", "--group-batches", "0",
               "--config1-seconds", "0", "--product-steps", "0", "--share-steps", "0", "--queue-callers", "0",
               "--config5-proofs", "0", "--air", args.air, "--input-form", args.input_form]
        t = time.time()
        try:
            out = subprocess.run(cmd, env=dict(os.environ, NHIP_BENCH_FORCE_DIST="1"), stdout=subprocess.PIPE,
                                 stderr=subprocess.DEVNULL, timeout=600, check=True)
            h = json.loads(out.stdout.decode().strip().splitlines()[-1])
            rank_path = {"value": h["value"], "ms_per_step": h["ms_per_step"], "steps": h["steps"],
                         "inflight": h["inflight"], "verdicts_correct": h["verdicts_correct"],
                         "verdict_exchange": h["config"].get("verdict_exchange"),
                         "measured": f"a {total // 8}-proof config-4 job (the N = 8 rank's share size) in a child "
                                     "under torch.distributed.run at world size 1 with NHIP_BENCH_FORCE_DIST=1: "
                                     "the rank's process group, per-step exchange and final all-reduce"}
            log(f"[rank path] {h['value']:.0f} proofs/s ({time.time() - t:.1f}s)")
        except (subprocess.SubprocessError, ValueError, KeyError, IndexError) as e:
            rank_path = {"error": f"{type(e).__name__}: {e}"[:300]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        t = time.time()
        cpu = cpu_baseline(air_words, claims, proofs, expect, args.cpu_seconds, args.cpu_threads)
        log(f"[cpu] {cpu['value']:.1f} proofs/s ({time.time() - t:.1f}s)")

    dist = None
    dev_index = local_rank
    gpu_shared = False  # several ranks on one GPU (the gloo rehearsals)
    if multi:
        import torch
        import torch.distributed as dist
        # The per-step verdict exchange runs on the host (gloo): the verdicts are host bytes after
        # every step's wait, and an RCCL communicator alive in the process costs a 512-proof rank ~6%
        # of its rate with no collective running.  The job's verdict AND (with the
        # timing's max over ranks) is ONE RCCL all-reduce over xGMI after the timed region, on a group
        # made there.  NHIP_DIST_BACKEND=nccl runs the per-step exchange on RCCL device buffers
        # instead; NHIP_FINAL_BACKEND=gloo keeps the final all-reduce on the host (several ranks on
        # one GPU: RCCL refuses two ranks on one device).
        backend = os.environ.get("NHIP_DIST_BACKEND", "gloo")
        final_backend = os.environ.get("NHIP_FINAL_BACKEND", "nccl")
        if backend != "nccl" and final_backend != "nccl":
            dev_index = local_rank % max(1, torch.cuda.device_count())
            gpu_shared = world > max(1, torch.cuda.device_count())
        if os.environ.get("NHIP_BENCH_NO_SET_DEVICE") != "1":  # A/B only (one rank, host collectives only)
            torch.cuda.set_device(dev_index)
        if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
            # one node: gloo over the loopback device (the container's hostname may not resolve)
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        dist.init_process_group(backend)
        flags = ctypes.c_uint(0)
        try:
            ctypes.CDLL("libamdhip64.so").hipGetDeviceFlags(ctypes.byref(flags))
        except OSError:
            pass
        log(f"[rank {rank}] {backend} process group: {len(os.sched_getaffinity(0))} CPUs in affinity, "
            f"{len(os.listdir('/proc/self/task'))} threads, HIP device flags {flags.value:#x}, "
            f"env {sorted(k for k in os.environ if k.startswith(('HIP_', 'HSA_', 'GPU_', 'AMD_', 'ROC')))}")
    import neptune_hip as nh
    import neptune_hip.stark as NS
    from neptune_hip import shard

    mont = args.input_form == "montgomery"
    # the words as the library gets them: a node holds its proofs as Vec<BFieldElement>, i.e. in
    # Montgomery form already, so the conversion of these canonical test proofs is data preparation
    dev_claims, dev_proofs = device_form(claims, proofs, mont)
    ctx = nh.Context(dev_index)
    t0 = time.time()
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default().montgomery() if mont else NS.Stark.default()
    ncl = [NS.Claim(*c) for c in dev_claims]
    # R resident copies of the raw proof words (each step decodes them on the device again)
    # resident one-stream batches (<= 64 proofs per GPU) replay a captured HIP graph
    ring = [NS.Batch(ctx, gair, stark, ncl, dev_proofs).set_streams(streams_for(n)).set_graph(streams_for(n) == 1)
            for _ in range(R)]
    prep_s = time.time() - t0
    st0 = ring[0].stats()
    log(f"[rank {rank}] batch ready: {n} proofs x {R} resident copies, {st0['proof_words']} words, "
        f"prepare {prep_s:.2f}s (host stage {st0['ms_decode']:.0f} ms, upload wait {st0['ms_upload']:.0f} ms)")

    launched = []   # ring slots in flight, oldest first
    next_slot = [0]
    to_launch = [0]  # launches left in the current region: each region starts and ends with nothing in flight
    # configs 4 / 5 with several ranks: one all-gather per step carries every rank's batch verdict
    # and per-proof verdicts (shard.VerdictExchange), posted without waiting and completed one step
    # later; config 3 (no per-proof exchange): the all-reduce(MIN) of the batch verdict
    exch = (shard.VerdictExchange(shards, total, dist, depth=EXCHANGE_DEPTH)
            if (dist is not None and shards is not None) else None)
    no_exchange = os.environ.get("NHIP_BENCH_NO_EXCHANGE", "0")  # A/B only (one rank): 1 = all_ok per step, 2 = nothing
    if no_exchange != "0":
        exch = None
    exchanged = []  # (batch verdict, job verdict vector) of every completed exchange

    # NHIP_BENCH_TIMELINE=<file>: host times of every launch and wait return of the timed region
    # (a diagnostic of the pipeline's fill and drain; the kernel tracer stretches small steps)
    timeline = [] if os.environ.get("NHIP_BENCH_TIMELINE") else None

    def launch_one():
        ring[next_slot[0]].launch()
        if timeline is not None:
            timeline.append(("L", time.perf_counter()))
        launched.append(next_slot[0])
        next_slot[0] = (next_slot[0] + 1) % R
        to_launch[0] -= 1

    def step():
        # keep up to R steps in flight (one per resident copy); wait for the oldest, take its
        # verdicts and stats, and relaunch its slot at once (before any bookkeeping) so the GPU
        # never waits on the host between steps
        while to_launch[0] and len(launched) < R:
            launch_one()
        b = ring[launched.pop(0)]
        v, ok = b.wait()
        if timeline is not None:
            timeline.append(("W", time.perf_counter()))
        st = b.stats()
        if to_launch[0]:
            launch_one()
        if exch is not None:  # block validation: every rank gets every proof's verdict
            exch.post(ok, v)
            if len(exch.pending) >= exch.depth:  # complete step k - depth + 1
                exchanged.append(exch.complete())
        elif dist is not None and no_exchange != "2":
            ok = shard.all_ok(ok, dist)  # all-reduce(MIN) of the batch verdict
        return st, v, ok

    def drain_exchange():
        while exch is not None and exch.pending:
            exchanged.append(exch.complete())

    def barrier_sync():
        ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            if os.environ.get("NHIP_BENCH_NO_BARRIER") != "1":  # A/B only (one rank): no collective before the region
                dist.barrier()

    # NHIP_BENCH_REGION_TIMING=1 (A/B of their cost): the timed region and the share leg with the
    # per-dispatch timestamps on, as bench.py ran them before round 5
    region_timing = os.environ.get("NHIP_BENCH_REGION_TIMING", "0") == "1"
    kernel_timing(ring, region_timing)
    to_launch[0] = args.warmup
    for _ in range(args.warmup):
        step()
    drain_exchange()
    exchanged.clear()
    barrier_sync()
    acc = {}
    batch_ok = None
    correct = True
    t_start = time.perf_counter()
    to_launch[0] = args.steps  # every timed step is launched and waited inside the timed region
    if timeline is not None:
        timeline.clear()
    for _ in range(args.steps):
        st, v, batch_ok = step()
        correct = correct and bool((np.asarray(v, dtype=bool) == expect).all())
        for k, x in st.items():
            acc[k] = acc.get(k, 0.0) + x
    drain_exchange()  # the last step's exchange completes inside the timed region
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    if timeline is not None and rank == 0:
        with open(os.environ["NHIP_BENCH_TIMELINE"], "w") as f:
            json.dump({"t_start": t_start, "elapsed": elapsed, "inflight": R,
                       "events": [(k, t - t_start) for k, t in timeline]}, f)
    if exch is not None:
        correct = correct and len(exchanged) == args.steps
        for ok_all, full in exchanged:
            correct = correct and bool((full.astype(bool) == expect_all).all())
            batch_ok = ok_all
    # the kernel-timing passes, right after the timed region (which ran the product's configuration,
    # without per-dispatch timestamps): the same R-in-flight shape again with them
    # (roofline.inflight), then the same steps one at a time (roofline, the kernel's own rate)
    kernel_timing(ring, True)
    acc_if, if_steps = {}, max(1, min(args.steps, 50))
    ctx.synchronize()
    t_if = time.perf_counter()
    q_if, launched_if, ok_if = [], 0, True
    for i in range(min(R, if_steps)):
        ring[i].launch()
        q_if.append(i)
        launched_if += 1
    while q_if:
        i = q_if.pop(0)
        v_if, _ = ring[i].wait()
        for k, x in ring[i].stats().items():  # before the relaunch re-records the events
            acc_if[k] = acc_if.get(k, 0.0) + x
        if launched_if < if_steps:
            ring[i].launch()
            q_if.append(i)
            launched_if += 1
        ok_if = ok_if and bool((np.asarray(v_if, dtype=bool) == expect).all())
    if_ms = (time.perf_counter() - t_if) / if_steps * 1e3
    correct = correct and ok_if
    acc_iso, iso_ms = {}, 0.0
    iso_steps = args.iso_steps
    if R > 1 and iso_steps:
        t_iso = time.perf_counter()
        for _ in range(iso_steps):
            ring[0].launch()
            ring[0].wait()
            for k, x in ring[0].stats().items():
                acc_iso[k] = acc_iso.get(k, 0.0) + x
        iso_ms = (time.perf_counter() - t_iso) / iso_steps * 1e3
    kernel_timing(ring, False)

    # the product's own pipeline depth beside the bench's: a queue or a group member keeps two
    # batches in flight (two slots), with the library's recommended hardware queues enough for it
    product = None
    if world == 1 and R > 2 and args.product_steps > 0:
        ctx.synchronize()
        dt, ok2 = pipelined(ring, args.product_steps, 2, expect)
        product = {"value": total * args.product_steps / dt, "unit": "proofs/s", "inflight": 2,
                   "steps": args.product_steps, "ms_per_step": dt / args.product_steps * 1e3, "verdicts_correct": ok2,
                   "measured": "the same resident batches, 2 in flight (nhip_queue / nhip_group_stream keep two "
                               "slots per GPU), right after the timed region"}
        correct = correct and ok2

    if dist is not None:
        import torch
        # ONE all-reduce(MAX) over [elapsed, any rank wrong, NOT the job's verdict] = the max over
        # ranks of the timed region and the job's logical AND: RCCL over xGMI (a group made here,
        # after every timed region of the run), or on the exchange's group when that is RCCL already.
        # shard.agreed_max: every rank tries the RCCL all-reduce (synchronized inside the try), then
        # the ranks agree over the host group whether all of them got it; if any failed, all reduce on
        # the host group, so one rank's RCCL fault never leaves the ranks in different collectives.
        vals = [elapsed, 0.0 if correct else 1.0, 0.0 if batch_ok else 1.0]
        final_error, fast_used = None, False
        if final_backend == "nccl" and backend != "nccl":
            import datetime

            def rccl_max(v):
                grp = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=120))
                t = torch.tensor(v, dtype=torch.float64, device=torch.device("cuda", dev_index))
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)
                return t.cpu().tolist()  # synchronizes: a device-side fault raises here, inside the try

            vals, fast_used, final_error = shard.agreed_max(vals, dist, rccl_max)
            if final_error:
                log(f"[rank {rank}] RCCL all-reduce failed ({final_error}); every rank reduced on the host group")
        else:
            t = torch.tensor(vals, dtype=torch.float64, device=shard._device_for(dist))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            vals = t.cpu().tolist()
            fast_used = dist.get_backend() == "nccl"
        elapsed, any_bad, not_ok = float(vals[0]), float(vals[1]), float(vals[2])
        correct = any_bad == 0.0
        batch_ok = not_ok == 0.0
        final_collective = {"backend": "nccl" if fast_used else dist.get_backend(),
                            "op": "all_reduce(MAX) of [elapsed, any rank wrong, NOT job verdict]",
                            "fallback": "agreed over the host group (shard.agreed_max)"}
        if final_error:
            final_collective["rccl_error"] = final_error
    perms_rank = (acc.get("tip5_perms_static", 0.0) + acc.get("tip5_perms_merkle", 0.0)) / max(args.steps, 1)
    perms_job = perms_rank
    if dist is not None:
        import torch
        tp = torch.tensor([perms_rank], dtype=torch.float64, device=shard._device_for(dist))
        dist.all_reduce(tp, op=dist.ReduceOp.SUM)
        perms_job = float(tp[0].item())
    if not correct:
        log("ERROR: verdicts differ from expected")
    K = args.steps
    avg = {k: v / K for k, v in acc.items()}
    perms = avg["tip5_perms_static"] + avg["tip5_perms_merkle"]
    step_ms = elapsed / K * 1e3

    # roofline of the dominant kernel, the Merkle hash launches (k_mp_hash, + k_mp_hash_wide /
    # k_mp_hash_tail on the smallest levels): permutations per launch x the analytic VALU lane-ops per
    # permutation / the average launch duration.  Each launch is timed by the HIP start / stop events
    # of hipExtLaunchKernel on its stream (the dispatch's own begin / end timestamps, what the
    # rocprofv3 kernel trace reports per dispatch).  `roofline`: the launches of ISO_STEPS steps run
    # one at a time right after the timed region (the kernel's own rate; launches x average <= that
    # step time <= ms_per_step, asserted).  `roofline.inflight`: the same launches inside the timed
    # region, where R steps are in flight, so launches of different steps overlap each other and the
    # other kernels (launches x average <= R x step time only): how the level launches share the
    # machine, not the kernel's rate.  kernel_avg_ms_events: the HIP-event span of one step's
    # back-to-back hash launches / launches (adds the dispatch gaps between levels).
    traffic, traffic_tag = pmc_traffic("k_mp_hash", args.config, len(proofs))
    mp_valu, mp_valu_tag = pmc_mp_valu_per_launch(args.config, len(proofs))

    def roofline(a, steps, step_ms_, overlap, measured):
        a = {k: v / steps for k, v in a.items()}
        launches = max(a["mp_hash_kernel_launches"], 1.0)
        kern_avg_s = a["ms_mp_hash_exec"] / launches / 1e3
        kern_avg_ev_s = a["ms_mp_hash_kernel"] / launches / 1e3
        perms_per_launch = a["mp_hash_kernel_perms"] / launches
        achieved = perms_per_launch * TIP5_VALU_OPS_PER_PERM / kern_avg_s if kern_avg_s > 0 else 0.0
        assert launches * kern_avg_s * 1e3 <= overlap * step_ms_ * 1.0001, (launches, kern_avg_s, step_ms_, overlap)
        r = {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12,
             "unit": "T VALU lane-ops/s", "frac": achieved / VALU_PEAK_LANE_OPS, "traffic": traffic,
             "traffic_unit": "HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B; MI355X_MICROARCH.md HBM corrections)",
             "traffic_profile": traffic_tag,
             "kernel": "k_mp_hash (+ k_mp_hash_wide / k_mp_hash_tail on the smallest levels)",
             "kernel_avg_ms": kern_avg_s * 1e3, "kernel_avg_ms_events": kern_avg_ev_s * 1e3,
             "launches_per_step": launches, "launches_x_avg_ms": launches * kern_avg_s * 1e3,
             "perms_per_launch": perms_per_launch, "valu_ops_per_perm": TIP5_VALU_OPS_PER_PERM,
             "step_ms": step_ms_,
             # the same launches counted with the ~6,070 VALU a pair hash needs (the kernel skips
             # hash_pair's constant capacity and dead last-round outputs)
             "pair_hash_valu_ops_per_perm": PAIR_HASH_VALU_OPS,
             "frac_pair_hash_ops": achieved * PAIR_HASH_VALU_OPS / TIP5_VALU_OPS_PER_PERM / VALU_PEAK_LANE_OPS,
             # beside the spec peak: the measured integer issue ceiling (1 wave64 instruction
             # per 4 clocks per SIMD = 64 lane-ops per instruction), DESIGN.md §3
             "measured_ceiling": VALU_ISSUE_CEILING * 64 / 1e12,
             "frac_of_measured_ceiling": achieved / (VALU_ISSUE_CEILING * 64),
             "measured": measured}
        if mp_valu:
            # executed lane-instructions per permutation (committed PMC pass of this library:
            # SQ_INSTS_VALU of the step's hash launches x 64 / the step's Merkle permutations)
            ex = mp_valu * 64 / max(a["mp_hash_kernel_perms"], 1.0)
            r.update({"valu_ops_per_perm_executed": ex, "executed_profile": mp_valu_tag,
                      "frac_executed": perms_per_launch * ex / kern_avg_s / VALU_PEAK_LANE_OPS,
                      "frac_pair_hash_need_of_executed": PAIR_HASH_VALU_OPS / ex})
        return r

    if args.config == 3:
        workload = (f"BASELINE config 3: {args.collections} ProofCollections x 8 proofs (log2 padded heights "
                    f"{COLLECTION_HEIGHTS}) = {n} STARK verifications per GPU, Stark::default()")
    elif args.config == 4:
        workload = (f"BASELINE config 4: {total} transaction proofs (log2 padded heights drawn from "
                    f"{COLLECTION_HEIGHTS}, 1% corrupted), LPT-sharded over {world} GPU(s), Stark::default()"
                    + (", verified in a random order" if args.shuffle and world == 1 else ""))
    else:
        workload = (f"BASELINE config 5: {total} proofs at log2 padded height {args.log2_height} (FRI domain "
                    f"2^{args.log2_height + 3}), sharded over {world} GPU(s), Stark::default()")
    res = {
        "metric": "STARK proofs verified/sec (whole node) + Tip5 perms/sec vs VALU roofline",
        "value": total * K / elapsed,
        "unit": "proofs/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "weak" if args.config == 3 else "strong",
        "vs_baseline": None,
        "dtype": "u64 (Goldilocks mod p; XFE = cubic extension)",
        "data": ("synthetic: one accepting proof per padded height (tests/golden/c3_pool.npz, synthetic AIR with "
                 "triton-vm column counts), 5% of collections with one flipped MainRows word" if args.config == 3 else
                 "synthetic: 256 distinct accepting proofs (oracle/pool4.py: the 5 full proofs of "
                 "tests/golden/c3_pool.npz + 251 sparse-prover proofs, distinct claims and seeds), each used "
                 f"{total // 256 if total >= 256 else 1}x, 1% with one flipped MainRows word"
                 if args.config == 4 else
                 "synthetic: constant-codeword proofs (oracle/stark_prover_const.py), synthetic AIR with triton-vm "
                 "column counts"),
        "config": {"workload": workload, "proofs_total": total, "proofs_rank0": n,
                   "parallelism": f"proof-sharded x{world}", "air": args.air, "input_form": args.input_form,
                   # value's input: the raw proof words already in HBM when the timed region starts;
                   # the host-memory (PCIe-inclusive) rate is pcie_inclusive, never value
                   "input": "HBM-resident raw proof words (uploaded before the timed region; decoded on the "
                            "device every step)",
                   "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   "lib_sha256": lib_sha256()[:16],
                   "verdict_exchange": (None if dist is None else
                                        {"per_step": f"{dist.get_backend()} all-gather of [batch verdict, "
                                                     f"per-proof verdicts] (shard.VerdictExchange, "
                                                     f"{EXCHANGE_DEPTH} deep)",
                                         "final": final_collective})},
        # what one step is: the raw proof words are resident in HBM when the step starts; the step
        # decodes every proof stream on the device (k_decode) and runs every verifier phase
        "step": "device proof-stream decode + Fiat-Shamir replay + row hashing + Merkle multiproofs + OOD AIR + "
                "FRI + DEEP + verdicts back to the host",
        "verdicts_correct": correct,
        "batch_verdict": batch_ok,
        "expected_rejects_rank0": int((~expect).sum()),
        "tip5_perms_per_proof": perms / n,
        "tip5_perms_per_s": perms_job * K / elapsed,
        # BASELINE's second metric at the pipeline level: every Tip5 permutation of the step (sponge
        # replay, rows, Merkle levels) x the analytic VALU lane-ops per permutation, per second of
        # wall time, against the VALU peak
        "tip5_valu_frac": perms_job * K / elapsed * TIP5_VALU_OPS_PER_PERM / (VALU_PEAK_LANE_OPS * world),
        "phase_ms": {k[3:]: round(avg[k], 4) for k in ("ms_device_decode", "ms_fiat_shamir", "ms_row_hash",
                                                       "ms_merkle", "ms_merkle_hash", "ms_ood_air", "ms_fri",
                                                       "ms_deep", "ms_device_total")},
        "host_prepare_ms": {"stage": st0["ms_decode"], "upload_wait": st0["ms_upload"], "total": prep_s * 1e3},
        "inflight": R,
        "iso_steps": iso_steps if acc_iso else 0,
    }
    inflight = roofline(acc_if, if_steps, if_ms, R,
                        f"{if_steps} steps right after the timed region, {R} in flight as there (launches of "
                        f"different steps overlap); per-launch HIP events (hipExtLaunchKernel start/stop)")
    # that pass's own rate beside the timed region's: the cost of the per-dispatch timestamps
    inflight["proofs_per_s_gpu_timed_region"] = n * K / elapsed
    inflight["proofs_per_s_gpu_with_dispatch_timestamps"] = n / (if_ms / 1e3)
    inflight["pass_steps"] = if_steps
    if acc_iso:
        res["roofline"] = roofline(acc_iso, iso_steps, iso_ms, 1,
                                   f"the kernel's own rate: {iso_steps} steps one at a time right after the timed "
                                   f"region; per-launch HIP events (hipExtLaunchKernel start/stop)")
        if gpu_shared:  # ranks time-sharing one GPU (a rehearsal): the other ranks' steps stretch these
            res["roofline"]["gpu_shared_by_ranks"] = world
        else:
            assert res["roofline"]["launches_x_avg_ms"] <= step_ms, (res["roofline"], step_ms)
        # the row-hashing launch of the same isolated steps (k_hash_rows: one lane per revealed row,
        # every main / aux / quotient row's hash_varlen; dispatch begin / end events), beside the
        # Merkle launches: permutations per launch = proofs x checks x sum over the three trees of
        # (width // 10 + 1), priced at the same 7,520 lane-ops per permutation
        rows_ms = acc_iso.get("ms_row_hash_exec", 0.0) / iso_steps
        if rows_ms > 0:
            widths = (stark.num_main, 3 * stark.num_aux, 3 * stark.num_quotient_segments)
            rows_perms = n * stark.num_collinearity_checks * sum(w // 10 + 1 for w in widths)
            ach = rows_perms * TIP5_VALU_OPS_PER_PERM / (rows_ms / 1e3)
            res["roofline"]["rows_kernel"] = {
                "kernel": "k_hash_rows", "kernel_avg_ms": rows_ms, "perms_per_launch": rows_perms,
                "achieved": ach / 1e12, "frac": ach / VALU_PEAK_LANE_OPS,
                "frac_of_measured_ceiling": ach / (VALU_ISSUE_CEILING * 64),
                "row_bytes_per_launch": n * stark.num_collinearity_checks * sum(widths) * 8,
                "measured": f"the same {iso_steps} isolated steps; hipExtLaunchKernel start/stop of the row launch"}
            rv, rv_tag = pmc_rows_valu_per_launch(args.config, len(proofs))
            if rv:
                # a row permutation skips its capacity-only / digest-only last-round outputs, so it
                # executes fewer than the fixed 7,520: the executed count (committed PMC pass of this
                # library) against the measured issue ceiling is the kernel's own issue fraction
                ex = rv * 64 / rows_perms
                res["roofline"]["rows_kernel"].update({
                    "valu_ops_per_perm_executed": ex, "executed_profile": rv_tag,
                    "executed_frac_of_measured_ceiling": rows_perms * ex / (rows_ms / 1e3) / (VALU_ISSUE_CEILING * 64)})
        res["roofline"]["inflight"] = {k: inflight[k] for k in ("achieved", "frac", "kernel_avg_ms",
                                                                 "kernel_avg_ms_events", "launches_per_step",
                                                                 "perms_per_launch", "launches_x_avg_ms", "step_ms",
                                                                 "measured", "proofs_per_s_gpu_timed_region",
                                                                 "proofs_per_s_gpu_with_dispatch_timestamps",
                                                                 "pass_steps")}
    else:
        res["roofline"] = inflight
    valu_step, valu_tag = pmc_valu_per_step(args.config, len(proofs))
    if valu_step:
        # the whole pipeline against the measured VALU issue ceiling: committed PMC instruction
        # count of one step (per GPU) / this run's step time
        # frac: against the fastest issue rate measured for any instruction class (cheap movs /
        # adds, 1.7 wave64 instructions per CU-clock), a hard ceiling; vs_regular_rate: against the
        # rate of the regular and slow classes the Tip5 mix is made of (1 per CU-clock), which the
        # mix's cheap instructions let it exceed slightly
        rate = valu_step / (elapsed / K)
        res["valu_issue"] = {"wave_instr_per_step": valu_step, "profile": valu_tag,
                             "ceiling_wave_instr_per_s": VALU_ISSUE_MAX, "frac": rate / VALU_ISSUE_MAX,
                             "regular_rate_wave_instr_per_s": VALU_ISSUE_CEILING,
                             "vs_regular_rate": rate / VALU_ISSUE_CEILING}
    # proof streaming: every proof word is read by the device at least once per step
    words_step = st0["proof_words"]
    step_s = elapsed / K
    res["hbm"] = {"proof_bytes_per_step": words_step * 8, "achieved_GBps": words_step * 8 / step_s / 1e9,
                  "peak_GBps": HBM_PEAK / 1e9, "frac": words_step * 8 / step_s / HBM_PEAK}
    bytes_step, bytes_tag = pmc_bytes_per_step(args.config, len(proofs))
    if bytes_step:
        res["hbm"].update({"pmc_bytes_per_step": bytes_step, "pmc_GBps": bytes_step / step_s / 1e9,
                           "pmc_frac": bytes_step / step_s / HBM_PEAK, "pmc_profile": bytes_tag})
    if product is not None:
        product["vs_value"] = product["value"] / res["value"]
        res["product_pipeline"] = product
    for b in ring:
        b.close()
    # the N = 8 rank's share on this GPU (rank 0 of 8's LPT shard of the same 4,096-proof job), in
    # the same command's shape (its own ring, warm-up, `steps` timed steps): what each GPU of the
    # driver's 8-GPU run does, measured on one
    if world == 1 and args.config == 4 and total == 4096 and args.share_steps > 0:
        sc, sp, se, _, _, _ = make_config4(pool4, total, 0.01, 8, 0)
        scl, spr = device_form(sc, sp, mont)
        sn = [NS.Claim(*c) for c in scl]
        Rs = default_inflight(len(sp))  # the rank's own depth (its default host exchange holds no GPU streams)
        sring = [NS.Batch(ctx, gair, stark, sn, spr) for _ in range(Rs)]
        kernel_timing(sring, region_timing)
        pipelined(sring, args.warmup, Rs, se)
        ctx.synchronize()
        dt, ok3 = pipelined(sring, args.share_steps, Rs, se)
        for b in sring:
            b.close()
        sh = {"proofs_per_step": len(sp), "inflight": Rs, "steps": args.share_steps, "warmup": args.warmup,
              "value": len(sp) * args.share_steps / dt, "unit": "proofs/s (one GPU)",
              "ms_per_step": dt / args.share_steps * 1e3, "verdicts_correct": ok3,
              "measured": "rank 0 of 8's LPT shard of the 4,096-proof job, resident, the timed region's shape at "
                          "the rank's depth; without the rank's process group and verdict exchange (their cost "
                          "at this size: DESIGN.md section 6)"}
        sh["vs_value_per_proof"] = sh["value"] / res["value"]
        # the round-5 review's bar: the share at >= SHARE_TARGET of the per-proof rate (reported, never
        # fatal: a slow box must not fail the run)
        sh["target_vs_value"] = SHARE_TARGET
        sh["meets_target"] = sh["vs_value_per_proof"] >= SHARE_TARGET
        if rank_path is not None:
            if "value" in rank_path:
                rank_path["vs_value_per_proof"] = rank_path["value"] / res["value"]
                correct = correct and rank_path["verdicts_correct"]
            sh["rank_path"] = rank_path
        res["share_n8"] = sh
        correct = correct and ok3
    _assert_fracs(res)
    # the PCIe-inclusive leg and the config-2 microbench belong to the one-GPU report (N = 1): with
    # several ranks, rank 0 would run them alone while the others tear down
    if args.stream_batches > 0 and not gpu_shared:
        # every rank at once (its shard to its own GPU): the multi-process form of the node's feed
        pc = pcie_stream(ctx, gair, stark, dev_claims, dev_proofs, expect, args.stream_batches, dist, total)
        res["pcie_inclusive"] = pc
        correct = correct and pc["verdicts_correct"] is not False  # None: the leg raised (reported in it)
    if world == 1 and args.paths_log2 > 0:
        res["tip5_paths"] = tip5_paths(ctx, args.paths_log2, 5)
    if world == 1 and args.queue_callers > 0:
        t = time.time()
        res["queue"] = queue_leg(ctx, gair, stark, dev_claims, dev_proofs, expect, args.queue_callers)
        correct = correct and res["queue"]["verdicts_correct"]
        log(f"[queue] {res['queue']['value']:.0f} proofs/s ({time.time() - t:.1f}s)")
    if world == 1 and args.config5_proofs > 0:
        t = time.time()
        res["config5"] = config5_leg(ctx, gair, stark, args.config5_proofs, inflight=args.config5_inflight)
        correct = correct and res["config5"]["verdicts_correct"]
        if args.config5_proofs >= 16:
            # the N = 8 rank's share of config 5 (64 / 8 = 8 proofs per GPU), in the same shape
            sh5 = config5_leg(ctx, gair, stark, args.config5_proofs // 8)
            correct = correct and sh5["verdicts_correct"]
            res["config5"]["share_n8"] = {k: sh5[k] for k in ("value", "unit", "ms_per_step", "steps", "inflight",
                                                              "alone_ms", "transcript_equals_oracle",
                                                              "verdicts_correct")}
            res["config5"]["share_n8"]["proofs"] = args.config5_proofs // 8
            if args.config5_proofs == 64:  # the round-5 review's bar for this share (reported, never fatal)
                res["config5"]["share_n8"]["target"] = CONFIG5_SHARE_TARGET
                res["config5"]["share_n8"]["meets_target"] = sh5["value"] >= CONFIG5_SHARE_TARGET
        log(f"[config5] {res['config5']['value']:.0f} proofs/s ({time.time() - t:.1f}s)")
    if world == 1 and args.config1_seconds > 0 and not args.no_cpu:
        res["config1_latency"] = config1_latency(ctx, gair, stark, air_words, args.config1_seconds)
        correct = correct and res["config1_latency"]["verdict_accept"]
    if cpu is not None:
        res["cpu_baseline"] = cpu
    if hwq4 is not None:
        res["hw_queues_4"] = hwq4
        correct = correct and hwq4["verdicts_correct"]
    # the in-process multi-GPU form (one process, nhip_group_stream over every GPU of the job): rank
    # 0 drives all of them while the other ranks wait on the host with their batches freed
    if args.group_batches > 0 and args.config == 4 and not under_profiler():
        if dist is not None:
            dist.barrier()  # every rank's batches are closed

        def leg():
            job_claims, job_proofs, job_expect = claims, proofs, expect
            if world > 1:
                job_claims, job_proofs, job_expect, _, _, _ = make_config4(pool4, total, 0.01, 1, 0)
            dcl, dpr = device_form(job_claims, job_proofs, mont)
            # every GPU the job's ranks use (a gloo rehearsal puts several ranks on one GPU)
            n_dev = max(1, __import__("torch").cuda.device_count()) if dist is not None else 1
            devs = sorted({r % n_dev for r in range(world)})
            out = {}
            try:
                t = time.time()
                out["pinned"] = group_stream(devs, air_words, stark, dcl, dpr, job_expect, args.group_batches)
                out["pageable"] = group_stream(devs, air_words, stark, dcl, dpr, job_expect, args.group_batches,
                                               pageable=True)
                log(f"[group] {out['pinned']['value']:.0f} proofs/s pinned arenas, {out['pageable']['value']:.0f} "
                    f"pageable ({time.time() - t:.1f}s)")
                if args.node_batches > 0:
                    t = time.time()
                    stream = tx_stream(job_proofs)  # canonical words: the wire form
                    log(f"[node] {stream.size / 1e9:.2f} GB of TransferTransactions ({time.time() - t:.1f}s)")
                    out["node"] = node_from_bytes(devs, air_words, job_claims, job_proofs, job_expect,
                                                  args.node_batches, stream)
                    del stream
            except Exception as e:  # noqa: BLE001 -- a leg, never the headline
                for k in ("pinned", "pageable", "node"):
                    out.setdefault(k, {"error": repr(e)[:300], "verdicts_correct": None})
            finally:
                if dist is not None:
                    import torch
                    torch.cuda.set_device(dev_index)  # the members' threads ran on the other devices
            return out

        def safe_leg():  # whatever raises in the leg stays in the leg (reported in its fields)
            try:
                return leg()
            except Exception as e:  # noqa: BLE001
                return {k: {"error": repr(e)[:300], "verdicts_correct": None} for k in ("pinned", "pageable")}

        t = time.time()
        legs = shard.on_rank0(safe_leg, dist, "nhip_group_stream_done")
        if rank == 0:
            g, gp = legs["pinned"], legs["pageable"]
            res["group_stream"] = g
            res["group_stream_pageable"] = gp
            for x in (g, gp):
                if "value" in res.get("pcie_inclusive", {}) and "value" in x:
                    x["vs_pcie_inclusive"] = x["value"] / res["pcie_inclusive"]["value"]
            if "value" in g and "value" in gp:
                gp["vs_pinned"] = gp["value"] / g["value"]
            # None: a leg that raised (its error is in the line); False: wrong verdicts (fails the run)
            correct = correct and g["verdicts_correct"] is not False and gp["verdicts_correct"] is not False
            if "node" in legs:
                nd = legs["node"]
                res["node_bytes_to_verdicts"] = nd
                correct = correct and nd["verdicts_correct"] is not False
                if "value" in nd and "value" in g:
                    nd["vs_pinned_group"] = nd["value"] / g["value"]
            log(f"[group legs] over {world} GPU(s) ({time.time() - t:.1f}s)")
    if rank == 0:
        # the whole node fed from host memory, beside `value` (HBM-resident input, the bench
        # contract): bytes -> verdicts through the per-member pinned arenas (one process, every GPU),
        # and the multi-process form (every rank streaming its shard from pinned memory); the
        # binding ceiling is the host-to-device link (roofline.pcie)
        nfh = {}
        src = res.get("node_bytes_to_verdicts") if "value" in res.get("node_bytes_to_verdicts", {}) else None
        pc = res.get("pcie_inclusive")
        if pc is not None and "value" not in pc:
            pc = None  # the leg raised (its error is in the line)
        if src is not None:
            nfh = {"value": src["value"], "unit": "proofs/s", "gpus": src["gpus"],
                   "path": "wire bytes -> per-GPU pinned arenas -> GPUs -> verdicts (node_bytes_to_verdicts)"}
        elif pc is not None:
            nfh = {"value": pc["value"], "unit": "proofs/s", "gpus": world,
                   "path": "pinned host memory -> GPUs -> verdicts (pcie_inclusive)"}
        if nfh:
            nfh["vs_value"] = nfh["value"] / res["value"]
            res["node_from_host"] = nfh
        if pc is not None:
            peak = pc["h2d_peak_GBps"] * world
            ach = (src["h2d_GBps"] if src is not None else pc["h2d_GBps"] * world)
            res["roofline"]["pcie"] = {"bound": "pcie", "achieved": ach, "peak": peak, "unit": "GB/s",
                                       "frac": ach / peak if peak else None,
                                       "per_gpu_link_peak_GBps": pc["h2d_peak_GBps"],
                                       "measured": "achieved: the proof bytes of node_from_host's path per second; "
                                                   "peak: one pinned->device copy of the same bytes per GPU "
                                                   "(best of 3, pcie_inclusive) x GPUs"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist is not None:
        dist.barrier()  # every rank tears its communicator down together
        dist.destroy_process_group()
    return 0 if correct else 1


if __name__ == "__main__":
    sys.exit(main())
