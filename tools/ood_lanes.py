#!/usr/bin/env python3
"""Lane model of the compiled OOD program ("Lane efficiency of the steps"), host only.

k_ood_air runs a step's instructions on the workgroup's threads, instruction q on thread q mod 256;
a wave issues the union of the XFE operations its 64 lanes hold and idle lanes still take its issue
slots.  With a cost per operation (gfx950 ISA VALU counts: product ~200, sum ~24, difference ~15,
copy ~12) this prints the useful and the issued lane-operations per proof of the bench's
triton-size AIR (or the synthetic one), plus the constraint weighing after the last step.
Usage: python tools/ood_lanes.py [synthetic|triton-size] [threads]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OOD_ADD, OOD_SUB, OOD_MUL, OOD_LOAD, OOD_ACC = 2, 3, 4, 5, 6
COST = {OOD_ADD: 24, OOD_SUB: 15, OOD_MUL: 200, OOD_LOAD: 12, OOD_ACC: 12}
WEIGH = 2 * COST[OOD_MUL] + COST[OOD_ADD]  # w_c * (C_c * Z^-1) + acc, per constraint


def main():
    import bench
    import stark_ref as S  # descriptor construction only (the bench's --air triton-size)
    from neptune_hip import stark as NS
    which = sys.argv[1] if len(sys.argv) > 1 else "triton-size"
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    words = bench.load_pool4()["air"]
    if which == "triton-size":
        words = S.bloat_air(S.AirCircuit.from_words([int(w) for w in words]), 24000).to_words()
    air = NS.Air(words)
    off, ins = air.program()
    ops = ins[:, 0]
    n_cons = air.info()["constraints"]
    useful = sum(COST[int(o)] for o in ops) + n_cons * WEIGH
    issued = 0
    for s in range(len(off) - 1):
        seg = ops[off[s]:off[s + 1]]
        for base in range(0, len(seg), threads):
            chunk = seg[base:base + threads]
            for w in range(0, len(chunk), 64):
                issued += 64 * sum(COST[k] for k in set(int(x) for x in chunk[w:w + 64]))
    issued += 64 * WEIGH * ((n_cons + threads - 1) // threads) * (threads // 64)
    kinds = collections.Counter(int(o) for o in ops)
    print(f"{which}: {air.info()}, {len(off) - 1} steps, instructions {dict(kinds)}")
    print(f"useful {useful:,} lane-ops per proof, issued {issued:,}, lane efficiency {useful / issued:.3f}")


if __name__ == "__main__":
    main()
