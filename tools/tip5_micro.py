#!/usr/bin/env python3
"""Config-2 Tip5 microbench alone (k_mtree_verify over 2^N depth-N paths), for A/B and PMC runs.
Usage: python tools/tip5_micro.py [log2_leaves=20] [steps=5]   (library from NHIP_LIB if set)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import neptune_hip as nh  # noqa: E402

if __name__ == "__main__":
    log2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ctx = nh.Context(0)
    r = bench.tip5_paths(ctx, log2, steps)
    r["lib"] = os.environ.get("NHIP_LIB", "main")
    print(json.dumps(r))
