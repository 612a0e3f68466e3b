#!/bin/bash
# Per-tree climb threshold (NHIP_CLIMB_MAX): config 5 (log2 height 23) and config 4 shares of
# 16-256 proofs, with the climb up to 16 proofs (default) vs up to 256.
set -o pipefail
OUT=gpurun_out/ab_climb; mkdir -p $OUT
for rep in 1 2; do
for cfg in 5:8 5:32 5:64 4:32 4:64 4:128 4:256; do
  IFS=: read c p <<< "$cfg"
  for cm in 16 256; do
    f=$OUT/c${c}_p${p}_m${cm}_r$rep
    NHIP_CLIMB_MAX=$cm timeout -k 10 300 python -u bench.py --config $c --no-cpu --paths-log2 0 --stream-batches 0 --proofs $p --steps 30 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json c${c}_p${p}_m${cm}_r$rep
  done
done
done
