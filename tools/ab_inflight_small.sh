#!/bin/bash
# Steps in flight for tiny per-GPU batches: config 5 at 8 / 64 proofs, config 4 at 32 / 128.
set -o pipefail
OUT=gpurun_out/ab_infl; mkdir -p $OUT
for cfg in 5:8 5:64 4:32 4:128; do
  IFS=: read c p <<< "$cfg"
  for inf in 4 6; do
    f=$OUT/c${c}_p${p}_i$inf
    timeout -k 10 300 python -u bench.py --config $c --no-cpu --paths-log2 0 --stream-batches 0 --proofs $p --inflight $inf --steps 40 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json c${c}_p${p}_i$inf
  done
done
