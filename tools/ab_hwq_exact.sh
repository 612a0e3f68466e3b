#!/bin/bash
# Exact GPU_MAX_HW_QUEUES (NHIP_BENCH_HWQ) x steps in flight: config 5 at 8 proofs, config 4 at 512.
set -o pipefail
OUT=gpurun_out/ab_hwqx; mkdir -p $OUT
for cfg in ${CFGS:-5:8:4:10 5:8:6:8 5:8:6:10 5:8:6:14 4:512:4:6 4:512:4:8 4:512:4:10 4:512:6:8 4:512:6:10}; do
  IFS=: read c p inf q <<< "$cfg"
  f=$OUT/c${c}_p${p}_i${inf}_q$q
  NHIP_BENCH_HWQ=$q timeout -k 10 300 python -u bench.py --config $c --no-cpu --paths-log2 0 --stream-batches 0 --proofs $p --inflight $inf --steps 40 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json c${c}_p${p}_i${inf}_q$q
done
