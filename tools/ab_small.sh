#!/bin/bash
# Small-batch (one rank's share at N=8 / N=4) config-4 runs at several steps in flight.
set -o pipefail
OUT=gpurun_out/ab_small_$1; mkdir -p $OUT
for p in ${PROOFS:-512 1024}; do
  for inf in ${INFLIGHT:-2 3}; do
    f=$OUT/p${p}_i$inf
    timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $p --paths-log2 0 --stream-batches 0 --inflight $inf --steps 40 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json p${p}_i$inf
  done
done
