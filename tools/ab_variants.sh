#!/bin/bash
# Config-4 throughput of the current library against several variant libraries (NHIP_LIB),
# alternating: for each repetition, each share, each library in turn.
# Usage: SIZES="4096 512" REPS=2 bash tools/ab_variants.sh TAG NAME=VARIANT_SO ...
set -o pipefail
OUT=gpurun_out/ab_$1; shift; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for n in ${SIZES:-4096 512}; do
for spec in cur "$@"; do
  name=${spec%%=*}
  if [ "$spec" = cur ]; then unset NHIP_LIB; else export NHIP_LIB=$PWD/${spec#*=}; fi
  f=$OUT/n${n}_${name}_r$rep
  timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --iso-steps 0 --steps ${STEPS:-200} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json n${n}_${name}_r$rep
done
done
done
