#!/bin/bash
# A/B of environment variants over config-4 per-GPU shares, REPS alternating repetitions.
# Usage: SIZES="4096 512" REPS=2 tools/ab_env_sizes.sh TAG "name:VAR=v" "name2:" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for n in ${SIZES:-4096 1024 512}; do
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  f=$OUT/n${n}_${name}_r$rep
  env $envs timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps ${STEPS:-20} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),'rf',round(b['roofline']['frac'],3),'iso',round(b['roofline_isolated']['frac'],3),'L',b['roofline']['launches_per_step'],b['verdicts_correct'])" $f.json n${n}_${name}_r$rep
done
done
done
