#!/bin/bash
# A/B of the config-4 bench over environment variants x steps in flight.
# Usage: tools/ab_env_c4.sh TAG "name:VAR=v VAR2=w" "name2:" ...   (2 alternating repetitions)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in 1 2; do
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for inf in ${INFLIGHT:-1 2}; do
    f=$OUT/${name}_i${inf}_r$rep
    env $envs timeout -k 10 200 python -u bench.py --no-cpu --config 4 --paths-log2 0 --inflight $inf --steps 20 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),{k:round(v,2) for k,v in b['phase_ms'].items()},b['verdicts_correct'])" $f.json ${name}_i${inf}_r$rep
  done
done
done
