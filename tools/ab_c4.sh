#!/bin/bash
# A/B of config-4 bench: library variants x steps in flight.  Usage: tools/ab_c4.sh TAG lib1 lib2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in 1 2; do
for lib in "$@"; do
  for inf in 1 2; do
    name=$(basename $lib .so)_i${inf}_r$rep
    NHIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --config 4 --paths-log2 0 --inflight $inf --steps 20 > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),{k:round(v,2) for k,v in b['phase_ms'].items()},b['verdicts_correct'])" $OUT/$name.json $name
  done
done
done
