#!/bin/bash
# Steps in flight x per-GPU share (config 4), REPS alternating repetitions.
# Usage: SPECS="4096:2 4096:3 512:4:14 512:6" REPS=2 bash tools/ab_inflight.sh TAG   (n:inflight[:hw queues])
set -o pipefail
OUT=gpurun_out/ab_$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
for rep in $(seq 1 ${REPS:-2}); do
for spec in $SPECS; do
  n=${spec%%:*}; rq=${spec#*:}; r=${rq%%:*}; q=${rq#*:}
  [ "$q" = "$rq" ] && q=""
  f=$OUT/n${n}_r${r}_q${q}_rep$rep
  NHIP_BENCH_HWQ=$q timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --inflight $r --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps ${STEPS:-200} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json n${n}_inflight${r}_hwq${q}_rep$rep
done
done
