#!/bin/bash
# Config-4 share of PROOFS proofs: steps in flight x GPU_MAX_HW_QUEUES grid (bench sets the queue
# count only when the environment asks for fewer than it wants).
set -o pipefail
OUT=gpurun_out/ab_hwq_$1; mkdir -p $OUT
P=${PROOFS:-512}
for cfg in ${CFGS:-4:10 4:16 5:16 6:16}; do
  inf=${cfg%%:*}; q=${cfg##*:}
  f=$OUT/p${P}_i${inf}_q$q
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $P --paths-log2 0 --stream-batches 0 --inflight $inf --steps 60 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f.json p${P}_i${inf}_q$q
done
