#!/bin/bash
# Kernel traces of the config-4 bench at the per-GPU shares (default 512 and 1,024 proofs), with
# tools/trace_util.py's occupancy summary of each.
set -o pipefail
OUT=$PWD/gpurun_out/trace_shares; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
for n in ${SIZES:-512 1024}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t$n -o trace --output-format csv -- python3 bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps 100 --iso-steps 0 > $OUT/t$n.json 2> $OUT/t$n.err || exit 1
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[1],round(b['value']),round(b['ms_per_step'],3),b['phase_ms'])" $OUT/t$n.json
  python3 tools/trace_util.py $OUT/t$n 0.3 0.9
done
