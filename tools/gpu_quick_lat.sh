#!/bin/bash
# GPU tests matching $2 (default: the STARK parity core), then small-batch latency and the
# config-4 bench at 4,096 and 512 proofs per GPU.
set -o pipefail
T=$1; K=${2:-"tiny or decode or config4 or config5 or mutation or heights"}
tools/gpu_tests.sh $T "$K" || exit 1
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/latency.py 15 > gpurun_out/$T/lat.log 2>&1 || { tail -5 gpurun_out/$T/lat.log; exit 1; }
head -4 gpurun_out/$T/lat.log
for p in 4096 512; do
  timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $p --paths-log2 0 --stream-batches 0 --steps 30 > gpurun_out/$T/b$p.json 2> gpurun_out/$T/b$p.err || { tail -5 gpurun_out/$T/b$p.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" gpurun_out/$T/b$p.json p$p
done
