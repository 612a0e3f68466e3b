#!/bin/bash
# Round-start baseline: GPU parity tests, then config-4 and config-3 benches (no CPU leg).
set -o pipefail
OUT=gpurun_out/${1:-base}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu --config 4 --paths-log2 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u bench.py --no-cpu --config 4 --paths-log2 0 > $OUT/bench_c4_q4.json 2> $OUT/bench_c4_q4.err || { tail -20 $OUT/bench_c4_q4.err; exit 1; }
for f in $OUT/bench_c4.json $OUT/bench_c4_q4.json; do
python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[1],round(b['value']),round(b['ms_per_step'],3),b['phase_ms'],round(b['roofline']['frac'],4),b['verdicts_correct'],b['inflight'])" $f
done
