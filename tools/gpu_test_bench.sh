#!/bin/bash
# GPU parity tests, then a short bench (no CPU leg).  Usage: bash tools/gpu_test_bench.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu ${*} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print(b['value'],b['ms_per_step'],b['phase_ms'],b['roofline']['frac'],b['verdicts_correct'])"
