#!/bin/bash
# Full GPU round: parity tests, smoke, the default bench (with CPU baseline), then the rocprofv3
# passes of tools/profile_round.sh.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print(b['value'],b['ms_per_step'],b['roofline']['frac'],b.get('roofline_isolated',{}).get('frac'),b['cpu_baseline']['value'],b['tip5_paths']['perms_per_s'])"
bash tools/profile_round.sh $TAG
