#!/bin/bash
# Quick GPU check: parity tests + default bench (no CPU leg), printing value / phases / Tip5 microbench.
set -o pipefail
OUT=gpurun_out/${1:-q}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print(round(b['value']),round(b['ms_per_step'],3),b['phase_ms']['row_hash'],b['phase_ms']['merkle_hash'],round(b['roofline']['frac'],4),'paths',round(b['tip5_paths']['perms_per_s']/1e9,3),'e9',b['verdicts_correct'])"
