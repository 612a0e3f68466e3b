#!/bin/bash
# GPU parity tests, then bench configs 3 / 4 / 5 at N=1 (no CPU leg).
set -o pipefail
OUT=gpurun_out/cfg
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --no-cpu --paths-log2 0 --config $c > $OUT/c$c.json 2> $OUT/c$c.err || { tail -20 $OUT/c$c.err; exit 1; }
  python3 -c "import json;b=json.load(open('$OUT/c$c.json'));print('config $c',round(b['value']),b['unit'],round(b['ms_per_step'],3),b['tip5_perms_per_proof'],b['roofline']['frac'],b['verdicts_correct'])"
done
