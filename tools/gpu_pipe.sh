#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pipe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1 || { tail -30 gpurun_out/pipe/pytest.log; exit 1; }
tail -2 gpurun_out/pipe/pytest.log
for P in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --no-cpu --paths-log2 0 --pipeline $P > gpurun_out/pipe/p$P.json 2> gpurun_out/pipe/p$P.err || { tail gpurun_out/pipe/p$P.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/pipe/p$P.json'));print($P,round(b['value']),round(b['ms_per_step'],3),b['roofline']['frac'],b['verdicts_correct'])"
done
