#!/bin/bash
# A/B of the aux-chain release level (NHIP_AUX_AFTER_LEVEL).
set -o pipefail
mkdir -p gpurun_out/abx
for L in 0 2 4 6 8 10; do
  NHIP_AUX_AFTER_LEVEL=$L timeout -k 10 200 python -u bench.py --no-cpu --paths-log2 0 > gpurun_out/abx/l$L.json 2> gpurun_out/abx/l$L.err || { tail gpurun_out/abx/l$L.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/abx/l$L.json'));print('level $L',round(b['ms_per_step'],3),b['phase_ms']['merkle_hash'],b['verdicts_correct'])"
done
