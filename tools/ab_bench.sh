#!/bin/bash
# A/B of runtime toggles: per-launch hash events and device perm counting.
set -o pipefail
mkdir -p gpurun_out/ab
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  NHIP_HASH_TIMING=$1 NHIP_PERM_COUNT=$2 timeout -k 10 200 python -u bench.py --no-cpu --paths-log2 0 > gpurun_out/ab/t$1$2.json 2> gpurun_out/ab/t$1$2.err || { tail gpurun_out/ab/t$1$2.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/ab/t$1$2.json'));print('timing=$1 count=$2',round(b['ms_per_step'],3),b['phase_ms']['merkle_hash'])"
done
