#!/bin/bash
# A/B of whole-library variants (tools/build_variant.sh): alternating default-bench runs.
#   bash tools/ab_lib.sh TAG ROUNDS name1 name2 ...   ("main" = neptune_hip/libneptune_hip.so)
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = main ]; then L=neptune-core_amd/neptune_hip/libneptune_hip.so; else L=neptune-core_amd/build/variants/libneptune_hip_$v.so; fi
    NHIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail $OUT/$v.$r.err; exit 1; }
    python3 -c "import json;b=json.load(open('$OUT/$v.$r.json'));print('$v',round(b['ms_per_step'],3),'hash',b['phase_ms']['merkle_hash'],'row',b['phase_ms']['row_hash'],'paths',round(b['tip5_paths']['perms_per_s']/1e9,3),b['verdicts_correct'])"
  done
done
