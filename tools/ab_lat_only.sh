#!/bin/bash
# Small-batch device latency only (tools/latency.py resident runs) for library variants, alternating.
#   bash tools/ab_lat_only.sh TAG ROUNDS name1 name2 ...   ("main" = the in-tree library)
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = main ]; then L=neptune-core_amd/neptune_hip/libneptune_hip.so; else L=neptune-core_amd/build/variants/libneptune_hip_$v.so; fi
    NHIP_LIB=$L timeout -k 10 300 python -u tools/latency.py 15 > $OUT/lat_$v.$r.log 2>&1 || { tail $OUT/lat_$v.$r.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/lat_$v.$r.log').read().strip().splitlines()[-1]);print('$v',' '.join(f\"{k.split()[0]}:{v['resident_run_ms']}\" for k,v in d.items()))"
  done
done
