#!/bin/bash
# Small-batch latency (tools/latency.py) and default bench for library variants.
#   bash tools/ab_latency.sh TAG name1 name2 ...   ("main" = the in-tree library)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = main ]; then L=neptune-core_amd/neptune_hip/libneptune_hip.so; else L=neptune-core_amd/build/variants/libneptune_hip_$v.so; fi
  NHIP_LIB=$L timeout -k 10 300 python -u tools/latency.py 15 > $OUT/lat_$v.log 2>&1 || { tail $OUT/lat_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/lat_$v.log)"
  NHIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --paths-log2 0 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail $OUT/bench_$v.err; exit 1; }
  python3 -c "import json;b=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1]);p=b['phase_ms'];print('$v',round(b['ms_per_step'],3),'fs',p['fiat_shamir'],'rows',p['row_hash'],'hash',p['merkle_hash'],b['verdicts_correct'])"
done
