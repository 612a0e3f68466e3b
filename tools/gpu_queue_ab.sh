#!/bin/bash
# The coalescing queue's 64-caller rate and small-batch latency: this library vs older ones
# (NHIP_LIB), alternating, 2 repetitions.
set -o pipefail
OUT=gpurun_out/queue_ab; mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/neptune-core_amd/build/variants
for rep in 1 2; do for lib in cur r03r pre; do
  if [ $lib = cur ]; then unset NHIP_LIB; else export NHIP_LIB=$V/libneptune_hip_$lib.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -m gpu -q -s -k coalescing --timeout 200 --timeout-method thread > $OUT/q_${lib}_$rep.log 2>&1
  grep -h "serialized" $OUT/q_${lib}_$rep.log | sed "s/^/$lib r$rep: /"
  timeout -k 10 300 python -u tools/latency.py 10 > $OUT/lat_${lib}_$rep.json 2> $OUT/lat_${lib}_$rep.err || { tail -3 $OUT/lat_${lib}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], {k:v for k,v in d.items() if 'ms' in k or isinstance(v,(int,float))})" $OUT/lat_${lib}_$rep.json "$lib r$rep latency"
done; done
