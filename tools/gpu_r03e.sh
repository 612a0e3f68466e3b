#!/bin/bash
# Full GPU suite at HEAD, then the 1,024-thread OOD evaluator for small batches vs 256 threads
# (NHIP_OOD_WIDE_MAX=0): call latency, config 1's single-proof latency, config 5 at 8 proofs per GPU.
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum neptune-core_amd/neptune_hip/libneptune_hip.so > $OUT/LIB_SHA256
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for v in wide narrow; do
  if [ $v = narrow ]; then export NHIP_OOD_WIDE_MAX=0; else unset NHIP_OOD_WIDE_MAX; fi
  timeout -k 10 300 python -u tools/latency.py 20 > $OUT/latency_$v.log 2>&1 || { tail -10 $OUT/latency_$v.log; exit 1; }
  echo "== $v"; cat $OUT/latency_$v.log | head -4
  timeout -k 10 300 python -u bench.py --steps 50 --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --cpu-seconds 2 --config1-seconds 2 --iso-steps 0 > $OUT/c1_$v.json 2> $OUT/c1_$v.err || { tail -10 $OUT/c1_$v.err; exit 1; }
  python3 -c "import json;b=json.load(open('$OUT/c1_$v.json'));c=b['config1_latency'];print('config1', c['gpu_resident_ms'], c['gpu_from_host_ms'], c['cpu_ms'])"
  timeout -k 10 300 python -u bench.py --config 5 --proofs 8 --steps 100 --no-cpu --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --iso-steps 0 > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -10 $OUT/c5_$v.err; exit 1; }
  python3 -c "import json;b=json.load(open('$OUT/c5_$v.json'));print('config5 x8', round(b['value']), b['ms_per_step'], b['phase_ms'])"
done
NS=1 bash tools/trace_lat.sh r03e && python3 tools/timeline.py gpurun_out/trace_lat_r03e/n1 > gpurun_out/r03e/timeline_n1.txt
echo done
