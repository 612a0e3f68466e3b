#!/bin/bash
# Queue test + default bench (with the 4-queue leg) + a kernel trace of the N = 8 per-GPU share
# (512 proofs, 4 in flight).  Usage: bash tools/gpu_r03b.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
sha256sum neptune-core_amd/neptune_hip/libneptune_hip.so > $OUT/LIB_SHA256
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_stark.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_default.json')); print('default', round(b['value']), b['ms_per_step'], b['roofline']['frac'], b['verdicts_correct'], 'hwq4', b.get('hw_queues_4'))"
A="--proofs 512 --steps 60 --warmup 5 --no-cpu --paths-log2 0 --stream-batches 0 --config1-seconds 0 --hwq4-steps 0 --iso-steps 0"
timeout -k 10 300 python -u bench.py $A > $OUT/bench_512.json 2> $OUT/bench_512.err || { tail -20 $OUT/bench_512.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_512.json')); print('512', round(b['value']), b['ms_per_step'], b['phase_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace512 -o trace --output-format csv -- python3 bench.py $A > $OUT/bench_512_trace.json 2> $OUT/trace512.err || { tail -20 $OUT/trace512.err; exit 1; }
echo done
