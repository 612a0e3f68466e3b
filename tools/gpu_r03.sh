#!/bin/bash
# Round-3 GPU pass: the config-4 pool, the GPU parity tests, the default bench line and config 4 at
# the box's default 4 hardware queues.  Each GPU step under its own time limit; stops at the first
# failure.  Usage: bash tools/gpu_r03.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
sha256sum neptune-core_amd/neptune_hip/libneptune_hip.so > $OUT/LIB_SHA256
t=$(date +%s)
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; p = pool4.load(); print(len(p['proofs']), p['build_s'])" > $OUT/pool4.log 2>&1 || { tail -20 $OUT/pool4.log; exit 1; }
echo "pool4 $(cat $OUT/pool4.log) $(( $(date +%s) - t ))s"
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_default.json')); print('default', round(b['value']), b['ms_per_step'], b['roofline']['frac'], b.get('roofline_isolated',{}).get('frac'), b['verdicts_correct'], b['config']['gpu_max_hw_queues'])"
NHIP_BENCH_HWQ=4 timeout -k 10 300 python -u bench.py --no-cpu --paths-log2 0 --stream-batches 0 > $OUT/bench_hwq4.json 2> $OUT/bench_hwq4.err || { tail -20 $OUT/bench_hwq4.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_hwq4.json')); print('hwq4', round(b['value']), b['ms_per_step'], b['roofline']['frac'], b['verdicts_correct'], b['config']['gpu_max_hw_queues'])"
echo done
