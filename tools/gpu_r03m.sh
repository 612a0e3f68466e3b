#!/bin/bash
# Shape-grouped device order: the batch-API suites (config 4 incl. a shuffled batch, sponge forms,
# STARK, queue, group, concurrency, callers), then shuffled vs LPT order, this library vs HEAD's.
set -o pipefail
OUT=gpurun_out/r03m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_fs_forms.py tests/test_gpu_stark.py tests/test_gpu_queue.py tests/test_gpu_group.py tests/test_gpu_concurrent.py tests/test_gpu_callers.py tests/test_gpu_decode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
V=$PWD/neptune-core_amd/build/variants/libneptune_hip_head.so
for rep in 1 2; do for n in 4096 512; do for sh in lpt shuffle; do for lib in cur head; do
  f=$OUT/n${n}_${sh}_${lib}_r$rep.json
  a=""; [ $sh = shuffle ] && a="--shuffle"
  if [ $lib = head ]; then export NHIP_LIB=$V; else unset NHIP_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 $a > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1],round(b['value']),round(b['ms_per_step'],3),b['phase_ms']['fiat_shamir'],b['verdicts_correct'])" $f
done; done; done; done
# the driver's timed region (20 steps after 5 warm-up steps): steps in flight at the shares
STEPS=20 SPECS="512:4 512:8 1024:4 1024:8 2048:4 2048:8 4096:2" REPS=3 bash tools/ab_inflight.sh k20
