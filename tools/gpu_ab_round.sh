#!/bin/bash
# GPU tests + the queue test's profile + an A/B of library / environment variants (tools/ab.sh specs).
# Usage: SIZES="4096 512" REPS=2 bash tools/gpu_ab_round.sh TAG "name|ENV|args" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_tests.sh $TAG || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q -s --timeout 200 --timeout-method thread > $OUT/queue.log 2>&1 || { tail -20 $OUT/queue.log; exit 1; }
grep -E "serialized|queue per batch" $OUT/queue.log
bash tools/ab.sh $TAG "$@"
