#!/bin/bash
# k_deep_rows8 correctness (GPU STARK tests with NHIP_DEEP_ROWS8=1), then the A/B of the sponge form
# and the DEEP form at the N = 8 / N = 4 per-GPU shares and at 4,096 proofs.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
NHIP_DEEP_ROWS8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stark.py tests/test_gpu_deep_fri.py tests/test_gpu_payload_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_rows8.log 2>&1 || { tail -20 $OUT/pytest_rows8.log; exit 1; }
tail -1 $OUT/pytest_rows8.log
SIZES="512 1024 4096" REPS=2 STEPS=200 bash tools/ab_env_sizes.sh r03c "base:" "pair:NHIP_FS_PAIR=1" "rows8:NHIP_DEEP_ROWS8=1"
