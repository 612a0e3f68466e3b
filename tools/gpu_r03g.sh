#!/bin/bash
# Quad-form sponge replay: parity (every form on the pool proofs; config 4 and the STARK suites at
# the default selection), then the A/B of the replay form at the config-4 per-GPU shares.
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fs_forms.py tests/test_gpu_config4.py tests/test_gpu_stark.py tests/test_gpu_deep_fri.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
SIZES="4096 2048 1024" REPS=2 STEPS=200 bash tools/ab_env_sizes.sh r03g "row:NHIP_FS_FORM=row" "quad:NHIP_FS_FORM=quad"
