#!/bin/bash
# S-box byte packing by v_perm_b32: Tip5 KATs and the STARK suites, then the A/B against HEAD.
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tip5.py tests/test_gpu_stark.py tests/test_gpu_fs_forms.py tests/test_gpu_config4.py tests/test_gpu_pow.py tests/test_gpu_mast.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
SIZES="${SIZES:-4096 512}" REPS=${REPS:-3} STEPS=200 bash tools/ab_lib_sizes.sh r03i neptune-core_amd/build/variants/libneptune_hip_head.so
