#!/bin/bash
# DEEP with 22-bit weight limbs: the STARK parity suites (default and other Stark parameters, deep
# FRI, payload sweep, config 4), then the A/B against the HEAD library at the config-4 shares.
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stark.py tests/test_gpu_stark_params.py tests/test_gpu_deep_fri.py tests/test_gpu_payload_sweep.py tests/test_gpu_config4.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
SIZES="${SIZES:-4096 512}" REPS=${REPS:-3} STEPS=200 bash tools/ab_lib_sizes.sh r03h neptune-core_amd/build/variants/libneptune_hip_head.so
