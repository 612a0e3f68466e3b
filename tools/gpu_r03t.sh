#!/bin/bash
# FRI barycentric evaluation with one inversion per pair of points: the FRI / STARK parity suites,
# then the A/B against HEAD at 4,096 / 512 proofs.
set -o pipefail
OUT=gpurun_out/r03t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_deep_fri.py tests/test_gpu_stark.py tests/test_gpu_stark_params.py tests/test_gpu_payload_sweep.py tests/test_gpu_config4.py tests/test_gpu_config5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
V=$PWD/neptune-core_amd/build/variants
SIZES="4096 512" REPS=3 STEPS=200 bash tools/ab_env_sizes.sh r03t "cur:" "head:NHIP_LIB=$V/libneptune_hip_head.so"
