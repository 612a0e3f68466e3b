#!/bin/bash
# GPU parity tests only (one process), log under gpurun_out/<tag>/.
set -o pipefail
OUT=gpurun_out/${1:-t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${2:-} > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
