#!/bin/bash
# GPU parity tests only (one process), log under gpurun_out/<tag>/.  Optional 2nd arg: a pytest -k
# expression (output shown with -s).
set -o pipefail
OUT=gpurun_out/${1:-t}
mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$2" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
