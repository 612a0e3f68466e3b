#!/bin/bash
# One GPU round check: the GPU tests, smoke, the default bench line, and the input-form / AIR A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04}; mkdir -p $OUT
bash tools/gpu_tests.sh ${1:-r04} || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
tail -c 600 $OUT/bench_default.json
SIZES=${SIZES:-4096} REPS=${REPS:-1} bash tools/ab.sh ${1:-r04} "mont_tri||" "canon_tri||--input-form canonical" "mont_syn||--air synthetic" "canon_syn||--input-form canonical --air synthetic"
