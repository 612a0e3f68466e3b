#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (default config), outputs under gpurun_out/trace_TAG/.
set -o pipefail
TAG=${1:-c4}
shift || true
ARGS=${*:-"--steps 20 --warmup 3 --no-cpu --paths-log2 0"}
OUT=$PWD/gpurun_out/trace_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?
python3 tools/summarize_profile.py $OUT > $OUT/SUMMARY.md 2>/dev/null
head -40 $OUT/SUMMARY.md
exit $rc
