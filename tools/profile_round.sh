#!/bin/bash
# rocprofv3 passes for the bench workload (kernel trace + stats, then separate PMC passes).
# Usage: bash tools/profile_round.sh TAG   (outputs under gpurun_out/prof_TAG/)
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--steps 5 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc1 -o pmc1 --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc1.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc2 -o pmc2 --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc2.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o pmc3 --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc3.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o pmc4 --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc4.err
echo done
