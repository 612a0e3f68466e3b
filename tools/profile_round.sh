#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then separate PMC passes
# (one counter group per run, never combined with other tracing domains).
# Usage: bash tools/profile_round.sh TAG [bench args...]   (outputs under gpurun_out/prof_TAG/)
set -e
TAG=${1:-r01}
shift || true
ARGS=${*:-"--steps 20 --warmup 3 --no-cpu"}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_valu -o pmc_valu --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_valu.err
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_cycles -o pmc_cycles --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_cycles.err
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc_fetch --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc_write --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err
echo done
