#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then separate PMC passes
# (one counter group per run, never combined with other tracing domains), each under its own
# time limit; stops at the first failure.
# Usage: bash tools/profile_round.sh TAG [bench args...]   (outputs under gpurun_out/prof_TAG/)
set -o pipefail
TAG=${1:-r02}
shift || true
ARGS=${*:-"--steps 20 --warmup 5 --no-cpu --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --config1-seconds 0 --group-batches 0"}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# the library these counters belong to (bench.py attaches PMC figures only to a run of this library)
sha256sum neptune-core_amd/neptune_hip/libneptune_hip.so > $OUT/LIB_SHA256
# the config-4 proof pool, built once before any profiled process (oracle/pool4.py caches it in /tmp)
timeout -k 10 600 python3 -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
# the kernel trace of in-flight steps only (--iso-steps 0): trace_kernel_stats.csv's Merkle-hash average
# is then the bench roofline's own kernel_avg_ms; a second trace adds the one-at-a-time steps
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS --iso-steps 0 > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_iso -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace_iso.json 2> $OUT/trace_iso.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_valu -o pmc_valu --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_valu.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_cycles -o pmc_cycles --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_cycles.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc_fetch --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc_write --output-format csv -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err || exit 1
# the default bench line of this library, beside the profile
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python3 tools/summarize_profile.py $OUT > $OUT/SUMMARY.md && python3 tools/summarize_profile.py $OUT iso >> $OUT/SUMMARY.md
echo done
