#!/bin/bash
# One PMC pass (SQ_INSTS_VALU, SQ_WAVES, SQ_INSTS_LDS, SQ_INSTS_SALU) + kernel trace over a short bench run.
TAG=${1:-q}
OUT=$PWD/gpurun_out/pmcq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --config1-seconds 0 --group-batches 0 > $OUT/bench.json 2> $OUT/trace.err && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_valu -o pmc_valu --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --config1-seconds 0 --group-batches 0 > /dev/null 2> $OUT/pmc.err
python3 tools/summarize_profile.py $OUT | grep -v "SQ_WAVES\|SQ_INSTS_LDS\|SQ_INSTS_SALU" | grep -v rocclr
