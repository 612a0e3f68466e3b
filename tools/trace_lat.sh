#!/bin/bash
# rocprofv3 kernel trace of small resident batches (tools/lat_trace.py): 1 proof and 64 proofs.
set -o pipefail
OUT=$PWD/gpurun_out/trace_lat_$1; mkdir -p $OUT
export TMPDIR=/tmp
for n in ${NS:-1 64}; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/n$n -o trace --output-format csv -- python3 tools/lat_trace.py $n 20 > $OUT/n$n.log 2> $OUT/n$n.err || { tail -5 $OUT/n$n.err; exit 1; }
  cat $OUT/n$n.log
done
