#!/bin/bash
# Small-batch latency (tools/latency.py) of the current library vs a variant (NHIP_LIB), REPS
# alternating repetitions.  Usage: bash tools/ab_latency_lib.sh TAG VARIANT_SO [REPS]
set -o pipefail
OUT=gpurun_out/ab_$1; V=$2; mkdir -p $OUT
for rep in $(seq 1 ${3:-2}); do
  for v in cur var; do
    if [ $v = var ]; then export NHIP_LIB=$PWD/$V; else unset NHIP_LIB; fi
    timeout -k 10 200 python -u tools/latency.py 30 > $OUT/lat_${v}_$rep.json 2> $OUT/lat_${v}_$rep.err || { tail -5 $OUT/lat_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],{k.split(' (')[0]:(v['resident_run_ms'],v['verify_batch_ms']) for k,v in d.items()})" $OUT/lat_${v}_$rep.json ${v}_$rep
  done
done
