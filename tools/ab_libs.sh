#!/bin/bash
# A/B of library builds (NHIP_LIB): config 4 at 4,096 proofs (2 in flight) and 512 proofs (4 in
# flight), then small-batch call latency; 2 alternating repetitions.  Usage: tools/ab_libs.sh TAG lib...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    for p in 4096 512; do
      f=$OUT/${n}_p${p}_r$rep
      NHIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $p --paths-log2 0 --stream-batches 0 --steps 30 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),round(b['phase_ms']['fiat_shamir'],3),round(b['roofline']['frac'],3),b['verdicts_correct'])" $f.json ${n}_p${p}_r$rep
    done
    if [ $rep = 1 ]; then
      NHIP_LIB=$lib timeout -k 10 200 python -u tools/latency.py 15 > $OUT/${n}_lat.log 2>&1 || { tail -5 $OUT/${n}_lat.log; exit 1; }
      head -4 $OUT/${n}_lat.log
    fi
  done
done
