#!/bin/bash
# Config-4 throughput of the current library vs a variant (NHIP_LIB), per-GPU shares SIZES,
# REPS alternating repetitions; GPU parity tests of the current library first.
# Usage: SIZES="4096 2048" REPS=3 bash tools/ab_lib_sizes.sh TAG VARIANT_SO [pytest -k expr]
set -o pipefail
OUT=gpurun_out/ab_$1; V=$2; mkdir -p $OUT
if [ -n "$3" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$3" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for rep in $(seq 1 ${REPS:-3}); do
for n in ${SIZES:-4096 2048 512}; do
for v in cur var; do
  if [ $v = var ]; then export NHIP_LIB=$PWD/$V; else unset NHIP_LIB; fi
  f=$OUT/n${n}_${v}_r$rep
  timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps ${STEPS:-200} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),'fs',b['phase_ms']['fiat_shamir'],b['verdicts_correct'])" $f.json n${n}_${v}_r$rep
done
done
done
