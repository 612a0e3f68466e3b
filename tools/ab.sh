#!/bin/bash
# A/B of variants over config-4 per-GPU shares, REPS alternating repetitions (one bench line per
# variant x size x repetition, printed as it finishes).  A variant is "name|ENV=v ...|bench args":
# environment (NHIP_LIB=path selects a variant library, see build_variant.sh / build_head_variant.sh)
# and extra bench.py arguments, either part may be empty.
# Usage: SIZES="4096 512" REPS=2 STEPS=200 bash tools/ab.sh TAG "base||" "mont||--input-form montgomery" \
#          "old|NHIP_LIB=neptune-core_amd/build/variants/libneptune_hip_head.so|"
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for n in ${SIZES:-4096 512}; do
for spec in "$@"; do
  IFS='|' read -r name envs extra <<< "$spec"
  f=$OUT/n${n}_${name}_r$rep
  env $envs timeout -k 10 300 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 \
    --config1-seconds 0 --group-batches 0 --steps ${STEPS:-200} $extra > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "
import json, sys
b = json.load(open(sys.argv[1]))
r = b['roofline']
print(sys.argv[2], round(b['value']), round(b['ms_per_step'], 3), 'rf', round(r['frac'], 3),
      'inflight', round(r.get('inflight', r)['frac'], 3), 'ood', b['phase_ms']['ood_air'], b['verdicts_correct'])" \
    $f.json n${n}_${name}_r$rep
done
done
done
