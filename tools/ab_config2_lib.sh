#!/bin/bash
set -o pipefail
# Config-2 (Tip5 Merkle auth paths) rate of the current library against variant libraries.
# Usage: bash tools/ab_config2_lib.sh TAG NAME ...  (NAME: neptune-core_amd/build/variants/libneptune_hip_NAME.so)
OUT=gpurun_out/ab_$1; shift; mkdir -p $OUT
for rep in 1 2; do for v in new "$@"; do
  if [ $v != new ]; then export NHIP_LIB=$PWD/neptune-core_amd/build/variants/libneptune_hip_$v.so; else unset NHIP_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs 64 --steps 1 --warmup 1 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --iso-steps 0 > $OUT/c2_${v}_r$rep.json 2> $OUT/c2_${v}_r$rep.err || { tail -5 $OUT/c2_${v}_r$rep.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));t=b['tip5_paths'];print(sys.argv[2],t['perms_per_s'],t['kernel_avg_ms'],t['verdicts_correct'])" $OUT/c2_${v}_r$rep.json c2_${v}_r$rep
done; done
