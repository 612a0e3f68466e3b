#!/bin/bash
# computed S-box table (current) vs the table loaded from memory (variant), after the Tip5 / STARK GPU tests
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > /dev/null 2>&1 || exit 1
SIZES="512 4096" REPS=2 bash tools/ab_lib_sizes.sh r03d neptune-core_amd/build/variants/libneptune_hip_lutload.so "tip5 or stark or deep_fri or mast or pow"
# hardware-queue count sweep at 4,096 proofs (2 in flight): which queue count the pipeline needs
for q in 4 5 6 8; do
  f=gpurun_out/ab_r03d/hwq$q
  NHIP_BENCH_HWQ=$q timeout -k 10 200 python -u bench.py --no-cpu --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps 100 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['config']['gpu_max_hw_queues'],b['verdicts_correct'])" $f.json hwq$q
done
