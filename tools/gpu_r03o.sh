#!/bin/bash
# FixedLength-domain permutation (hash_pair with the capacity folded into round 0): every GPU test
# that hashes pairs (KAT-F, MTree, PoW, MAST, STARK multiproofs, config 4, deep FRI), then the A/B
# against HEAD (and a 4-wave build of k_mp_hash), and the config-2 Merkle-path microbench.
set -o pipefail
OUT=gpurun_out/${TAG:-r03o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_tip5.py tests/test_gpu_pow.py tests/test_gpu_mast.py tests/test_gpu_stark.py tests/test_gpu_config4.py tests/test_gpu_deep_fri.py tests/test_gpu_fs_forms.py tests/test_gpu_decode_fuzz.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
V=$PWD/neptune-core_amd/build/variants
SIZES="4096 512" REPS=3 STEPS=200 bash tools/ab_env_sizes.sh ${TAG:-r03o} "cur:" "head:NHIP_LIB=$V/libneptune_hip_head.so" || exit 1
for lib in cur head; do
  if [ $lib = head ]; then export NHIP_LIB=$V/libneptune_hip_head.so; else unset NHIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 --iso-steps 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --paths-log2 20 > $OUT/paths_$lib.json 2> $OUT/paths_$lib.err || exit 1
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],b['tip5_paths'])" $OUT/paths_$lib.json $lib
done
