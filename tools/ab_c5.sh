set -o pipefail
OUT=gpurun_out/ab_c5; mkdir -p $OUT
for rep in 1 2 3; do
for v in prelat head; do
  if [ $v = prelat ]; then export NHIP_LIB=$PWD/neptune-core_amd/build/variants/libneptune_hip_prelat.so; else unset NHIP_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu --config 5 > $OUT/c5_${v}_$rep.json 2> $OUT/c5_${v}_$rep.err || { tail -5 $OUT/c5_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['phase_ms'],b['verdicts_correct'])" $OUT/c5_${v}_$rep.json c5_${v}_$rep
done
done
