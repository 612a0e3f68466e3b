set -o pipefail
OUT=gpurun_out/ab_lat; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_stark.py tests/test_gpu_config5.py tests/test_gpu_callers.py tests/test_gpu_queue.py tests/test_gpu_stark_params.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for v in old new; do
  if [ $v = old ]; then export NHIP_LIB=$PWD/neptune-core_amd/build/variants/libneptune_hip_old.so; else unset NHIP_LIB; fi
  timeout -k 10 200 python -u tools/latency.py 20 > $OUT/lat_${v}_$rep.json 2> $OUT/lat_${v}_$rep.err || { tail -5 $OUT/lat_${v}_$rep.err; exit 1; }
  echo "$v lat $(cat $OUT/lat_${v}_$rep.json)"
  for n in 512 4096; do
    timeout -k 10 200 python -u bench.py --no-cpu --config 4 --proofs $n --paths-log2 0 --stream-batches 0 > $OUT/c4_${n}_${v}_$rep.json 2> $OUT/c4_${n}_${v}_$rep.err || { tail -5 $OUT/c4_${n}_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['phase_ms']['fiat_shamir'],b['verdicts_correct'])" $OUT/c4_${n}_${v}_$rep.json c4_${n}_${v}_$rep
  done
  for n in 8 64; do
    timeout -k 10 200 python -u bench.py --no-cpu --config 5 --proofs $((n*8)) --paths-log2 0 --stream-batches 0 > $OUT/c5_${n}_${v}_$rep.json 2> $OUT/c5_${n}_${v}_$rep.err || true
    python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[2],round(b['value']),round(b['ms_per_step'],3),b['phase_ms']['fiat_shamir'],b['verdicts_correct'])" $OUT/c5_${n}_${v}_$rep.json c5_${n}_${v}_$rep 2>/dev/null || echo "c5 $n $v failed"
  done
done
done
