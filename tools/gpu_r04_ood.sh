set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
bash tools/gpu_tests.sh r04d || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q -s --timeout 200 --timeout-method thread > $OUT/queue.log 2>&1 || { tail -20 $OUT/queue.log; exit 1; }
grep -E "serialized|queue per batch" $OUT/queue.log
H=$PWD/neptune-core_amd/build/variants/libneptune_hip_head.so
SIZES="4096 512" REPS=1 bash tools/ab.sh r04d "lvl|NHIP_LIB=$H|" "w512||" "w256|NHIP_OOD_STEP_WIDTH=256|" "w1024|NHIP_OOD_STEP_WIDTH=1024|" || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench_default.json'));print('default',round(b['value']),b['ms_per_step'],b['phase_ms'],b['roofline']['frac'],b['group_stream']['value'],b['verdicts_correct'])"
