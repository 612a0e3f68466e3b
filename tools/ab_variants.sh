set -e
mkdir -p gpurun_out
for v in w3_g12 w3_g6 w4_g6 w4_g4 w3_g4; do
  NHIP_LIB=neptune-core_amd/build/variants/libneptune_hip_$v.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$v', round(d['roofline']['kernel_avg_ms'],3), 'ms', d['verdicts_correct'])"
done
