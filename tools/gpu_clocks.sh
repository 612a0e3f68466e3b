#!/bin/bash
# Shader clock and power while the default config-4 bench runs (rocm-smi sampled every ~0.5 s).
set -o pipefail
OUT=gpurun_out/clocks; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
rocm-smi --showclocks --showpower --showtemp > $OUT/idle.txt 2>&1
( for i in $(seq 1 120); do date +%s.%N; rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|Power|Temperature|mclk"; sleep 0.4; done ) > $OUT/samples.txt &
SMI=$!
timeout -k 10 300 python -u bench.py --no-cpu --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps 1500 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print(round(b['value']),b['ms_per_step'])"
grep -E "sclk" $OUT/samples.txt | sort | uniq -c | sort -rn | head -8
grep -iE "power" $OUT/samples.txt | head -4; grep -iE "power" $OUT/samples.txt | tail -4
exit $rc
