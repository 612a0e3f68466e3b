#!/bin/bash
# Host staging A/B (current library vs a variant, NHIP_LIB): small-batch call latency from pageable
# host buffers (tools/latency.py), the queue's 64-caller rate, streaming from pageable memory.
set -o pipefail
OUT=gpurun_out/ab_$1; V=$2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_stark.py tests/test_gpu_queue.py tests/test_gpu_group.py tests/test_gpu_callers.py tests/test_gpu_config4.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in cur var; do
    if [ $v = var ]; then export NHIP_LIB=$PWD/$V; else unset NHIP_LIB; fi
    timeout -k 10 200 python -u tools/latency.py 30 > $OUT/lat_${v}_$rep.json 2> $OUT/lat_${v}_$rep.err || { tail -5 $OUT/lat_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],{k.split(' (')[0]:(v['verify_batch_ms'],v['decode_ms'],v['upload_ms']) for k,v in d.items()})" $OUT/lat_${v}_$rep.json ${v}_$rep
    timeout -k 10 200 python -u -m pytest tests/test_gpu_queue.py -x -q -s -k coalescing_rate --timeout 200 --timeout-method thread 2>&1 | grep serialized | sed "s/^/${v}_$rep queue: /"
    timeout -k 10 300 python -u tools/stream_e2e.py 8 512 > $OUT/stream_${v}_$rep.json 2> $OUT/stream_${v}_$rep.err || { tail -5 $OUT/stream_${v}_$rep.err; exit 1; }
    echo "${v}_$rep stream $(cat $OUT/stream_${v}_$rep.json)"
  done
done
