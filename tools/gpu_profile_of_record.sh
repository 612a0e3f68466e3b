#!/bin/bash
# The profile of record: GPU tests, smoke, tools/profile_round.sh (traces + PMC passes + the default
# bench line) and the driver's own command, under gpurun_out/<TAG>/ and gpurun_out/prof_<TAG>/.
# Usage: bash tools/gpu_profile_of_record.sh TAG   (then copy the summaries into profiles/<TAG>/)
set -o pipefail
TAG=${1:-r05z}
OUT=gpurun_out/$TAG; mkdir -p $OUT
# the box's clocks, power and temperature before anything runs (box-to-box spread of the rates)
rocm-smi --showclocks --showpower --showtemp --showmaxpower > $OUT/smi_idle.txt 2>&1 || true
bash tools/gpu_tests.sh $TAG && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
bash tools/profile_round.sh $TAG && \
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err && \
python3 -c "
import json; b=json.load(open('$OUT/bench_drv.json'))
print('value', round(b['value']), 'frac', round(b['roofline']['frac'],3), 'rows', b['roofline'].get('rows_kernel',{}).get('frac'), 'gs', round(b['group_stream']['value']), 'gsp', round(b['group_stream_pageable']['value']), 'share', round(b['share_n8']['value']), round(b['share_n8']['vs_value_per_proof'],3), 'prod', round(b['product_pipeline']['value']), 'c5', round(b['config5']['value']), 'c1', b['config1_latency']['gpu_resident_ms'], 'hwq', b['config']['gpu_max_hw_queues'], b['verdicts_correct'])"
