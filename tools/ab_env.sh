#!/bin/bash
# A/B of runtime environment settings on the default bench:  bash tools/ab_env.sh TAG ROUNDS "ENV=.." "ENV=.." ...
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python -u bench.py --no-cpu --paths-log2 0 > $OUT/v$i.$r.json 2> $OUT/v$i.$r.err || { tail $OUT/v$i.$r.err; exit 1; }
    python3 -c "import json;b=json.load(open('$OUT/v$i.$r.json'));p=b['phase_ms'];print('$v',round(b['ms_per_step'],3),'rf',round(b['roofline']['frac'],3),round(b['roofline']['kernel_avg_ms'],3),'rows',p['row_hash'],'hash',p['merkle_hash'],'ood',p['ood_air'],'fri',p['fri'],'deep',p['deep'],b['verdicts_correct'])"
  done
done
