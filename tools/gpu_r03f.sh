#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo; 2 ranks configs 3 / 4 and 8 ranks config 4, the pool lock
# raced by every rank on a fresh box), then the round-3 profile of record.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rehearse; mkdir -p $OUT
NHIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --steps 20 --warmup 2 --no-cpu \
  --paths-log2 0 --stream-batches 0 --config 4 > $OUT/c4_8.json 2> $OUT/c4_8.err || { tail -30 $OUT/c4_8.err; exit 1; }
python3 -c "import json;b=json.loads(open('$OUT/c4_8.json').read().strip().splitlines()[-1]);print('8 ranks',b['n_gpus'],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'],b['scaling'],b['config']['proofs_rank0'])"
bash tools/rehearse_multirank.sh || exit 1
bash tools/profile_round.sh r03f || exit 1
