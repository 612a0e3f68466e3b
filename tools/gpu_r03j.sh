#!/bin/bash
# Steps-in-flight default (8 below 4,096 proofs per GPU): the shares, configs 3 / 5, the default line,
# then the multi-rank rehearsal (2 ranks configs 3 / 4 with the default in-flight count; 8 ranks
# config 4) on one GPU over gloo.
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
Q="--no-cpu --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0"
run() { f=$OUT/$1.json; shift; timeout -k 10 300 python -u bench.py $Q "$@" > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1],round(b['value']),round(b['ms_per_step'],3),b['inflight'],b['verdicts_correct'])" $f; }
run c4_512 --proofs 512
run c4_1024 --proofs 1024
run c4_2048 --proofs 2048
run c3 --config 3
run c5_8 --config 5 --proofs 8
run c5_64 --config 5 --proofs 64
run c4_default
bash tools/rehearse_multirank.sh || exit 1
NHIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --steps 20 --warmup 2 --no-cpu \
  --paths-log2 0 --stream-batches 0 --config 4 --inflight 4 > $OUT/rehearse8.json 2> $OUT/rehearse8.err || { tail -30 $OUT/rehearse8.err; exit 1; }
python3 -c "import json;b=json.loads(open('$OUT/rehearse8.json').read().strip().splitlines()[-1]);print('8 ranks',b['n_gpus'],round(b['value']),b['verdicts_correct'],b['config']['proofs_rank0'])"
