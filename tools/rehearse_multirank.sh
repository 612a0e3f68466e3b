#!/bin/bash
# Rehearse bench.py's multi-rank path on ONE GPU: 2 ranks, gloo collectives on host tensors
# (NHIP_DIST_BACKEND=gloo, NHIP_FINAL_BACKEND=gloo), configs 3 and 4.  The real N>1 runs end with one RCCL
# all-reduce over the N GPUs.
set -o pipefail
OUT=gpurun_out/rehearse; mkdir -p $OUT
for cfg in 3 4; do
  NHIP_DIST_BACKEND=gloo NHIP_FINAL_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29500 + cfg)) bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
    --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --group-batches 2 --config $cfg > $OUT/c$cfg.json 2> $OUT/c$cfg.err || { tail -30 $OUT/c$cfg.err; exit 1; }
  python3 -c "import json;b=json.loads(open('$OUT/c$cfg.json').read().strip().splitlines()[-1]);print($cfg,b['n_gpus'],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'],b['scaling'],b.get('group_stream'))"
done
