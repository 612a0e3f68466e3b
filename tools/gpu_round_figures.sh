#!/bin/bash
# The round's headline figures at HEAD on one box: the default bench line (its PMC fields from
# profiles/LATEST), resident small-batch latency, the 512-proof per-GPU share (config 4 at N = 8)
# and one SQ_INSTS_VALU pass over that share.  Outputs under gpurun_out/figs_TAG/.
set -o pipefail
OUT=$PWD/gpurun_out/figs_${1:-x}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
timeout -k 10 200 python -u tools/latency.py 20 > $OUT/latency.json 2> $OUT/latency.err || { tail -5 $OUT/latency.err; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu --proofs 512 --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 > $OUT/bench_512.json 2> $OUT/bench_512.err || { tail -5 $OUT/bench_512.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc512 -o pmc_valu --output-format csv -- python3 bench.py --no-cpu --proofs 512 --paths-log2 0 --config5-proofs 0 --product-steps 0 --share-steps 0 --queue-callers 0 --stream-batches 0 --group-batches 0 --config1-seconds 0 > $OUT/bench_512_pmc.json 2> $OUT/pmc512.err || exit 1
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
b = json.load(open(f"{o}/bench_default.json"))
print("default", round(b["value"]), round(b["ms_per_step"], 3), b["roofline"]["frac"], b["roofline"].get("inflight", {}).get("frac"),
      b["valu_issue"], b["tip5_paths"]["perms_per_s"], b["cpu_baseline"]["value"], b["verdicts_correct"])
print("latency", open(f"{o}/latency.json").read().strip()[:400])
s = json.load(open(f"{o}/bench_512.json"))
print("512", round(s["value"]), round(s["ms_per_step"], 3), s["verdicts_correct"])
PY
