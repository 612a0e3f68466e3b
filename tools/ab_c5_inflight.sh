set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c5; mkdir -p $OUT
for rep in 1 2; do for n in 8 64; do for r in 8 10; do
  f=$OUT/n${n}_r${r}_$rep.json
  timeout -k 10 200 python -u bench.py --no-cpu --config 5 --proofs $n --inflight $r --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
  python3 -c "import json,sys;b=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1],round(b['value']),round(b['ms_per_step'],3),b['verdicts_correct'])" $f
done; done; done
