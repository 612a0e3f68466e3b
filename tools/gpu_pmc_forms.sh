#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES and a kernel trace of the config-4 bench with each sponge-replay form.
set -o pipefail
OUT=$PWD/gpurun_out/pmc_forms; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu --config 4 --proofs ${N:-4096} --paths-log2 0 --stream-batches 0 --hwq4-steps 0 --config1-seconds 0 --steps 20 --iso-steps 2"
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'oracle'); import pool4; pool4.load()" > $OUT/pool4.log 2>&1 || exit 1
for f in ${FORMS:-row quad}; do
  NHIP_FS_FORM=$f timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/pmc_$f -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$f.json 2> $OUT/pmc_$f.err || exit 1
  NHIP_FS_FORM=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$f -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/trace_$f.json 2> $OUT/trace_$f.err || exit 1
done
python3 - <<PY
import csv,glob,collections,os
out="$OUT"
for f in "${FORMS:-row quad}".split():
    tot=collections.defaultdict(float); n=collections.Counter()
    for r in csv.DictReader(open(glob.glob(f"{out}/pmc_{f}/**/*counter_collection.csv",recursive=True)[0])):
        k=(r["Kernel_Name"].split("(")[0][:40],r["Counter_Name"]); tot[k]+=float(r["Counter_Value"]); n[k]+=1
    for k in sorted(tot):
        if k[1]=="SQ_INSTS_VALU": print(f,k[0],f"{tot[k]/n[k]:.4g}",n[k])
    st=glob.glob(f"{out}/trace_{f}/**/*kernel_stats.csv",recursive=True)[0]
    for r in csv.DictReader(open(st)):
        print(f,"trace",r["Name"].split("(")[0][:40],r["Calls"],round(float(r["AverageNs"])/1e6,3))
PY
