#!/bin/bash
# PMC passes over the Tip5 microbench for several library variants: issue / wait / fetch counters.
#   bash tools/pmc_tip5.sh TAG name1 name2 ...   ("main" = the in-tree library)
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/pmct_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = main ]; then L=$PWD/neptune-core_amd/neptune_hip/libneptune_hip.so; else L=$PWD/neptune-core_amd/build/variants/libneptune_hip_$v.so; fi
  export NHIP_LIB=$L
  timeout -k 10 120 python3 tools/tip5_micro.py 20 5 > $OUT/$v.json 2> $OUT/$v.err || { tail $OUT/$v.err; exit 1; }
  cat $OUT/$v.json
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d $OUT/$v -o p1 --output-format csv -- python3 tools/tip5_micro.py 20 2 > /dev/null 2> $OUT/$v.p1.err || { tail -5 $OUT/$v.p1.err; exit 1; }
done
unset NHIP_LIB
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    acc = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{out}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mtree_verify" not in r.get("Kernel_Name", ""):
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(v, {k: f"{acc[k] / max(n[k], 1):.4g}" for k in sorted(acc)})
PY
