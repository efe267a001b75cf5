#!/bin/bash
# One rocprofv3 --pmc pass per quoted counter group (never combined with trace domains).
#   profiles/pmc.sh <tag> "<group1>" ["<group2>" ...] -- <bench args>
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
TAG=$1; shift; G=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do G+=("$1"); shift; done; shift
OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT; cd /tmp
i=0
for P in "${G[@]}"; do i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed ($P)"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "k_mode" in r["Kernel_Name"] and "<false>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()): print(f"{k:32s} {sum(v)/len(v):.4g}")
PY
