#!/bin/bash
# rocprofv3 --kernel-trace --stats of any python3 command (run from the repo root on the GPU box),
# printing every kernel's calls and average duration:
#   profiles/ktrace_cmd.sh <tag> <python args...>
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
D=$R/gpurun_out/kt_$TAG
mkdir -p $D
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 "$@" > $D.log 2>&1 ) || { echo "ktrace fail $TAG"; tail -5 $D.log; exit 1; }
python3 - "$D" "$TAG" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(gi::.*|\(unsigned.*", "", r["Name"].replace("void gi::(anonymous namespace)::", "").replace("gi::(anonymous namespace)::", ""))
    print("%-12s %-50s calls %5d  avg %9.1f us  total %9.1f us" % (sys.argv[2], n[:50], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
