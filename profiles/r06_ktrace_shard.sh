#!/bin/bash
# rocprofv3 kernel trace of one workload's per-rank shares (profiles/shard_scaling.py --ns <N>) per library
#   profiles/r06_ktrace_shard.sh <workload> <ns> <variant...>   ("default" = libgi.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
W=$1; NS=$2; shift 2
O=$R/gpurun_out/r06kts; mkdir -p $O
for V in "$@"; do
  if [ $V = default ]; then L=$R/2019global_amd/libgi.so; else L=$R/2019global_amd/_variants/libgi_$V.so; fi
  D=$O/${W}_n${NS}_$V
  ( cd /tmp && GI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/profiles/shard_scaling.py --workload $W --ns $NS > $D.log 2>&1 ) || { echo "ktrace fail $V"; tail -5 $D.log; exit 1; }
  python3 - "$D" "$V" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("void gi::(anonymous namespace)::", "").replace("gi::(anonymous namespace)::", "").split("(gi::")[0]
    print("%-10s %-60s calls %4d  avg %9.1f us  max %9.1f us" % (sys.argv[2], n[:60], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
done
