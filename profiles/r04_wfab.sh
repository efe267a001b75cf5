#!/bin/bash
# round 4: wavefront-form A/B over kernel variants (profiles/wf_probe.py, frames checked against k_mode_x)
#   profiles/r04_wfab.sh <workloads, comma> <variant>[:ENV=v,...] ...   (variant "default" = libgi.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04wfab; mkdir -p $O
WL=${1//,/ }; shift
for SPEC in "$@"; do
  V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
  if [ "$V" = default ]; then LIB=$GRAFT_REPO_ROOT/2019global_amd/libgi.so; else LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_$V.so; fi
  env GI_LIB=$LIB $E timeout -k 10 300 python3 -u profiles/wf_probe.py --steps 3 --warmup 1 $WL > $O/$V.jsonl 2> $O/$V.err || { echo "FAIL $SPEC"; tail -5 $O/$V.err; exit 1; }
  python3 - "$O/$V.jsonl" "$SPEC" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print("%-34s %-8s mega %8.3f  wf %8.3f  identical %s" % (sys.argv[2], d["workload"], d["mega"]["pass_ms"], d["wf"]["pass_ms"], d["identical"]), flush=True)
PY
done
