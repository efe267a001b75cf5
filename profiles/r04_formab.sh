#!/bin/bash
# round 4: the three Mode X forms (k_mode_x / k_wf_bounce / k_seg) per workload and kernel variant;
# every form's frame checked bit for bit against k_mode_x's
#   profiles/r04_formab.sh <workloads, comma> <variant>[:ENV=v,...] ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04form; mkdir -p $O
WL=${1//,/ }; shift
for SPEC in "$@"; do
  V=${SPEC%%:*}; E=""; [[ "$SPEC" == *:* ]] && E=${SPEC#*:}; E=${E//,/ }
  if [ "$V" = default ]; then LIB=$GRAFT_REPO_ROOT/2019global_amd/libgi.so; else LIB=$GRAFT_REPO_ROOT/2019global_amd/_variants/libgi_$V.so; fi
  T=${V}_$(echo "$E" | tr ' =' '_-')
  env GI_LIB=$LIB $E timeout -k 10 400 python3 -u profiles/wf_probe.py --steps 3 --warmup 1 --forms ${FORMS:-mega,wf,seg} $WL > $O/$T.jsonl 2> $O/$T.err || { echo "FAIL $SPEC"; tail -5 $O/$T.err; exit 1; }
  python3 - "$O/$T.jsonl" "$SPEC" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    f = " ".join("%s %8.3f" % (k, d[k]["pass_ms"]) for k in ("mega", "wf", "seg") if k in d)
    print("%-30s %-11s %s  identical %s" % (sys.argv[2], d["workload"], f, d.get("identical")), flush=True)
PY
done
