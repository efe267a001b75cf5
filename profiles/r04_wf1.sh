#!/bin/bash
# round 4: first wavefront Mode X run -- A/B probe (frames identical, times), then the GPU suite with
# the wavefront form forced on every Mode X launch (GI_X_WF=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04wf1; mkdir -p $O
timeout -k 10 300 python3 -u profiles/wf_probe.py --steps 10 C2 C3 > $O/probe_a.jsonl 2> $O/probe_a.err || { echo probe_a failed; tail -20 $O/probe_a.err; exit 1; }
cat $O/probe_a.jsonl
GI_X_WF=1 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite_wf.log 2>&1; rc=$?
tail -15 $O/suite_wf.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u profiles/wf_probe.py --steps 5 C4 X-soup1000 X-zoo X-main > $O/probe_b.jsonl 2> $O/probe_b.err || { echo probe_b failed; tail -20 $O/probe_b.err; exit 1; }
cat $O/probe_b.jsonl
