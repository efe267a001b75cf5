#!/bin/bash
# round 4: the GPU suite with the default form choice, then with each Mode X form forced on every
# launch (GI_X_WF=0 persistent kernel, 1 wavefront, 2 segment-synchronous)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04suite; mkdir -p $O
for F in default ${FORMS:-2 1 0}; do
  if [ $F = default ]; then E=""; else E="GI_X_WF=$F"; fi
  env $E timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite_$F.log 2>&1; rc=$?
  echo "suite $F: $(tail -1 $O/suite_$F.log)"
  [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/suite_$F.log | head -5; exit 1; }
done
