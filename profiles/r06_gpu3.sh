cd $GRAFT_REPO_ROOT
bash profiles/pcsample.sh C3 c3 10; echo "pcs C3 rc $?"
ls -la gpurun_out/pcs_c3/raw/*/ 2>/dev/null | head; find gpurun_out/pcs_c3 -name "*.csv" | head
