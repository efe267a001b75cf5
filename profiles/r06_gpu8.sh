cd $GRAFT_REPO_ROOT
bash profiles/r06.sh evidence 2 || exit $?
STEPS=10 bash profiles/r06.sh ab R-C4,R-C3 default spf
