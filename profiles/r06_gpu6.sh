cd $GRAFT_REPO_ROOT
bash profiles/r06.sh suite; S=$?
echo "suite rc $S"
if [ $S -ne 0 ]; then exit $S; fi
STEPS=10 bash profiles/r06.sh ab R-C4,R-C3,R-main,C3 default base
