cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/ab_libs.sh m1w4 m2 w4 w1 && bash tools/ab_libs.sh m2 m1w4
