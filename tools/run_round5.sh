cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
MODE=api LIBS="gym-chess_amd/gym_chess_amd/libgymchess.so tools/_lib_S1.so tools/_lib_S2.so" REPS=3 bash tools/ab.sh 2>&1 | tail -3
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench_full.log; exit $rc
