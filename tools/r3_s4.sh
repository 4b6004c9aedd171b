#!/bin/bash
# GC_FAIR A/B: launch anatomy with and without the per-CU feedback priority, driver-shaped and
# long bench lines interleaved, the GPU suite on the default (GC_FAIR=1) build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local n=$1 s=$2; shift 2; timeout -k 10 "$s" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; tail -${TAILN:-6} gpurun_out/$n.log; [ $rc -eq 0 ] || { echo "STOP $n rc=$rc"; exit $rc; }; }
TAILN=4 PST_LIB=tools/_lib_pstnf.so run pst20_nf 120 python tools/pstamp_probe.py 65536 20
TAILN=4 PST_LIB=tools/_lib_pst.so run pst20_f 120 python tools/pstamp_probe.py 65536 20
TAILN=4 PST_LIB=tools/_lib_pstnf.so run pst1000_nf 120 python tools/pstamp_probe.py 65536 1000
TAILN=4 PST_LIB=tools/_lib_pst.so run pst1000_f 120 python tools/pstamp_probe.py 65536 1000
B="--no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --perft-roots 0"
for r in 1 2 3; do
  TAILN=1 run ab_s_nf$r 200 python tools/ab_lib.py tools/_lib_nofair.so --steps 20 --warmup 5 $B
  TAILN=1 run ab_s_f$r 200 python tools/ab_lib.py gym-chess_amd/gym_chess_amd/libgymchess.so --steps 20 --warmup 5 $B
done
for r in 1 2; do
  TAILN=1 run ab_l_nf$r 200 python tools/ab_lib.py tools/_lib_nofair.so --steps 1000 --warmup 5 $B
  TAILN=1 run ab_l_f$r 200 python tools/ab_lib.py gym-chess_amd/gym_chess_amd/libgymchess.so --steps 1000 --warmup 5 $B
done
STEPS="pytest" bash tools/gpu_run.sh
