#!/bin/bash
# One gpurun session: each GPU step under its own timeout; stop at the first fault,
# abort, segfault, timeout or hang (any exit code other than 0 / 1 = test failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/steps.log
step() {
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.log
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
}
# PMC passes time the bench's own steady-state launches (bench defaults: --settle 1000
# --warmup 50), 20 of them; one counter group per pass (rocprofv3 does not split passes)
PMCB="python bench.py --no-cpu-baseline --steps 20 --launched-steps 20 --api-steps 0 --single-episodes 0 --perft-roots 0 --variant-steps 0"
# the headline: the driver's own shape (--steps 20 --warmup 5), the fused launch of 20 steps is
# the LAST k_env_rollout4 dispatch of the process
PMCR="python bench.py --no-cpu-baseline --steps 20 --warmup 5 --launched-steps 0 --api-steps 0 --single-episodes 0 --perft-roots 0 --variant-steps 0"
PMCRL="python bench.py --no-cpu-baseline --steps 1000 --warmup 5 --launched-steps 0 --api-steps 0 --single-episodes 0 --perft-roots 0 --variant-steps 0"  # the K = 1 000 line
MIXC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
# perft passes: the bench's perft leg (65 536 mid-game FEN roots, perft(5)) without the step legs
PERFTB="python bench.py --no-cpu-baseline --steps 5 --warmup 5 --settle 0 --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --oracle-perft-roots 0"
for s in ${STEPS:-smoke pytest bench prof}; do
  case $s in
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) step pytest 1100 python -u -m pytest ${PYTEST_ARGS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread ;;  # PYTEST_ARGS: a subset
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --oracle-perft-roots 0 ;;  # bench defaults: the same launches bench.py times
    profs)  step profs 300 rocprofv3 --kernel-trace --stats -d $OUT/profs -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --oracle-perft-roots 0 ;;  # the driver's command
    pmcf)   step pmcf 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $PMCB ;;
    pmcw)   step pmcw 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $PMCB ;;
    pmcv)   step pmcv 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_valu -o run --output-format csv -- $PMCB ;;
    pmcm)   step pmcm 300 rocprofv3 --pmc $MIXC -d $OUT/pmc_mix -o run --output-format csv -- $PMCB ;;
    pmcpf)  step pmcpf 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_perft_fetch -o run --output-format csv -- $PERFTB ;;
    pmcpw)  step pmcpw 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_perft_write -o run --output-format csv -- $PERFTB ;;
    pmcpm)  step pmcpm 300 rocprofv3 --pmc $MIXC -d $OUT/pmc_perft_mix -o run --output-format csv -- $PERFTB ;;
    pmcrf)  step pmcrf 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_roll_fetch -o run --output-format csv -- $PMCR ;;
    pmcrw)  step pmcrw 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_roll_write -o run --output-format csv -- $PMCR ;;
    pmcrm)  step pmcrm 300 rocprofv3 --pmc $MIXC -d $OUT/pmc_roll_mix -o run --output-format csv -- $PMCR ;;
    pmcrl)  step pmcr_longf 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_roll_long_fetch -o run --output-format csv -- $PMCRL &&
            step pmcr_longw 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_roll_long_write -o run --output-format csv -- $PMCRL &&
            step pmcr_longm 300 rocprofv3 --pmc $MIXC -d $OUT/pmc_roll_long_mix -o run --output-format csv -- $PMCRL ;;
    perftab) step perft_dedup 300 $PERFTB --perft-roots 65536 &&  # the perft leg, transpositions merged / not
            GC_PERFT_DEDUP=0 step perft_every 300 $PERFTB --perft-roots 65536 ;;
    profp)  step profp 300 rocprofv3 --kernel-trace --stats -d $OUT/profp -o run --output-format csv -- $PERFTB &&
            cp $OUT/profp/run_kernel_stats.csv $OUT/perft_kernel_stats.csv ;;  # the perft leg's kernels
    fcp)    step fcp 300 python tools/fixed_cost_probe.py ;;  # the timed region's fixed cost, by K and wait
    anat)   step anat 120 tools/_region_anatomy ;;  # one launch's round trip by parts (build it first)
    pst)    for k in 20 1000; do PST_QUAD=1 PST_LIB=tools/_lib_pst.so step pst_$k 120 python tools/pstamp_probe.py 65536 $k; done ;;  # wave placement / phase stamps (build tools/_lib_pst.so with -DGC_PSTAMPS first)
    sprobe) step single_probe 300 python tools/single_probe.py ;;
    soak)   step soak 800 python -u tools/soak.py --plies ${SOAK_PLIES:-20000} --chunk 2000 --seeds ${SOAK_SEEDS:-10} ;;  # long rollouts vs the oracle  # the single-board server's step and segments vs the oracle
    eprobe) step engine_probe 120 python tools/engine_probe.py &&  # ChessEngine per-call latency: server / staged in host memory / copies
            GC_ENGINE_SERVER=0 step engine_probe_zc 120 python tools/engine_probe.py &&
            GC_ENGINE_SERVER=0 GC_ENGINE_ZC=0 step engine_probe_staged 120 python tools/engine_probe.py ;;
    calib)  step calib 120 rocprofv3 --pmc $MIXC -d $OUT/pmc_calib -o run --output-format csv -- tools/_valu_calib ;;
    short)  for i in 1 2 3; do step short$i 300 python bench.py --gpus 1 --steps 20 --warmup 5; done
            step long 300 python bench.py --gpus 1 --steps 1000 --warmup 5 --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --perft-roots 0 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
# summaries on the box (the raw per-dispatch CSVs stay here: gpurun returns <= 64 MiB)
if [ -n "${PROFILE_TAG:-}" ]; then
  mkdir -p $OUT/summary/$PROFILE_TAG
  [ -f $OUT/prof/run_kernel_stats.csv ] && cp $OUT/prof/run_kernel_stats.csv $OUT/summary/$PROFILE_TAG/kernel_stats.csv
  [ -f $OUT/profs/run_kernel_stats.csv ] && cp $OUT/profs/run_kernel_stats.csv $OUT/summary/$PROFILE_TAG/kernel_stats_driver_cmd.csv
  [ -d $OUT/pmc_calib ] && python tools/pmc_summary.py $OUT $OUT/summary/$PROFILE_TAG --calib > /dev/null
  [ -f $OUT/pmc_calib/run_counter_collection.csv ] && cp $OUT/pmc_calib/run_counter_collection.csv $OUT/summary/$PROFILE_TAG/calib_counters.csv
  [ -d $OUT/pmc_fetch ] && python tools/pmc_summary.py $OUT $OUT/summary/$PROFILE_TAG --kernel "k_env_step2<false, 0>" --dispatches-per-ply ${GC_STREAMS:-2} > /dev/null
  [ -d $OUT/pmc_perft_fetch ] && python tools/pmc_summary.py $OUT $OUT/summary/$PROFILE_TAG --perft > /dev/null
  [ -d $OUT/pmc_roll_fetch ] && python tools/pmc_summary.py $OUT $OUT/summary/$PROFILE_TAG --rollout > /dev/null
  [ -d $OUT/pmc_roll_long_fetch ] && python tools/pmc_summary.py $OUT $OUT/summary/$PROFILE_TAG --rollout --roll-tag _long > /dev/null
  for f in short1 short2 short3 long; do [ -f $OUT/$f.log ] && grep '^{' $OUT/$f.log | tail -1 > $OUT/summary/$PROFILE_TAG/$f.json; done
  for f in bench pmcf; do [ -f $OUT/$f.log ] && grep '^{' $OUT/$f.log | tail -1 > $OUT/summary/$PROFILE_TAG/$f.json; done
  rm -rf $OUT/prof $OUT/profs $OUT/pmc_*
fi
echo ALLDONE
