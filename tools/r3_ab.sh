#!/bin/bash
# same-box A/B of libgymchess.so builds on the driver-shaped (--steps 20) and long (--steps 1000)
# headline lines, interleaved:  LIBS="tools/_lib_a.so gym-chess_amd/gym_chess_amd/libgymchess.so" bash tools/r3_ab.sh
# (an entry lib.so@VAR=VALUE runs that build with an environment switch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "${PYTEST:-}" ] && { STEPS="pytest" bash tools/gpu_run.sh || exit $?; }
B="--no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --perft-roots 0"
: > gpurun_out/ab.jsonl
for r in $(seq ${REPS:-3}); do
  for lib in $LIBS; do
    for k in 20 1000; do
      so=${lib%%@*}; ev=""; [ "$so" != "$lib" ] && ev=${lib#*@}  # lib@VAR=VALUE: the same build with an env switch
      env $ev timeout -k 10 200 python tools/ab_lib.py $so --steps $k --warmup 5 $B > gpurun_out/ab_one.log 2>&1 || { echo "STOP $lib rc=$?"; tail -5 gpurun_out/ab_one.log; exit 3; }
      python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_one.log') if l.startswith('{')][-1]); print(json.dumps({'lib': sys.argv[1], 'k': d['steps'], 'value': d['value'], 'ev_us': d['event_ms_per_step']*1e3}))" $lib >> gpurun_out/ab.jsonl
    done
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/ab.jsonl")]
g = collections.defaultdict(list)
for r in rows:
    g[(r["lib"], r["k"])].append(r)
for (lib, k), rs in sorted(g.items()):
    v = sorted(x["value"] / 1e9 for x in rs)
    e = sorted(x["ev_us"] for x in rs)
    print(f"{lib:50s} K={k:5d}: value {' '.join(f'{x:.3f}' for x in v)} e9 | event us/ply {' '.join(f'{x:.3f}' for x in e)}")
PY
