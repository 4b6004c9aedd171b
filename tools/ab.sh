#!/bin/bash
# Same-box A/B of libgymchess.so builds, interleaved REPS times (one gpurun call).
#   LIBS="tools/_lib_a.so gym-chess_amd/gym_chess_amd/libgymchess.so" bash tools/ab.sh
#   an entry lib.so@VAR=VALUE runs that build with an environment switch
# MODE=step  (default) the headline fused rollout at K = 20 (the driver's shape) and K = 1000 (KS: other K)
# MODE=perft the perft leg (configs[3]: 65 536 mid-game roots, perft(5)) and its leaf kernel time
# MODE=var   the fused variants on the paired kernel: the random opponent (K=1), FIDE rules (K=2)
# MODE=api   the API-shaped device step (gc_env_step_device); apiv: its random-opponent form
# PARITY=1   first run tools/ab_parity.py for every build (rollout / step parity subset vs the oracle)
# PYTEST=1   first run the whole -m gpu suite on the in-tree build
# Variants are built here (tools/build_variants.sh); they ship to the box as tools/_lib_*.so,
# so delete them when the A/B is done.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "${PYTEST:-}" ] && { STEPS="pytest" bash tools/gpu_run.sh || exit $?; }
MODE=${MODE:-step}
if [ -n "${PARITY:-}" ]; then
  for lib in $LIBS; do
    so=${lib%%@*}; ev=""; [ "$so" != "$lib" ] && ev=$(echo "${lib#*@}" | tr "@" " ")
    env $ev timeout -k 10 300 python tools/ab_parity.py $so > gpurun_out/ab_parity.log 2>&1 || { echo "PARITY FAILED $lib"; tail -20 gpurun_out/ab_parity.log; exit 3; }
    echo "parity ok: $lib $(tail -1 gpurun_out/ab_parity.log)"
  done
fi
NOLEG="--no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0"
case $MODE in
  step)  KS=${KS:-"20 1000"}; ARGS="--warmup 5 $NOLEG --perft-roots 0" ;;
  perft) KS="5"; ARGS="--warmup 5 --settle 0 --no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --oracle-perft-roots 0" ;;
  var)   KS="5"; ARGS="--warmup 5 --no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 300 --perft-roots 0 --configs1-roots 0" ;;
  api|apiv) KS="5"; ARGS="--warmup 5 --settle 0 --no-cpu-baseline --launched-steps 0 --api-steps 200 --single-episodes 0 --variant-steps 0 --perft-roots 0" ;;
  *) echo "unknown MODE $MODE"; exit 2 ;;
esac
: > gpurun_out/ab.jsonl
for r in $(seq ${REPS:-3}); do
  for lib in $LIBS; do
    for k in $KS; do
      so=${lib%%@*}; ev=""; [ "$so" != "$lib" ] && ev=$(echo "${lib#*@}" | tr "@" " ")
      env $ev timeout -k 10 240 python tools/ab_lib.py $so --steps $k $ARGS > gpurun_out/ab_one.log 2>&1 || { echo "STOP $lib rc=$?"; tail -5 gpurun_out/ab_one.log; exit 3; }
      python - "$lib" "$MODE" >> gpurun_out/ab.jsonl <<'PY'
import json, sys
lib, mode = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open("gpurun_out/ab_one.log") if l.startswith("{")][-1])
if mode == "perft":
    p = d["perft"]
    print(json.dumps({"lib": lib, "k": 0, "value": p["value"], "aux": p["roofline"]["kernel_ms"], "nodes": p["nodes"]}))
elif mode == "var":  # the fused variants (k_env_rollout2): k = 1 the random opponent, 2 FIDE rules
    v = d["variants"]
    print(json.dumps({"lib": lib, "k": 1, "value": v["opponent_random"]["value"], "aux": 0}))
    print(json.dumps({"lib": lib, "k": 2, "value": v["rules_fide"]["value"], "aux": 0}))
elif mode in ("api", "apiv"):
    p = d["api_step"] if mode == "api" else d["api_step"]["opponent_random"]
    print(json.dumps({"lib": lib, "k": 0, "value": p["value"], "aux": p["roofline"]["avg_launch_us"]}))
else:
    print(json.dumps({"lib": lib, "k": d["steps"], "value": d["value"], "aux": d["event_ms_per_step"] * 1e3}))
PY
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
    e = sorted(x["aux"] for x in rs)
    nodes = sorted(set(x.get("nodes") for x in rs if x.get("nodes") is not None))
    print(f"{lib:55s} K={k:5d}: value {' '.join(f'{x:.3f}' for x in v)} e9 | aux {' '.join(f'{x:.3f}' for x in e)}"
          + (f" | nodes {nodes}" if nodes else ""))
PY
