#!/bin/bash
# same-box A/B of libgymchess.so builds on the perft leg (configs[3]: 65 536 mid-game roots, perft(5))
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
P="--no-cpu-baseline --steps 5 --warmup 5 --settle 0 --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --oracle-perft-roots 0"
: > gpurun_out/perft_ab.jsonl
for r in $(seq ${REPS:-2}); do
  for lib in $LIBS; do
    so=${lib%%@*}; ev=""; [ "$so" != "$lib" ] && ev=${lib#*@}  # lib@VAR=VALUE: the same build with an env switch
    env $ev timeout -k 10 200 python tools/ab_lib.py $so $P > gpurun_out/pab_one.log 2>&1 || { echo "STOP $lib rc=$?"; tail -5 gpurun_out/pab_one.log; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/pab_one.log') if l.startswith('{')][-1])['perft']; print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'leaf_ms': d['roofline']['kernel_ms']}))" $lib >> gpurun_out/perft_ab.jsonl
  done
done
cat gpurun_out/perft_ab.jsonl
