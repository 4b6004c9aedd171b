#!/bin/bash
# instruction classes of the fused launch (driver shape) + perft leaf PMC passes (current build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
PMCR="python bench.py --no-cpu-baseline --steps 20 --warmup 5 --launched-steps 0 --api-steps 0 --single-episodes 0 --perft-roots 0 --variant-steps 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc_cls -o run --output-format csv -- $PMCR > gpurun_out/pmc_cls.log 2>&1 || { echo "cls rc=$?"; tail -5 gpurun_out/pmc_cls.log; exit 1; }
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/pmc_cls/run_counter_collection.csv")))
k = [r for r in rows if "k_env_rollout2<false, 0>" in r.get("Kernel_Name", "")]
last = max(int(r["Dispatch_Id"]) for r in k)
v = collections.defaultdict(float)
for r in k:
    if int(r["Dispatch_Id"]) == last:
        v[r["Counter_Name"]] += float(r["Counter_Value"])
w = v["SQ_WAVES"]
print({c: round(x / w / 20, 1) for c, x in v.items()}, "per wave per ply (20 plies)")
PY
STEPS="pmcpf pmcpw" PROFILE_TAG=r03_v5 bash tools/gpu_run.sh
