#!/bin/bash
# PMC of the perft leg's kernels (the transposition pass -- k_dedup_keys, the radix sort, k_dedup_runs (or k_dedup_bin) -- and the leaf): SQ mix, fetch, write
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
P="python bench.py --no-cpu-baseline --steps 5 --warmup 5 --settle 0 --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --oracle-perft-roots 0"
MIXC="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
timeout -s KILL 120 rocprofv3 --pmc $MIXC -d gpurun_out/pd_v -o run --output-format csv -- $P > /dev/null 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pd_f -o run --output-format csv -- $P > /dev/null 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pd_w -o run --output-format csv -- $P > /dev/null 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pd_s -o run --output-format csv -- $P > /dev/null 2>&1 || exit 7
python - <<'PY'
import csv, glob, collections
for tag in ("pd_v", "pd_f", "pd_w"):
    f = glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0]
        if not any(x in k for x in ("dedup", "perft2_val", "place_leaders", "followers", "expand_range_rec", "leader_hist", "Onesweep", "onesweep", "radix", "Radix", "count_children", "scan", "Scan")): continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(tag, k, {c: round(sum(v)/len(v)) for c, v in cs.items()})
f = glob.glob("gpurun_out/pd_s/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if any(x in r["Name"] for x in ("dedup", "perft2_val", "place_leaders", "followers", "expand_range_rec", "leader_hist", "Onesweep", "onesweep", "radix", "Radix", "count_children", "scan", "Scan")):
        print("stats", r["Name"].split("(")[0][:60], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY
rm -rf gpurun_out/pd_*
