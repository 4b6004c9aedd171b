# VALU mix / lane utilisation / dual issue of the step kernel (diagnostic; one PMC pass)
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 20 --warmup 400 --launched-steps 0 --perft-roots 0"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mix -o run --output-format csv -- $B > gpurun_out/pmc_mix.log 2>&1 || { tail -5 gpurun_out/pmc_mix.log; exit 1; }
python - <<'PY'
import csv, collections
d = collections.defaultdict(dict)
for r in csv.DictReader(open('gpurun_out/pmc_mix/run_counter_collection.csv')):
    if 'k_env_step2' in r['Kernel_Name']:
        d[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
ks = sorted(d)[-10:]
a = {c: sum(d[k][c] for k in ks) / len(ks) for c in d[ks[-1]]}
w = a['SQ_WAVES']
for c, v in sorted(a.items()):
    print(f"{c:24s} total {v:14.1f}  per wave {v / w:10.1f}")
print("lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*64)):", a['SQ_THREAD_CYCLES_VALU'] / (a['SQ_ACTIVE_INST_VALU'] * 64))
PY
