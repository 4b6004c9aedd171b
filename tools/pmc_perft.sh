# VALU lane utilisation / mix of the perft kernels (diagnostic; one PMC pass)
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/pmc_perft -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 10 --warmup 10 --launched-steps 0 --perft-roots 8192 > gpurun_out/pmc_perft.log 2>&1 || { tail -5 gpurun_out/pmc_perft.log; exit 1; }
python - <<'PY'
import csv, collections
d = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open('gpurun_out/pmc_perft/run_counter_collection.csv')):
    k = r['Kernel_Name'].split('(')[0]
    d[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in d.items():
    if c['SQ_WAVES'] == 0 or c['SQ_ACTIVE_INST_VALU'] == 0:
        continue
    print(f"{k:28s} waves {c['SQ_WAVES']:10.0f} valu/wave {c['SQ_INSTS_VALU']/c['SQ_WAVES']:9.0f} "
          f"lane util {c['SQ_THREAD_CYCLES_VALU']/(c['SQ_ACTIVE_INST_VALU']*64):.3f} "
          f"busy {c['SQ_ACTIVE_INST_VALU']*4/(c['SQ_BUSY_CYCLES']*32):.3f} lds/wave {c['SQ_INSTS_LDS']/c['SQ_WAVES']:.0f} "
          f"wave_cycles/wave {4*c['SQ_WAVE_CYCLES']/c['SQ_WAVES']:.0f}")
PY
