# I-cache counters for the step kernels (diagnostic)
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 20 --warmup 400 --launched-steps 0 --perft-roots 0"
for v in "pair:X=1" "one:GC_STEP1=1"; do
  n=${v%%:*}; ev=${v#*:}
  env $ev timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d gpurun_out/pmc_ic_$n -o run --output-format csv -- $B > gpurun_out/pmc_ic_$n.log 2>&1 || { tail -5 gpurun_out/pmc_ic_$n.log; exit 1; }
done
python - <<'PY'
import csv, collections, glob
for path in sorted(glob.glob('gpurun_out/pmc_ic_*/run_counter_collection.csv')):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if 'k_env_step' in r['Kernel_Name']:
            d[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
    ks = sorted(d)[-10:]
    print(path, {c: round(sum(d[k][c] for k in ks) / len(ks)) for c in d[ks[-1]]})
PY
