# SQ counter passes for the step kernels (one pass per counter group; each pass its own run)
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 20 --warmup 400 --launched-steps 0 --perft-roots 0"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  for v in "one:GC_STEP1=1" "pair:X=1"; do
    n=${v%%:*}; ev=${v#*:}
    env $ev timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc_${n}_$i -o run --output-format csv -- $B > gpurun_out/pmc_${n}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${n}_$i.log; exit 1; }
  done
done
python - <<'PY'
import csv, collections, glob
for path in sorted(glob.glob('gpurun_out/pmc_*_*/run_counter_collection.csv')):
    d = collections.defaultdict(dict); names = {}
    for r in csv.DictReader(open(path)):
        if 'k_env_step' in r['Kernel_Name']:
            d[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value']); names[int(r['Dispatch_Id'])] = r['Kernel_Name'][:40]
    ks = sorted(d)[-10:]
    if not ks: print(path, 'no rows'); continue
    waves = sum(d[k]['SQ_WAVES'] for k in ks) / len(ks)
    print(path, names[ks[-1]], 'waves', waves)
    for c in d[ks[-1]]:
        if c != 'SQ_WAVES':
            print('   %-22s per wave %10.1f' % (c, sum(d[k][c] for k in ks) / len(ks) / waves))
PY
