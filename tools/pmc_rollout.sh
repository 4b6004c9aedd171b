# SQ counters of the fused rollout kernels (steady-state per-ply costs), diagnostic
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 50 --warmup 400 --launched-steps 0 --perft-roots 0"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  for v in "one:GC_STEP1=1" "pair:X=1"; do
    n=${v%%:*}; ev=${v#*:}
    env $ev timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmcr_${n}_$i -o run --output-format csv -- $B > gpurun_out/pmcr_${n}_$i.log 2>&1 || { tail -5 gpurun_out/pmcr_${n}_$i.log; exit 1; }
  done
done
python - <<'PY'
import csv, collections, glob
for path in sorted(glob.glob('gpurun_out/pmcr_*_*/run_counter_collection.csv')):
    d = collections.defaultdict(dict); names = {}
    for r in csv.DictReader(open(path)):
        if 'rollout' in r['Kernel_Name']:
            d[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value']); names[int(r['Dispatch_Id'])] = r['Kernel_Name'][:40]
    ks = sorted(d)[-1:]
    if not ks: print(path, 'no rows'); continue
    waves = d[ks[0]]['SQ_WAVES']
    print(path, names[ks[-1]], 'waves', waves, '(per wave per ply, 201-ply launch)')
    for c in d[ks[-1]]:
        if c != 'SQ_WAVES':
            print('   %-22s %10.1f' % (c, d[ks[0]][c] / waves / 200))
PY
