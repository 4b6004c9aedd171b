cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for v in "k0:X=1" "k1:HIP_FORCE_DEV_KERNARG=1" "k2:HIP_FORCE_DEV_KERNARG=0"; do
  n=${v%%:*}; ev=${v#*:}
  env $ev timeout -k 10 120 python bench.py --perft-roots 0 --no-cpu-baseline --fused-plies 0 > gpurun_out/$n.log 2>&1 || exit 1
  env $ev timeout -k 10 60 python tools/stamp_probe2.py > gpurun_out/st_$n.log 2>&1 || exit 1
done
python -c "
import json
for f in ('k0','k1','k2'):
    d=json.loads(open('gpurun_out/'+f+'.log').read().strip().splitlines()[-1]); print(f, d['value'], d['roofline']['avg_launch_us'])"
grep -h "load inputs\|span" gpurun_out/st_k*.log
