cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
A="python bench.py --no-cpu-baseline --steps 5 --warmup 5 --settle 200 --launched-steps 0 --api-steps 100 --single-episodes 0 --variant-steps 0 --perft-roots 0"
for nb in 65536; do
  timeout -k 10 120 $A --boards $nb > gpurun_out/api_n$nb.log 2>&1 || exit 3
  python -c "import json;d=json.loads([l for l in open('gpurun_out/api_n$nb.log') if l.startswith('{')][-1]);a=d['api_step'];print($nb, a['value']/1e9, a['roofline']['avg_launch_us'])"
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/apipmc_v -o run --output-format csv -- $A > /dev/null 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/apipmc_f -o run --output-format csv -- $A > /dev/null 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/apipmc_w -o run --output-format csv -- $A > /dev/null 2>&1 || exit 6
python - <<'PY'
import csv, glob, collections, json
res = collections.defaultdict(dict)
for tag in ("apipmc_v", "apipmc_f", "apipmc_w"):
    f = glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True)
    if not f: print(tag, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "api" not in k and "rollout4" not in k: continue
        agg[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(tag, k, {c: sum(v)/len(v) for c, v in cs.items()})
        for c, v in cs.items():
            res[k][c] = sum(v) / len(v)
# HBM bytes per launch (MI355X guide, gfx950: FETCH_SIZE KiB x2 + WRITE_SIZE KiB), 65 536 boards
out = {"boards": 65536, "note": "rocprofv3 PMC of the API legs of bench.py (100 steps each), FETCH_SIZE x2 + WRITE_SIZE per launch", "kernels": {}}
for k, cs in res.items():
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        b = cs["FETCH_SIZE"] * 1024 * 2 + cs["WRITE_SIZE"] * 1024
        name = k.replace("void ", "").split("(")[0].replace(" ", "")  # k_env_step_api4_vs<true> / <false> apart
        out["kernels"][name] = {"bytes_per_launch": b, "bytes_per_board": b / 65536,
                                "fetch_bytes": cs["FETCH_SIZE"] * 2048, "write_bytes": cs["WRITE_SIZE"] * 1024}
json.dump(out, open("gpurun_out/pmc_api.json", "w"), indent=1)
print(json.dumps(out))
PY
rm -rf gpurun_out/apipmc_*
