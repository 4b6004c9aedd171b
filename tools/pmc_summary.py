#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/gpu_run.sh steps pmcf / pmcw / pmcv) for one kernel.

HBM traffic per launch, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
FETCH_SIZE (KiB) counts half the bytes of wide streaming reads -> x2; WRITE_SIZE (KiB) as is.
Writes <out>/pmc_traffic_latest.json (read by bench.py for roofline.traffic) and prints a table.

  python tools/pmc_summary.py gpurun_out profiles/r01_v7 [--kernel 'void k_env_step<true>'] [--last 20]
"""
import argparse
import collections
import csv
import json
import os


def per_dispatch(path, kernel):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--kernel", default="void k_env_step<true>")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--alg-bytes-per-board", type=int, default=282)
    ap.add_argument("--dispatches-per-ply", type=int, default=1,
                    help="dispatches of the kernel per ply (bench.py's board-range streams, GC_STREAMS)")
    ap.add_argument("--perft", action="store_true",
                    help="perft leaf kernel (k_perft2_perm) passes pmc_perft_{fetch,write,mix} -> pmc_perft.json")
    a = ap.parse_args()
    if a.perft:
        return perft_summary(a)
    mean = lambda rows, k: sum(r[k] for r in rows) / len(rows)  # noqa: E731
    f = per_dispatch(os.path.join(a.src, "pmc_fetch/run_counter_collection.csv"), a.kernel)[-a.last:]
    w = per_dispatch(os.path.join(a.src, "pmc_write/run_counter_collection.csv"), a.kernel)[-a.last:]
    k = a.dispatches_per_ply
    fetch = mean(f, "FETCH_SIZE") * 1024 * 2 * k
    write = mean(w, "WRITE_SIZE") * 1024 * k
    out = {"kernel": a.kernel, "launches_averaged": len(f), "boards": a.boards, "dispatches_per_ply": k,
           "fetch_bytes_corrected": fetch, "fetch_size_kib_raw": mean(f, "FETCH_SIZE") * k, "write_bytes": write,
           "bytes_per_launch": fetch + write, "bytes_per_board": (fetch + write) / a.boards,
           "alg_bytes_per_launch": a.alg_bytes_per_board * a.boards,
           "note": "per ply (all boards; the sum of its dispatches); FETCH_SIZE x2 (gfx950 correction for wide "
                   "streaming reads; 8-B/lane loads uncalibrated)"}
    vp = os.path.join(a.src, "pmc_valu/run_counter_collection.csv")
    if os.path.exists(vp):
        v = per_dispatch(vp, a.kernel)[-a.last:]
        waves = mean(v, "SQ_WAVES")
        sq = {k: mean(v, k) / waves for k in v[0] if k != "SQ_WAVES"}
        out["per_wave"] = sq
        out["per_wave"]["note"] = "SQ_*_CYCLES / WAIT / ACTIVE in units of 4 cycles (quad-cycles)"
    mp = os.path.join(a.src, "pmc_mix/run_counter_collection.csv")
    if os.path.exists(mp):  # VALU utilisation (SURVEY 8d asks for it beside the HBM figure)
        v = per_dispatch(mp, a.kernel)[-a.last:]
        waves = mean(v, "SQ_WAVES")
        simds_per_se = 1024 / 32  # MI355X: 256 CUs x 4 SIMDs over 8 XCDs x 4 SEs
        out["valu"] = {
            "insts_per_wave": mean(v, "SQ_INSTS_VALU") / waves,
            "lane_utilisation": mean(v, "SQ_THREAD_CYCLES_VALU") / (mean(v, "SQ_ACTIVE_INST_VALU") * 64),
            "busy_frac": mean(v, "SQ_ACTIVE_INST_VALU") * 4 / (mean(v, "SQ_BUSY_CYCLES") * simds_per_se),
            "note": "busy_frac = SQ_ACTIVE_INST_VALU x 4 cycles / (SQ_BUSY_CYCLES x SIMDs per SE), whole launch "
                    "incl. ramp and tail; lane_utilisation = active lanes per VALU instruction / 64",
        }
    bl = bench_line(os.path.join(a.src, "pmcf.log"))
    if bl:  # the steady state the counters describe
        out["mean_window"] = bl["roofline"]["mean_window"]
        out["settle_plies"] = bl["config"].get("settle_plies")
    out["profile"] = os.path.basename(a.dst.rstrip("/"))
    os.makedirs(a.dst, exist_ok=True)
    for p in (os.path.join(a.dst, "pmc_traffic.json"),):
        json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


def bench_line(path):
    try:
        for ln in reversed(open(path).read().splitlines()):
            if ln.startswith("{"):
                return json.loads(ln)
    except (OSError, ValueError):
        pass
    return None


def perft_summary(a):
    """k_perft2_perm (the split leaf pass: one lane = one depth-2 subtree, bulk-counted last
    ply) over the bench's perft leg.  Per launch: HBM bytes (FETCH_SIZE x2 + WRITE_SIZE),
    VALU instructions per wave, lane utilisation, VALU busy fraction.  Algorithmic bytes per
    subtree: the root's 7 bitboards + meta (60) + its permutation index (4) read, its count
    (8) written = 72 B; the leaves never touch memory."""
    kern = "k_perft2_perm"
    rows = lambda sub: per_dispatch(os.path.join(a.src, sub, "run_counter_collection.csv"), kern)  # noqa: E731
    f, w, m = rows("pmc_perft_fetch"), rows("pmc_perft_write"), rows("pmc_perft_mix")
    tot = lambda rs, k: sum(r[k] for r in rs)  # noqa: E731
    waves = tot(m, "SQ_WAVES")
    simds_per_se = 1024 / 32
    out = {"kernel": kern, "launches": len(m),
           "hbm_bytes_total": tot(f, "FETCH_SIZE") * 1024 * 2 + tot(w, "WRITE_SIZE") * 1024,
           "subtrees_total": waves * 64,
           "alg_bytes_per_subtree": 72,
           "valu": {"insts_per_wave": tot(m, "SQ_INSTS_VALU") / waves,
                    "lane_utilisation": tot(m, "SQ_THREAD_CYCLES_VALU") / (tot(m, "SQ_ACTIVE_INST_VALU") * 64),
                    "busy_frac": tot(m, "SQ_ACTIVE_INST_VALU") * 4 / (tot(m, "SQ_BUSY_CYCLES") * simds_per_se),
                    "lds_insts_per_wave": tot(m, "SQ_INSTS_LDS") / waves,
                    "salu_insts_per_wave": tot(m, "SQ_INSTS_SALU") / waves},
           "profile": os.path.basename(a.dst.rstrip("/"))}
    out["hbm_bytes_per_subtree"] = out["hbm_bytes_total"] / max(out["subtrees_total"], 1)
    os.makedirs(a.dst, exist_ok=True)
    for p in (os.path.join(a.dst, "pmc_perft.json"),):
        json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
