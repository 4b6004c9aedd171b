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
                    help="perft leaf kernel (--perft-kernel) passes pmc_perft_{fetch,write,mix} -> pmc_perft.json")
    ap.add_argument("--rollout", action="store_true",
                    help="the headline kernel (last dispatch of --rollout-kernel) passes pmc_roll_* -> pmc_rollout.json")
    ap.add_argument("--perft-kernel", default="k_perft2_val",
                    help="the split leaf kernel (k_perft2_rec: GC_PERFT_DEDUP=0, k_perft2_perm_rec: GC_PERFT_GATHER)")
    ap.add_argument("--rollout-kernel", default="k_env_rollout4",
                    help="the fused rollout's kernel: k_env_rollout4 (quads), k_env_rollout2<false, 0> (pairs)")
    ap.add_argument("--roll-tag", default="",
                    help="the rollout passes' directory tag: pmc_roll<TAG>_* -> pmc_rollout<TAG>.json (_long: K = 1000)")
    ap.add_argument("--calib", action="store_true",
                    help="tools/_valu_calib under the mix counters (pmc_calib + calib.log) -> valu_calib.json")
    a = ap.parse_args()
    if a.calib:
        return calib_summary(a)
    if a.perft:
        return perft_summary(a)
    if a.rollout:
        return rollout_summary(a)
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
        out["valu"] = {
            "insts_per_wave": mean(v, "SQ_INSTS_VALU") / waves,
            "lane_utilisation": mean(v, "SQ_THREAD_CYCLES_VALU") / (mean(v, "SQ_ACTIVE_INST_VALU") * 64),
            "wait_any_share": mean(v, "SQ_WAIT_ANY") / mean(v, "SQ_WAVE_CYCLES"),
            "note": "lane_utilisation = active lanes per VALU instruction / 64; issue_frac: calibrated class costs "
                    "(tools/valu_calib.hip) over SIMDs x dispatch cycles (GRBM_GUI_ACTIVE / XCDs)",
        }
        cal = load_calib(a.dst)
        if cal:
            out["valu"].update(valu_issue({k: mean(v, k) for k in v[0]}, cal))
    bl = bench_line(os.path.join(a.src, "pmcf.log"))
    if bl:  # the steady state the counters describe
        out["mean_window"] = bl["roofline"]["mean_window"]
        out["settle_plies"] = bl["config"].get("settle_plies")
    out["profile"] = os.path.basename(a.dst.rstrip("/"))
    os.makedirs(a.dst, exist_ok=True)
    for p in (os.path.join(a.dst, "pmc_traffic.json"),):
        json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


SIMDS = 1024  # MI355X: 256 CUs x 4 SIMDs
XCDS = 8      # GRBM_GUI_ACTIVE is summed over the XCDs (MI355X_MICROARCH.md, DVFS give-back)
CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "valu_calib.json")


def calib_summary(a):
    """What the VALU counters count, from kernels of known instruction count and class
    (tools/valu_calib.hip: every SIMD at 4 waves issuing independent chains of one class).
    cyc_per_winst = cycles each SIMD spends per wave-instruction at full issue =
    (GRBM_GUI_ACTIVE / XCDs) * SIMDs / wave-instructions."""
    known = [json.loads(ln) for ln in open(os.path.join(a.src, "calib.log")) if ln.startswith('{"mode"')]
    rows = per_dispatch(os.path.join(a.src, "pmc_calib", "run_counter_collection.csv"), "k_cal")
    # two dispatches per mode (warm, timed), in mode order
    out = {"modes": []}
    for j, kn in enumerate(known):
        r = rows[2 * j + 1]
        wi = kn["wave_insts"]
        cyc = r["GRBM_GUI_ACTIVE"] / XCDS
        out["modes"].append({"op": kn["op"], "wave_insts": wi, "ms": kn["ms"],
                             "insts_valu_per_winst": r["SQ_INSTS_VALU"] / wi,
                             "int32_per_winst": r["SQ_INSTS_VALU_INT32"] / wi,
                             "int64_per_winst": r["SQ_INSTS_VALU_INT64"] / wi,
                             "active_inst_valu_per_winst": r["SQ_ACTIVE_INST_VALU"] / wi,
                             "thread_cycles_valu_per_winst": r["SQ_THREAD_CYCLES_VALU"] / wi,
                             "clock_ghz": cyc / (kn["ms"] * 1e-3) / 1e9,
                             "cyc_per_winst": cyc * SIMDS / wi})
    m = {x["op"]: x for x in out["modes"]}
    out["c32"] = m["v_xor_b32"]["cyc_per_winst"]
    out["c64"] = m["v_lshlrev_b64"]["cyc_per_winst"]
    out["c32_slow"] = m["v_bcnt_u32_b32"]["cyc_per_winst"]
    out["note"] = ("VALU issue fraction of a kernel = (INT64 x c64 + (VALU - INT64) x c32) / (SIMDs x GRBM_GUI_ACTIVE / "
                   "XCDs); c32_slow (v_bcnt class) bounds it from above for 32-bit work")
    out["profile"] = os.path.basename(a.dst.rstrip("/"))
    os.makedirs(a.dst, exist_ok=True)
    json.dump(out, open(os.path.join(a.dst, "valu_calib.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


def load_calib(dst):
    """this session's calibration (dst/valu_calib.json) or the committed one"""
    for p in (os.path.join(dst, "valu_calib.json"), CALIB):
        if os.path.exists(p):
            return json.load(open(p))
    return None


def valu_issue(rows_sum, calib, mix=None):
    """VALU issue fraction of summed dispatch counters, by the calibrated class costs.  With a
    static class mix of the kernel's ISA (tools/isa_mix.py) the fraction at that mix replaces
    the bracket's upper end (every non-INT64 instruction at the slow class)."""
    v, i64 = rows_sum["SQ_INSTS_VALU"], rows_sum.get("SQ_INSTS_VALU_INT64", 0.0)
    cyc = rows_sum["GRBM_GUI_ACTIVE"] / XCDS * SIMDS
    issued = i64 * calib["c64"] + (v - i64) * calib["c32"]
    out = {"issue_frac": issued / cyc, "int64_share": i64 / v,
           "clock_ghz_note": "GRBM_GUI_ACTIVE / XCDs = cycles of the dispatch"}
    if mix:
        sl = mix["slow_share"]
        out["issue_frac_mix"] = v * (sl * calib["c32_slow"] + (1 - sl) * calib["c32"]) / cyc
        out["mix_source"] = {"slow_share": sl, "valu_static": mix["valu_static"], "tool": "tools/isa_mix.py"}
    else:
        out["issue_frac_upper"] = (i64 * calib["c64"] + (v - i64) * calib["c32_slow"]) / cyc
    return out


def load_mix(kern):
    p = os.path.join(os.path.dirname(CALIB), f"isa_mix_{kern}.json")
    return json.load(open(p)) if os.path.exists(p) else None


def rollout_summary(a):
    """The headline kernel: the LAST dispatch of the fused rollout of the bench command
    (its timed launch of K steps).  HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE), per
    board per ply; VALU instructions per wave, lane utilisation, INT64 share, issue fraction
    (calibrated, tools/valu_calib.hip); SQ_WAIT_ANY share of wave cycles."""
    kern = a.rollout_kernel
    t = a.roll_tag
    f = per_dispatch(os.path.join(a.src, f"pmc_roll{t}_fetch", "run_counter_collection.csv"), kern)[-1]
    w = per_dispatch(os.path.join(a.src, f"pmc_roll{t}_write", "run_counter_collection.csv"), kern)[-1]
    bl = bench_line(os.path.join(a.src, f"pmcr{t}f.log")) or {}
    plies = bl.get("steps", 20)
    fetch, write = f["FETCH_SIZE"] * 1024 * 2, w["WRITE_SIZE"] * 1024
    out = {"kernel": kern, "boards": a.boards, "plies_per_launch": plies, "fetch_bytes_corrected": fetch,
           "write_bytes": write, "bytes_per_launch": fetch + write,
           "bytes_per_board_ply": (fetch + write) / a.boards / plies,
           "mean_window": bl.get("roofline", {}).get("mean_window"),
           "note": f"the timed launch of the bench command (--steps {plies} --warmup 5); FETCH_SIZE x2"}
    mp = os.path.join(a.src, f"pmc_roll{t}_mix", "run_counter_collection.csv")
    if os.path.exists(mp):
        m = per_dispatch(mp, kern)[-1]
        waves = m["SQ_WAVES"]
        out["valu"] = {"insts_per_wave_per_ply": m["SQ_INSTS_VALU"] / waves / plies,
                       "lane_utilisation": m["SQ_THREAD_CYCLES_VALU"] / (m["SQ_ACTIVE_INST_VALU"] * 64),
                       "wait_any_share": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]}
        cal = load_calib(a.dst)
        if cal:
            out["valu"].update(valu_issue(m, cal))
    out["profile"] = os.path.basename(a.dst.rstrip("/"))
    os.makedirs(a.dst, exist_ok=True)
    json.dump(out, open(os.path.join(a.dst, f"pmc_rollout{t}.json"), "w"), indent=1)
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
    """k_perft2_val (the split leaf pass: one lane = one distinct depth-2 subtree, bulk-counted
    last ply) over the bench's perft leg.  Per launch: HBM bytes (FETCH_SIZE x2 + WRITE_SIZE),
    VALU instructions per wave, lane utilisation, VALU busy fraction.  Algorithmic bytes per
    subtree: the root's 64-byte record (7 bitboards + meta, read in order) + its count (8) added
    into the parent's sum = 72 B, + the 8-B count kept for the followers = 80 B; the leaves
    never touch memory.  (--perft-kernel k_perft2_rec: every record counted, 72 B;
    k_perft2_perm_rec: the earlier gathering form, + a 4-B permutation index.)"""
    kern = a.perft_kernel
    rows = lambda sub: per_dispatch(os.path.join(a.src, sub, "run_counter_collection.csv"), kern)  # noqa: E731
    f, w, m = rows("pmc_perft_fetch"), rows("pmc_perft_write"), rows("pmc_perft_mix")
    tot = lambda rs, k: sum(r[k] for r in rs)  # noqa: E731
    waves = tot(m, "SQ_WAVES")
    out = {"kernel": kern, "launches": len(m),
           "hbm_bytes_total": tot(f, "FETCH_SIZE") * 1024 * 2 + tot(w, "WRITE_SIZE") * 1024,
           "subtrees_total": waves * 64,
           "alg_bytes_per_subtree": 76 if "perm" in kern else (80 if "val" in kern else 72),
           "valu": {"insts_per_wave": tot(m, "SQ_INSTS_VALU") / waves,
                    "lane_utilisation": tot(m, "SQ_THREAD_CYCLES_VALU") / (tot(m, "SQ_ACTIVE_INST_VALU") * 64),
                    "wait_any_share": tot(m, "SQ_WAIT_ANY") / tot(m, "SQ_WAVE_CYCLES")},
           "profile": os.path.basename(a.dst.rstrip("/"))}
    out["hbm_bytes_per_subtree"] = out["hbm_bytes_total"] / max(out["subtrees_total"], 1)
    cal = load_calib(a.dst)
    if cal:
        out["valu"].update(valu_issue({k: tot(m, k) for k in m[0]}, cal, load_mix(kern)))
    os.makedirs(a.dst, exist_ok=True)
    for p in (os.path.join(a.dst, "pmc_perft.json"),):
        json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
