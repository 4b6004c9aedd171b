"""Static VALU class mix of one kernel in the gfx950 ISA of gymchess.hip (diagnostic).

The VALU counters cannot split a bitboard kernel's mix (profiles/valu_calib.json: INT32 and
INT64 count only some opcodes), so the issue-fraction bracket of the roofline blocks used the
fast class (v_xor_b32, 2.44 cycles per wave-instruction) for every non-INT64 instruction at
its lower end and the slow class (v_bcnt_u32_b32, 4.30) at its upper end.  This script counts
the kernel's VALU instructions by class in its ISA: slow = the calibrated 4.26-4.35-cycle
classes (64-bit shifts, v_lshl_add_u64, v_bcnt) plus 64-bit moves / adds / multiplies and
32-bit multiplies; fast = the rest.  A static count weights every instruction once: it stands
for the dynamic mix where one loop body dominates the kernel (the perft leaf: perft2's
per-child count).  pmc_summary.py reads the result (profiles/isa_mix_<kernel>.json) and
prints `issue_frac_mix` = SQ_INSTS_VALU x (slow x c_slow + fast x c32) / (SIMDs x cycles).

    python tools/isa_mix.py k_perft2_val [--out profiles/isa_mix_k_perft2_val.json]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gym-chess_amd", "csrc", "gymchess.hip")
SLOW = re.compile(r"^v_(\w+_(b64|u64|i64|f64)|bcnt_\w+|mul_(lo|hi)_[ui]32|mad_u64_u32|mad_i64_i32|mul_u32_u24)\b")


def kernel_body(asm, name):
    """the instruction lines of the first kernel whose (mangled) symbol contains name"""
    lines = asm.splitlines()
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", ln)
        if m and name in m.group(1):
            out = []
            for x in lines[i + 1:]:
                if x.startswith(".Lfunc_end"):
                    return m.group(1), out
                out.append(x.strip())
    raise SystemExit(f"kernel {name} not found")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--asm", default=None, help="an existing device .s (default: compile SRC)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.asm:
        asm = open(a.asm).read()
    else:
        with tempfile.TemporaryDirectory() as td:
            s = os.path.join(td, "k.s")
            subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                            "-mllvm", "-amdgpu-kernarg-preload-count=16", "-o", s, SRC], check=True)
            asm = open(s).read()
    sym, body = kernel_body(asm, a.kernel)
    ops = [ln.split()[0] for ln in body if ln.startswith("v_")]
    slow = [o for o in ops if SLOW.match(o)]
    hist = {}
    for o in slow:
        hist[o] = hist.get(o, 0) + 1
    cal = json.load(open(os.path.join(ROOT, "profiles", "valu_calib.json")))
    out = {"kernel": a.kernel, "symbol": sym, "valu_static": len(ops), "slow_static": len(slow),
           "slow_share": len(slow) / max(1, len(ops)), "slow_ops": dict(sorted(hist.items(), key=lambda kv: -kv[1])),
           "c32": cal["c32"], "c_slow": cal["c32_slow"],
           "note": "static counts of the kernel's ISA (every instruction once); slow = 64-bit ALU ops, bcnt, "
                   "32-bit multiplies (calibrated 4.26-4.35 cycles per wave-instruction), fast = the rest (2.44)"}
    path = a.out or os.path.join(ROOT, "profiles", f"isa_mix_{a.kernel}.json")
    json.dump(out, open(path, "w"), indent=1)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
