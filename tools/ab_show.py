"""Diagnostic only: print the headline of one bench.py JSON line (used by tools/ab_lib.sh)."""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
line = [l for l in open(path).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
rf = d.get("roofline") or {}
ls = d.get("launched_step") or {}
print(tag, "%.3fe9 %s" % (d["value"] / 1e9, d["unit"]), "ms/step %.4f" % d["ms_per_step"],
      "launch_us %s" % rf.get("avg_launch_us"), "launched %.3fe9" % (ls.get("value", 0) / 1e9),
      "launched_ply_us %s" % (ls.get("roofline") or {}).get("avg_ply_us"))
