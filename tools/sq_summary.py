"""Print per-kernel SQ counter averages from a rocprofv3 PMC pass (tools/sq_counters*.sh):
per-wave instruction counts and the cycle buckets as fractions of SQ_WAVE_CYCLES."""
import sqlite3
import sys

import json

c = sqlite3.connect(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq/run_results.db")
out_json = sys.argv[2] if len(sys.argv) > 2 else None   # optional: per-kernel per-wave counts (bench.py reads it)
d = {}
for k, cn, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"):
    d.setdefault(k.split("(")[0], {})[cn] = v
for k, v in d.items():
    if not any(t in k for t in ("t1", "dwt", "rct", "ht", "gather")):
        continue
    w = v.get("SQ_WAVES", 1) or 1
    cyc = v.get("SQ_WAVE_CYCLES", 0) or 1
    parts = ["waves %d" % w]
    for n, x in sorted(v.items()):
        if n in ("SQ_WAVES", "SQ_WAVE_CYCLES"):
            continue
        if n.startswith("SQ_INSTS"):
            parts.append("%s/wave %.0f" % (n[8:], x / w))
        else:
            parts.append("%s %.3f" % (n[3:], x / cyc))
    parts.append("WAVE_CYCLES/wave %.0f" % (cyc / w))
    print("%-26s %s" % (k[:26], "  ".join(parts)))
if out_json:
    js = {}
    for k, v in d.items():
        w = v.get("SQ_WAVES", 1) or 1
        js[k] = {"waves": w, "wave_cycles_per_wave": v.get("SQ_WAVE_CYCLES", 0) / w,
                 "insts_per_wave": {n[9:].lower(): x / w for n, x in v.items() if n.startswith("SQ_INSTS_")},
                 "wait_any": v.get("SQ_WAIT_ANY", 0) / (v.get("SQ_WAVE_CYCLES", 0) or 1),
                 "active_inst_any": v.get("SQ_ACTIVE_INST_ANY", 0) / (v.get("SQ_WAVE_CYCLES", 0) or 1)}
    json.dump(js, open(out_json, "w"), indent=1, sort_keys=True)
