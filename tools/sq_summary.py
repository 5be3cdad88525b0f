"""Print per-kernel SQ counter averages from tools/sq_counters.sh output."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq/run_results.db")
d = {}
for k, cn, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection group by kernel_name, counter_name"):
    d.setdefault(k.split("(")[0], {})[cn] = v
for k, v in d.items():
    if any(t in k for t in ("t1", "dwt", "rct", "ht")):
        w = v.get("SQ_WAVES", 1)
        print("%-22s waves %6d  VALU/wave %10.0f SALU/wave %9.0f LDS/wave %8.0f  active %5.2f wait %5.2f waitinst %5.2f" % (
            k[:22], w, v["SQ_INSTS_VALU"] / w, v["SQ_INSTS_SALU"] / w, v["SQ_INSTS_LDS"] / w,
            v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"], v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"],
            v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"]))
