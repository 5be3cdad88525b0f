"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE / WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts half
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section):
it is doubled here.  WRITE_SIZE is taken as is.  Output: JSON keyed by kernel
base name with the average HBM bytes per launch (read by bench.py for
roofline.traffic) and a text table.

Usage: python tools/pmc_summary.py FETCH.db WRITE.db OUT.json
"""
import json
import sqlite3
import sys
from collections import defaultdict


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name = ?", (counter,)):
        acc[name.split("(")[0]].append(float(val) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(fetch):
        rd = 2.0 * fetch[k]
        wr = write.get(k, 0.0)
        out[k] = {"fetch_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
                  "launches": nf[k]}
    json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
    print("%-28s %8s %16s %16s %16s" % ("kernel", "launches", "read_B(x2)", "write_B", "total_B"))
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        print("%-28s %8d %16.0f %16.0f %16.0f" % (k[:28], v["launches"], v["fetch_bytes_per_launch"],
                                                   v["write_bytes_per_launch"], v["hbm_bytes_per_launch"]))


if __name__ == "__main__":
    main()
