"""Instructions issued per decision step of the T1 decoder (k_t1_dec2<false>), counted from
the gfx950 ISA: compile gk_t1dec.hip with `hipcc -S`, take the unrolled step blocks of the
decoder loop (the T1DEC_UNROLL repeated basic blocks) and report the median count per step by
class.  bench.py's issue roofline uses this count (a wave alone issues one instruction per 4
cycles).

Usage: python tools/isa_step_count.py [path/to/gk_t1dec.hip]
"""
import os
import re
import statistics
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def count(src):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "t1dec.s")
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                               "-I", os.path.dirname(src), src, "-o", out])
        lines = open(out).read().split("\n")
    s = next(i for i, l in enumerate(lines) if re.match(r"^_Z9k_t1_dec2IL(?:b0|i0)EE.*:", l))
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], None
    for l in lines[s:e]:
        if re.match(r"^\.LBB\d+_\d+:", l):
            cur = {}
            blocks.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")) or cur is None:
            continue
        op = t.split()[0]
        k = ("valu" if op.startswith("v_") else "wait" if op.startswith("s_waitcnt") else
             "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "vmem")
        cur[k] = cur.get(k, 0) + 1
    # the step bodies: the largest group of basic blocks with near-identical sizes and LDS use
    sizes = [sum(b.values()) for b in blocks]
    big = [b for b, n in zip(blocks, sizes) if n > 150 and b.get("lds", 0) >= 10 and b.get("vmem", 0) == 0]
    tot = statistics.median(sum(b.values()) for b in big)
    by = {k: statistics.median(b.get(k, 0) for b in big) for k in ("valu", "salu", "lds", "wait")}
    return len(big), tot, by


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "grok_amd", "csrc", "gk_t1dec.hip")
    n, tot, by = count(src)
    print("step bodies %d, instructions per step %d (%s)" % (n, tot, ", ".join("%s %d" % kv for kv in by.items())))
