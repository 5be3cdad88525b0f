"""Instructions issued per decision step of the T1 decoder (k_t1_dec2<false>), counted from
the gfx950 ISA: compile gk_t1dec.hip with `hipcc -S`, take the unrolled step blocks of the
decoder loop (the T1DEC_UNROLL repeated basic blocks) and report the median count per step by
class.  bench.py's issue roofline uses this count (a wave alone issues one instruction per 4
cycles).

By default the count comes from the BUILT library (grok_amd/libgrok_amd.so): its gfx950 code
objects are unbundled and disassembled with ROCm's llvm-objdump, so the number describes the
code that runs; with a .hip path the source is compiled with `hipcc -S` instead.

Usage: python tools/isa_step_count.py [path/to/libgrok_amd.so | path/to/gk_t1dec.hip]
"""
import os
import re
import statistics
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
KERNEL = re.compile(r"^[0-9a-f]+ <_Z9k_t1_dec2ILi0ELi4EE.*>:")   # k_t1_dec2<0, 4>


def _classify(blocks, lines):
    cur = None
    for l in lines:
        if re.match(r"^[0-9a-f]+ <L\d+>:", l) or re.match(r"^\.LBB\d+_\d+:", l):
            cur = {}
            blocks.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or cur is None:
            continue
        op = t.split()[0]
        k = ("valu" if op.startswith("v_") else "wait" if op.startswith("s_waitcnt") else
             "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "vmem")
        cur[k] = cur.get(k, 0) + 1


def _summarise(blocks):
    # the step bodies: the largest group of basic blocks with near-identical sizes and LDS use
    sizes = [sum(b.values()) for b in blocks]
    big = [b for b, n in zip(blocks, sizes) if n > 150 and b.get("lds", 0) >= 10 and b.get("vmem", 0) == 0]
    tot = statistics.median(sum(b.values()) for b in big)
    by = {k: statistics.median(b.get(k, 0) for b in big) for k in ("valu", "salu", "lds", "wait")}
    return len(big), tot, by


def count_so(so):
    """Step count of k_t1_dec2<0, 4> in the built library's gfx950 code object."""
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "lib.so")
        with open(so, "rb") as f, open(lib, "wb") as g:
            g.write(f.read())
        subprocess.run([OBJDUMP, "--offloading", lib], cwd=d, capture_output=True, check=True)
        for co in sorted(os.listdir(d)):
            if "gfx950" not in co:
                continue
            dis = subprocess.run([OBJDUMP, "-d", "--symbolize-operands", "--no-show-raw-insn",
                                  os.path.join(d, co)], capture_output=True, text=True, check=True).stdout
            lines = dis.split("\n")
            s = next((i for i, l in enumerate(lines) if KERNEL.match(l)), None)
            if s is None:
                continue
            e = next((i for i in range(s + 1, len(lines)) if re.match(r"^[0-9a-f]+ <_Z", lines[i])), len(lines))
            blocks = []
            _classify(blocks, lines[s + 1:e])
            return _summarise(blocks)
    raise RuntimeError("k_t1_dec2<0, 4> not found in the gfx950 code objects of " + so)


def count(src):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "t1dec.s")
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                               "-I", os.path.dirname(src), src, "-o", out])
        lines = open(out).read().split("\n")
    s = next(i for i, l in enumerate(lines) if re.match(r"^_Z9k_t1_dec2ILi0ELi4EE.*:", l))
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = []
    _classify(blocks, lines[s:e])
    return _summarise(blocks)


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "grok_amd", "libgrok_amd.so")
    n, tot, by = count(src) if src.endswith(".hip") else count_so(src)
    print("step bodies %d, instructions per step %d (%s)" % (n, tot, ", ".join("%s %d" % kv for kv in by.items())))
