"""SIMT-efficiency model of the lane-per-code-block T1 decoder (analysis tool).

Encodes a crop of a benchmark image with the oracle, replays every code-block
decode with per-(pass, stripe) decision counts (orc_t1_decode_stripe_counts),
groups blocks into 64-lane waves the way gk_engine.cpp does (bucketed by pass
count, descending) and reports, per wave, the loop steps of
  * the stripe-synchronous kernel: sum over (plane, pass, stripe) of the max
    decisions over the wave's lanes (k_t1_dec today), and
  * a lane-independent kernel: max over lanes of the block's total decisions.
Usage: python tools/t1_simt_stats.py [--size 1024] [--config C2]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from grok_amd.synth import synth_image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--seed", type=int, default=10)
    ap.add_argument("--irreversible", action="store_true")
    a = ap.parse_args()
    img = synth_image(a.size, a.size, 3, a.bits, a.seed).astype(np.int32)
    kw = dict(irreversible=True) if a.irreversible else {}
    blocks, data = O.encode_blocks(img, a.bits, **kw)
    lib = O.lib()
    lib.orc_t1_decode_stripe_counts.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    recs = []
    for b in blocks:
        w, h = b.x1 - b.x0, b.y1 - b.y0
        ns = (h + 3) // 4
        if not b.npasses:
            recs.append((0, 0, np.zeros((0, ns), np.int64)))
            continue
        buf = np.concatenate([data[b.data_off:b.data_off + b.len], np.zeros(16, np.uint8)])
        cnt = np.zeros(b.npasses * ns + 1, np.uint32)
        orient = b.band + 1 if b.res else 0
        lib.orc_t1_decode_stripe_counts(buf.ctypes.data, b.len, b.npasses, b.numbps, orient, w, h, cnt.ctypes.data)
        c = np.maximum.accumulate(cnt.astype(np.int64))
        d = np.diff(c).reshape(b.npasses, ns)
        recs.append((b.numbps, b.npasses, d))
    n = len(recs)
    order = sorted(range(n), key=lambda i: -recs[i][1])
    sync_steps, indep_steps, pass_steps, syms = [], [], [], []
    for w0 in range(0, n, 64):
        lanes = [recs[i] for i in order[w0:w0 + 64]]
        tot = [int(r[2].sum()) for r in lanes]
        syms += tot
        indep_steps.append(max(tot))
        maxplanes = max(r[0] for r in lanes)
        ns = max(r[2].shape[1] for r in lanes)
        st = pst = 0
        for k in range(maxplanes):
            for t in ([2] if k == 0 else [0, 1, 2]):
                pidx = 0 if k == 0 else 1 + 3 * (k - 1) + t
                act = [r for r in lanes if k < r[0] and pidx < r[1]]
                if not act:
                    continue
                pst += max(1, max(int(r[2][pidx].sum()) for r in act))
                for s in range(ns):
                    m = max((int(r[2][pidx, s]) if s < r[2].shape[1] else 0) for r in act)
                    st += max(1, m)
        sync_steps.append(st)
        pass_steps.append(pst)
    syms = np.array(syms)
    if os.environ.get("T1SIM_VERBOSE"):
        wmax = int(np.argmax(sync_steps))
        lanes = [recs[i] for i in order[wmax * 64:wmax * 64 + 64]]
        print("heaviest sync wave %d: numbps %s npasses %s" % (wmax, sorted(set(r[0] for r in lanes)),
                                                            sorted(set(r[1] for r in lanes))))
        print("  lane totals min/avg/max %d %.0f %d" % (min(int(r[2].sum()) for r in lanes),
                                                     np.mean([r[2].sum() for r in lanes]),
                                                     max(int(r[2].sum()) for r in lanes)))
    print("blocks %d  waves %d  decisions/block avg %.0f max %d" % (n, len(sync_steps), syms.mean(), syms.max()))
    print("stripe-synchronous: steps/wave avg %.0f max %.0f  (SIMT efficiency %.2f)" % (
        np.mean(sync_steps), np.max(sync_steps), syms.sum() / (64.0 * np.sum(sync_steps))))
    print("pass-synchronous:   steps/wave avg %.0f max %.0f  (SIMT efficiency %.2f)" % (
        np.mean(pass_steps), np.max(pass_steps), syms.sum() / (64.0 * np.sum(pass_steps))))
    print("lane-independent:   steps/wave avg %.0f max %.0f  (SIMT efficiency %.2f)" % (
        np.mean(indep_steps), np.max(indep_steps), syms.sum() / (64.0 * np.sum(indep_steps))))


if __name__ == "__main__":
    main()
