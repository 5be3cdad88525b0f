"""Full-size reference facts for configs no Grok-produced hash covers here.

Grok 9.2.0 is built with cmake and needs generated headers, so this repository does
not rebuild it; the survey-stage Grok hashes in full_size.json cover
C1, C2, C2p, C3p, C3_4k, C3_l1, C4, C4_4k, C4_p1.  For the remaining BASELINE configs
this script records the output of the CPU oracle (oracle/j2k_oracle.cpp, pinned
byte-for-byte to Grok's fixtures and to the Grok hashes above) under
"oracle_fullsize" in full_size.json, marked source = "oracle":

  C3  8192^2 12-bit RGB, -I -r 40,20,10, single precinct (the bench's exact C3 stream;
      Grok's encoder runs on it, only its decoder is broken here, SURVEY R-BUG-3);
  C5  32768^2 RGB8 .jp2, -t 1024,1024 -X -L, plus the SHA-256 of the source samples of
      the four SURVEY windows (the lossless window decodes must equal them).

A maintainer with Grok can check both against grk_compress with the flags recorded
in make_fullsize.py (C3 / C5 entries) — same seeded inputs.

Usage: python tests/golden/make_oracle_fullsize.py [--only C3,C5] [--threads 8]
"""
import argparse
import hashlib
import json
import os
import struct
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from grok_amd.bigimage import slabs  # noqa: E402
from grok_amd.synth import synth_image  # noqa: E402
import oracle as O  # noqa: E402

C5_WINDOWS = {"w1k_origin": (0, 0, 1024, 1024), "w4k_unaligned": (12345, 23456, 16441, 27552),
              "w_edge": (30000, 30000, 32768, 32768), "w16k": (8000, 8000, 24384, 24384)}
C5 = dict(w=32768, h=32768, c=3, bits=8, seed=30, flags="-t 1024,1024 -X -L", format="jp2")
C3 = dict(w=8192, h=8192, c=3, bits=12, seed=11, flags="-I -r 40,20,10")


def make_c3(threads):
    img = synth_image(C3["h"], C3["w"], 3, 12, C3["seed"])
    O.set_threads(threads)
    t0 = time.time()
    cs = O.encode(img.astype(np.int32), 12, irreversible=True, layer_rate=[40.0, 20.0, 10.0])
    print("C3 oracle encode %.1fs, %d bytes" % (time.time() - t0, len(cs)), flush=True)
    return dict(C3, bytes=len(cs), sha256=hashlib.sha256(cs).hexdigest(),
                input_sha256=hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest(), source="oracle")


def make_c5(threads):
    W, H, C = C5["w"], C5["h"], C5["c"]
    kw = dict(tiles=(1024, 1024), tlm=True, plt=True)
    O.set_threads(threads)
    hdr, tlm = O.main_header(W, H, C, 8, **kw)
    crops = {k: np.empty((C, y1 - y0, x1 - x0), np.uint8) for k, (x0, y0, x1, y1) in C5_WINDOWS.items()}
    parts, lens = [], []
    ih = hashlib.sha256()
    t0 = time.time()
    for y0, slab in slabs(H, W, C, 8, C5["seed"], 1024, threads=threads):
        ih.update(slab.tobytes())   # input hash: (C, rows, W) slabs in order, not the (C, H, W) layout
        for k, (x0, wy0, x1, wy1) in C5_WINDOWS.items():
            a, b = max(y0, wy0), min(y0 + slab.shape[1], wy1)
            if a < b:
                crops[k][:, a - wy0:b - wy0] = slab[:, a - y0:b - y0, x0:x1]
        j = y0 // 1024
        body, ln = O.encode_tile_parts(slab.astype(np.int32), y0, (H, W), 8, j * 32, (j + 1) * 32, **kw)
        parts.append(body)
        lens += ln
        print("C5 rows %d / %d (%.0fs)" % (y0 + slab.shape[1], H, time.time() - t0), flush=True)
    h = bytearray(hdr)
    for t, n in enumerate(lens):
        h[tlm + 6 * t:tlm + 6 * t + 6] = struct.pack(">HI", t, n)
    cs_len = len(h) + sum(len(p) for p in parts) + 2
    pre = O.jp2_header(W, H, C, 8, cs_len)
    d = hashlib.sha256()
    d.update(pre)
    d.update(bytes(h))
    for p in parts:
        d.update(p)
    d.update(b"\xff\xd9")
    return dict(C5, bytes=len(pre) + cs_len, sha256=d.hexdigest(), input_slab_sha256=ih.hexdigest(),
                windows={k: dict(rect=list(C5_WINDOWS[k]), source_sha256=hashlib.sha256(v.tobytes()).hexdigest())
                         for k, v in crops.items()},
                source="oracle")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C3,C5")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    path = os.path.join(HERE, "full_size.json")
    res = json.load(open(path))
    ent = res.setdefault("oracle_fullsize", {})
    ent["_comment"] = ("CPU oracle (Grok-pinned restatement) outputs for configs without a Grok hash here; "
                       "made by make_oracle_fullsize.py. source = 'oracle', not Grok.")
    for name in args.only.split(","):
        ent[name] = make_c3(args.threads) if name == "C3" else make_c5(args.threads)
        print(name, json.dumps(ent[name]), flush=True)
        json.dump(res, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
