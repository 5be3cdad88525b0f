"""Record reference-Grok facts for the full-size BASELINE configs.

Runs the Grok 9.2.0 CLI built by the survey stage (SURVEY.md §8(c),
/tmp/grok-build/bin) on the seeded synthetic images of grok_amd/synth.py and
writes tests/golden/full_size.json: codestream size + SHA-256 per config, and
for lossy configs the PSNR of Grok's own decode vs the source.  Data only —
the GPU tests compare against these numbers; nothing at test time needs Grok.

Usage: python tests/golden/make_fullsize.py [--grok-bin DIR] [--only C2,C3]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from grok_amd.synth import synth_image, write_pnm  # noqa: E402
import oracle as O  # noqa: E402

CONFIGS = {
    "C1": dict(w=1920, h=1080, c=3, bits=8, seed=1, flags=""),
    "C2": dict(w=8192, h=8192, c=3, bits=8, seed=10, flags=""),
    "C2p": dict(w=8192, h=8192, c=3, bits=8, seed=10, flags="-c [256,256]"),
    "C3_4k": dict(w=4096, h=4096, c=3, bits=12, seed=11, flags="-I -r 40,20,10"),
    "C3p": dict(w=8192, h=8192, c=3, bits=12, seed=11, flags="-I -r 40,20,10 -c [256,256]"),
    "C3_l1": dict(w=2048, h=2048, c=3, bits=12, seed=11, flags="-I"),
    "C4": dict(w=16384, h=16384, c=1, bits=16, seed=20, flags="-M 64 -t 1024,1024 -X -L"),
    "C4_4k": dict(w=4096, h=4096, c=1, bits=16, seed=20, flags="-M 64 -t 1024,1024 -X -L"),
    "C4_p1": dict(w=4096, h=4096, c=1, bits=16, seed=20, flags="-t 1024,1024 -X -L"),
}


def psnr(a, b, bits):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return float(10 * np.log10(((1 << bits) - 1) ** 2 / mse)) if mse > 0 else float("inf"), float(mse), int(
        np.abs(a.astype(np.int64) - b).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grok-bin", default="/tmp/grok-build/bin")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    env = dict(os.environ, LD_LIBRARY_PATH=args.grok_bin)
    out_path = os.path.join(HERE, "full_size.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    res["_comment"] = ("Reference Grok 9.2.0 (survey build, grk_compress -H 8) on grok_amd/synth.py images: codestream "
                       "size + SHA-256, and for lossy configs Grok's own decode PSNR vs source. Made by make_fullsize.py.")
    names = [n for n in CONFIGS if not args.only or n in args.only.split(",")]
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for name in names:
            cfg = CONFIGS[name]
            img = synth_image(cfg["h"], cfg["w"], cfg["c"], cfg["bits"], cfg["seed"])
            ext = "ppm" if cfg["c"] == 3 else "pgm"
            src = os.path.join(td, "in." + ext)
            write_pnm(src, img, cfg["bits"])
            j2k = os.path.join(td, name + ".j2k")
            subprocess.run([os.path.join(args.grok_bin, "grk_compress"), "-i", src, "-o", j2k, "-H", "8"]
                           + cfg["flags"].split(), env=env, check=True, capture_output=True)
            cs = open(j2k, "rb").read()
            entry = dict(cfg, bytes=len(cs), sha256=hashlib.sha256(cs).hexdigest(),
                         input_sha256=hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest())
            if "-I" in cfg["flags"]:
                dec = os.path.join(td, "dec." + ext)
                subprocess.run([os.path.join(args.grok_bin, "grk_decompress"), "-i", j2k, "-o", dec, "-H", "8"],
                               env=env, check=True, capture_output=True)
                if cfg["c"] == 3 and os.path.exists(os.path.join(td, "dec_0.pgm")):
                    d = np.stack([O.read_pnm(os.path.join(td, "dec_%d.pgm" % k))[0][0] for k in range(3)])
                else:
                    d = O.read_pnm(dec)[0]
                p, mse, mx = psnr(d, img, cfg["bits"])
                entry.update(grok_psnr_db=round(p, 4), grok_mse=round(mse, 4), grok_maxabs=mx,
                             grok_decoded_sha256=hashlib.sha256(d.astype(np.uint16).tobytes()).hexdigest())
            res[name] = entry
            print(name, json.dumps(entry), flush=True)
            json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
