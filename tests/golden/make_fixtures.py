"""Generate the golden parity fixtures from reference Grok 9.2.0.

Runs the `grk_compress` / `grk_decompress` binaries that the survey stage
built from /root/reference (/tmp/grok-build/bin) on small
seeded synthetic images, and stores input + reference codestream (+ reference
decode for lossy cases) as .npz fixtures next to this script.  The reference
is only *run* here, in the build container; the fixtures are plain data and
nothing under tests/ needs /root/reference or Grok at test time.

Usage:  python tests/golden/make_fixtures.py [--grok-bin DIR]
"""
import argparse
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


def cases():
    rng = np.random.default_rng(1234)
    C = []
    C.append(("rgb8_64", synth_image(64, 64, 3, 8, 1), 8, []))
    C.append(("rgb8_odd", synth_image(131, 257, 3, 8, 2), 8, []))
    C.append(("rgb8_tiny", synth_image(3, 5, 3, 8, 3), 8, ["-n", "2"]))
    C.append(("mono8_col", synth_image(37, 1, 1, 8, 4), 8, ["-n", "3"]))
    C.append(("mono8_noise", rng.integers(0, 256, size=(1, 128, 128)).astype(np.uint16), 8, []))
    C.append(("mono8_const", np.full((1, 60, 100), 200, np.uint16), 8, []))
    C.append(("rgb12_192", synth_image(192, 192, 3, 12, 11), 12, []))
    C.append(("mono16_noise", rng.integers(0, 65536, size=(1, 64, 96)).astype(np.uint16), 16, []))
    C.append(("mono16_300", synth_image(200, 300, 1, 16, 20), 16, []))
    C.append(("rgb8_prc", synth_image(256, 256, 3, 8, 5), 8, ["-c", "[64,64],[32,32]"]))
    C.append(("rgb8_cb32", synth_image(136, 200, 3, 8, 6), 8, ["-b", "32,32", "-n", "4"]))
    C.append(("rgb8_cbrect", synth_image(96, 160, 3, 8, 7), 8, ["-b", "64,16"]))
    C.append(("rgb12_97", synth_image(256, 256, 3, 12, 11), 12, ["-I"]))
    C.append(("rgb12_97_r", synth_image(384, 384, 3, 12, 11), 12, ["-I", "-r", "40,20,10"]))
    C.append(("mono16_ht", synth_image(256, 256, 1, 16, 20), 16, ["-M", "64"]))
    C.append(("rgb8_ht", synth_image(128, 128, 3, 8, 8), 8, ["-M", "64"]))
    # multi-tile (tile origins are multiples of 2^(levels)), TLM (-X) and PLT (-L) markers
    C.append(("rgb8_tiles", synth_image(300, 200, 3, 8, 41), 8, ["-t", "128,128"]))
    C.append(("rgb8_tiles_xl", synth_image(300, 200, 3, 8, 42), 8, ["-t", "128,128", "-X", "-L"]))
    C.append(("mono16_ht_tiles", synth_image(192, 256, 1, 16, 43), 16, ["-M", "64", "-t", "64,64", "-X", "-L"]))
    C.append(("rgb12_97_tiles", synth_image(160, 256, 3, 12, 44), 12, ["-I", "-t", "128,128"]))
    C.append(("mono8_tiles_n3", synth_image(77, 99, 1, 8, 45), 8, ["-t", "32,32", "-n", "3", "-b", "16,16"]))
    return C


def run(cmd, env):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed: %s %s" % (cmd, r.stdout[-500:], r.stderr[-500:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grok-bin", default="/tmp/grok-build/bin")
    ap.add_argument("--only", nargs="*", help="regenerate only these fixture names")
    args = ap.parse_args()
    env = dict(os.environ, LD_LIBRARY_PATH=args.grok_bin)
    comp = os.path.join(args.grok_bin, "grk_compress")
    dec = os.path.join(args.grok_bin, "grk_decompress")
    with tempfile.TemporaryDirectory() as td:
        for name, img, bits, flags in cases():
            if args.only and name not in args.only:
                continue
            ext = "ppm" if img.shape[0] == 3 else "pgm"
            src = os.path.join(td, name + "." + ext)
            write_pnm(src, img, bits)
            j2k = os.path.join(td, name + ".j2k")
            run([comp, "-i", src, "-o", j2k, "-H", "1"] + flags, env)
            cs = open(j2k, "rb").read()
            out = os.path.join(td, name + "_dec." + ext)
            run([dec, "-i", j2k, "-o", out, "-H", "1"], env)
            if img.shape[0] == 3:
                planes = [O.read_pnm(os.path.join(td, name + "_dec_%d.pgm" % k))[0][0] for k in range(3)] \
                    if os.path.exists(os.path.join(td, name + "_dec_0.pgm")) else list(O.read_pnm(out)[0])
                decoded = np.stack(planes, 0)
            else:
                decoded = O.read_pnm(out)[0]
            np.savez_compressed(os.path.join(HERE, name + ".npz"), img=img, bits=np.int32(bits),
                                flags=np.array(" ".join(flags)), cs=np.frombuffer(cs, np.uint8),
                                grok_decoded=decoded.astype(np.uint16))
            lossless = bool((decoded.astype(np.int64) == img.astype(np.int64)).all())
            print("%-14s %s %6d B  grok-roundtrip-lossless=%s" % (name, img.shape, len(cs), lossless))


if __name__ == "__main__":
    main()
