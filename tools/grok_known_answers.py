"""Run the oracle on the Grok 9.2.0 known answers (size + SHA-256 prefix) the reviews
recorded (VERDICT.md rounds 3-4), print which match.  Debugging aid for tiled PCRD."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from conftest import parse_flags  # noqa: E402
from grok_amd.synth import synth_image  # noqa: E402

# (input, flags, Grok bytes, Grok SHA-256 prefix or None)
CASES = [
    ("A", "-t 256,256 -r 20,5 -X", 118560, None),
    ("A", "-t 128,128 -r 30", 22142, None),
    ("A", "-r 20,10 -P T0=0,0,2,3,3,RLCP/T0=3,0,2,6,3,LRCP", 59621, "0be62df5a6eaa292"),
    ("A", "-P T0=0,0,2,3,3,RLCP/T0=3,0,2,6,3,LRCP", 410830, None),
    ("A", "-t 64,64 -r 40,10", 58693, "74e205793d99ec86"),
    ("A", "-t 64,64 -r 40,10 -X", 59057, "3aed03d6d38355b3"),
    ("A", "-t 64,64 -r 40,10 -X -L", 61386, "e0f30b121f864170"),
    ("A", "-t 128,128 -r 20,5 -M 1", 116460, "5e610ced8e4b3ec4"),
    ("A", "-M 3 -t 128,128 -r 20,5", 116863, "761c07175aa1d9ef"),
    ("A", "-p PCRL -c [128,128] -r 30,10 -t 256,256", 59432, "9ea438908929a4fe"),
    ("A", "-S -E -p RPCL -c [64,64],[32,32] -r 20,5 -t 256,256 -X -L", 126044, "cf3dffa94f7c4d5d"),
    ("A", "-t 256,256 -r 20,5 -u L", 118792, "8eb104ee7af67c2f"),
    ("A", "-t 200,160 -r 30,10", 59002, "233358c512356ea7"),
    ("A", "-p CPRL -c [64,64],[32,32] -r 20,5,1", 430903, "4b2a4e73b5768a8a"),
    ("B", "-t 96,96 -r 30,5", 31004, "a484a6cb530b7307"),
]
IMGS = {"A": (synth_image(384, 520, 3, 8, 7).astype(np.int32), 8),
        "B": (synth_image(300, 260, 1, 16, 21).astype(np.int32), 16)}


def run(sel=None):
    ok = 0
    for which, f, n, h in CASES:
        if sel and sel not in f:
            continue
        im, bits = IMGS[which]
        cs = O.encode(im, bits, **parse_flags(f))
        hh = hashlib.sha256(cs).hexdigest()[:16]
        good = len(cs) == n and (h is None or hh == h)
        ok += good
        print("%-62s grok %7d  ours %7d %+5d %s" % (f, n, len(cs), len(cs) - n, "OK" if good else ""))
    print("matched", ok)


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else None)
