"""Solo T1 decoding (one wave per code-block, gk_t1dec.hip solo_block) against the oracle.

The engine gives the heaviest blocks of a decode to solo waves on the SIMDs the lane-parallel
waves leave (gk_t1dec_solo_blocks); every GPU decode test therefore runs some blocks through
it.  Here GK_T1DEC_SOLO forces the split (every block solo, none, a few) in fresh processes (the
switch is read once), over block sizes, bit depths, both filters, truncated passes (quality
layers, rate control) and stripe heights that are not multiples of 4.  Bar: samples identical
to the oracle's decode (oracle/j2k_oracle.cpp t1_decode_block, T1.cpp:934-1446).
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CODE = r'''
import sys, numpy as np
sys.path[:0] = [%r, %r]
import grok_amd as G, oracle as O
from grok_amd.synth import synth_image
e = G.Engine(0)
cases = [
    ((256, 264, 3, 8), dict()),
    ((200, 136, 3, 12), dict(irreversible=True)),
    ((130, 70, 1, 16), dict(numres=4)),
    ((150, 97, 3, 8), dict(cblk=(32, 32))),
    ((99, 141, 1, 8), dict(cblk=(16, 64), numres=3)),
    ((64, 64, 1, 8), dict(cblk=(64, 64), numres=1)),
    ((256, 256, 3, 8), dict(layer_rate=[40.0, 10.0], nlayers=2)),
    ((180, 220, 3, 12), dict(irreversible=True, layer_rate=[30.0])),
    ((70, 90, 3, 8), dict(tiles=(33, 41), numres=3)),
]
for (h, w, c, bits), kw in cases:
    img = synth_image(h, w, c, bits, 3).astype(np.int32)
    nr = kw.pop("numres", 6)
    cs = O.encode(img, bits, numres=nr, **kw)
    want, _ = O.decode(cs)
    got = e.decode(cs)
    assert np.array_equal(got, want), ((h, w, c, bits), kw, int(np.abs(got.astype(np.int64) - want).max()))
e.close()
print("ok")
''' % (ROOT, os.path.join(ROOT, "oracle"))


@pytest.mark.parametrize("solo", ["100000", "0", "5"])
def test_solo_decode_vs_oracle(solo):
    env = dict(os.environ, GK_T1DEC_SOLO=solo)
    r = subprocess.run([sys.executable, "-c", CODE], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
