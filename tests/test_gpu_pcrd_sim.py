"""PCRD rate control: the band-parallel packet-size simulation (gk_engine.cpp T2Enc::code_layer)
against real packet writes.

GK_T2_CHECK_SIM=1 makes the engine write every simulated packet for real and raise on any size
difference, at every bisection step (TileProcessor.cpp:1196-1365 pcrdBisectSimple + T2Compress
compressPacketsSimulate).  The variable is read once per process, so the cases run in a child
process; each codestream must also equal the oracle's byte for byte.  The check also compares the
coding state the simulation leaves (tag trees, pass counts, length indicators) with the packets'.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/oracle")
import grok_amd as G
import oracle as O
from grok_amd.synth import synth_image
cases = [
    (dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0]), 3, 12, (520, 700)),
    (dict(irreversible=True, layer_rate=[30.0, 8.0], precincts=[(128, 128), (64, 64)]), 3, 8, (400, 333)),
    (dict(irreversible=True, layer_rate=[50.0, 25.0, 12.0, 0.0], cblk=(32, 32), numres=4), 3, 12, (301, 257)),
    (dict(layer_rate=[20.0, 5.0, 0.0]), 3, 8, (256, 384)),
    (dict(irreversible=True, layer_rate=[12.0], precincts=[(64, 64)], numres=5), 3, 8, (640, 480)),
]
eng = G.Engine(0)
for i, (kw, c, bits, (h, w)) in enumerate(cases):
    img = synth_image(h, w, c, bits, 40 + i).astype(np.int32)
    k = {kk: kw[kk] for kk in ("cblk", "precincts", "irreversible", "layer_rate") if kk in kw}
    if "numres" in kw:
        k["numresolution"] = kw["numres"]
    k["numlayers"] = len(kw["layer_rate"])
    cs = eng.encode(img, bits, params=G.default_params(**k))
    assert cs == O.encode(img, bits, **kw), "case %d differs from the oracle" % i
eng.close()
print("pcrd simulation check ok")
"""


def test_pcrd_simulation_matches_packet_writes():
    env = dict(os.environ, GK_T2_CHECK_SIM="1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "pcrd simulation check ok" in r.stdout
