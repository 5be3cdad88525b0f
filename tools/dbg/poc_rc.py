"""Debug: engine vs oracle on POC + rate control (tests/test_gpu_progression.py cases)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa
import grok_amd as G
import oracle as O
from test_gpu_progression import POCS, _img
eng = G.Engine(0)
for pi in (0, 1, 2):
    img = _img(20 + pi, 3, 150, 170)
    for kw in (dict(tiles=(64, 96), plt=True, tlm=True), dict(precincts=[(32, 32)], layer_rate=[20, 5, 0])):
        gkw = dict(kw)
        if "layer_rate" in gkw:
            gkw["numlayers"] = len(gkw["layer_rate"])
        for serial in (0, 1):
            if serial: os.environ["GK_T2_SERIAL_SIM"] = "1"
            else: os.environ.pop("GK_T2_SERIAL_SIM", None)
            cs = eng.encode(img, 8, params=G.default_params(numresolution=4, cblk=(16, 16), pocs=POCS[pi], **gkw))
            ref = O.encode(img, 8, numres=4, cblk=(16, 16), pocs=POCS[pi], **kw)
            d = next((i for i in range(min(len(cs), len(ref))) if cs[i] != ref[i]), None)
            print(pi, list(kw), "serial" if serial else "fast", len(cs), len(ref), "first diff", d, flush=True)
eng.close()
