"""GK_DWT_ANY 9/7 bisection aid: which sizes / level counts differ from the oracle."""
import sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import grok_amd as G
import oracle as O
from grok_amd.synth import synth_image
e = G.Engine(0)
for (h, w, c, nr) in [(128, 128, 1, 3), (130, 130, 1, 2), (132, 132, 1, 3), (130, 40, 1, 3), (40, 130, 1, 3),
                      (130, 130, 1, 3), (260, 40, 1, 3), (40, 260, 1, 3)]:
    img = synth_image(h, w, c, 12, 5).astype(np.int32)
    cs = e.encode(img, 12, params=G.default_params(numresolution=nr, irreversible=True))
    ref = O.encode(img, 12, numres=nr, irreversible=True)
    d_ok = None
    want, _ = O.decode(ref)
    got = e.decode(ref)
    d = int(np.abs(got.astype(np.int64) - want).max())
    print((h, w, c, nr), "enc", cs == ref, len(cs), len(ref), "dec maxdiff", d, flush=True)
e.close()
