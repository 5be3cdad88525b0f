"""Step-by-step run of one unaligned-tile case with progress lines (GPU debugging aid)."""
import sys, os, time
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import grok_amd as G
import oracle as O
from grok_amd.synth import synth_image

def log(*a):
    print("%.2f" % time.time(), *a, flush=True)

h, w, tiles, nr = int(sys.argv[1]), int(sys.argv[2]), (int(sys.argv[3]), int(sys.argv[4])), int(sys.argv[5])
img = synth_image(h, w, 3, 8, 3).astype(np.int32)
log("oracle encode")
ref = O.encode(img, 8, tiles=tiles, numres=nr)
log("oracle done", len(ref))
e = G.Engine(0)
log("engine up")
cs = e.encode(img, 8, params=G.default_params(numresolution=nr, tiles=tiles))
log("encode done", len(cs), cs == ref)
d = e.decode(ref)
log("decode done", bool((d == img).all()))
e.close()
