"""Compare the engine's forward-DWT planes (GK_DUMP_DWT) with the oracle's coefficients, band by band."""
import sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "oracle")]
import oracle as O
from grok_amd.synth import synth_image
mode = sys.argv[1]
h, w, nr = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
img = synth_image(h, w, 1, 12, 5).astype(np.int32)
if mode == "enc":
    import grok_amd as G
    e = G.Engine(0)
    e.encode(img, 12, params=G.default_params(numresolution=nr, irreversible=True))
    e.close()
    sys.exit(0)
ref = O.forward_coefs(img, 12, irreversible=True, numres=nr).view(np.float32)[0]
def load(p):
    a = np.fromfile(p, dtype=np.int32)
    nc, stride, rh, rw = a[:4]
    pl = a[4:].view(np.float32).reshape(nc, 2, rh, stride)
    return pl[0]
L = nr - 1
rw = [-(-w // (1 << l)) for l in range(L + 1)]
rh = [-(-h // (1 << l)) for l in range(L + 1)]
for name in sys.argv[5:]:
    P = load(name)
    print(name)
    for l in range(1, L + 1):
        pl = P[l & 1]
        for (bx, by, tag) in ((1, 0, "HL"), (0, 1, "LH"), (1, 1, "HH")) + (((0, 0, "LL"),) if l == L else ()):
            x0 = rw[l] if bx else 0; x1 = rw[l - 1] if bx else rw[l]
            y0 = rh[l] if by else 0; y1 = rh[l - 1] if by else rh[l]
            a = pl[y0:y1, x0:x1]; b = ref[y0:y1, x0:x1]
            nd = int((a.view(np.int32) != b.view(np.int32)).sum())
            print("  level %d %s %dx%d differ %d maxabs %.3g" % (l, tag, x1 - x0, y1 - y0, nd, float(np.abs(a - b).max()) if a.size else 0))
