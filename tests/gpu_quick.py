"""Quick GPU bring-up check (run on the GPU box): encode/decode golden fixtures."""
import glob, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import grok_amd as G

eng = G.Engine(0)
ok = True
for fn in sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))):
    z = np.load(fn)
    flags = str(z["flags"])
    if "-I" in flags or "-M" in flags:
        continue
    name = os.path.basename(fn)[:-4]
    img = z["img"].astype(np.int32); bits = int(z["bits"]); ref = z["cs"].tobytes()
    kw = {}
    t = flags.split()
    if "-n" in t: kw["numresolution"] = int(t[t.index("-n") + 1])
    if "-b" in t: kw["cblk"] = tuple(int(v) for v in t[t.index("-b") + 1].split(","))
    if "-c" in t:
        import re
        kw["precincts"] = [tuple(map(int, m)) for m in re.findall(r"\[(\d+),(\d+)\]", t[t.index("-c") + 1])]
    try:
        cs = eng.encode(img, bits, params=G.default_params(**kw))
        exact = cs == ref
        d = next((i for i in range(min(len(cs), len(ref))) if cs[i] != ref[i]), None)
        dec = eng.decode(ref)
        dec_ok = bool((dec == img).all())
        print("%-14s enc_exact=%s (first diff %s, %d vs %d) dec_lossless=%s" % (name, exact, d, len(cs), len(ref), dec_ok), flush=True)
        ok &= exact and dec_ok
    except Exception as e:
        print("%-14s ERROR %s" % (name, e), flush=True)
        ok = False
print("ALL_OK" if ok else "FAILURES")
