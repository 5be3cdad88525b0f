"""Shared test configuration.

`-m "not gpu"` runs here (no GPU): oracle vs Grok golden vectors, host logic,
C-ABI loading.  `-m gpu` runs on an MI355X: the HIP path against the oracle
and the golden fixtures, through the C ABI.
"""
import glob
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    # torch's bundled HIP runtime must initialise before libgrok_amd.so's (see
    # grok_amd.Engine); import it up front so GPU tests can share device tensors.
    import torch  # noqa: F401
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size cases (minutes on CPU)")


def parse_flags(flags):
    """Grok CLI flags of a fixture -> keyword arguments shared by oracle.encode
    and grok_amd.default_params (grk_compress.cpp:476-615 option meanings)."""
    t = flags.split()
    kw = {}
    if "-n" in t:
        kw["numres"] = int(t[t.index("-n") + 1])
    if "-b" in t:
        kw["cblk"] = tuple(int(v) for v in t[t.index("-b") + 1].split(","))
    if "-c" in t:
        kw["precincts"] = [tuple(map(int, m)) for m in re.findall(r"\[(\d+),(\d+)\]", t[t.index("-c") + 1])]
    if "-I" in t:
        kw["irreversible"] = True
    if "-r" in t:   # a ratio of 1 means lossless (0) (grk_compress.cpp:781-786)
        kw["layer_rate"] = [0.0 if float(v) == 1 else float(v) for v in t[t.index("-r") + 1].split(",")]
    if "-M" in t:
        kw["cblk_sty"] = int(t[t.index("-M") + 1])
    if "-t" in t:
        kw["tiles"] = tuple(int(v) for v in t[t.index("-t") + 1].split(","))
    if "-X" in t:
        kw["tlm"] = True
    if "-S" in t:
        kw["sop"] = True
    if "-E" in t:
        kw["eph"] = True
    if "-q" in t:
        kw["quality"] = [float(v) for v in t[t.index("-q") + 1].split(",")]
    if "-p" in t:
        kw["prog_order"] = t[t.index("-p") + 1]
    if "-d" in t:   # image offset (the readers set grk_image::x0 / y0 from it)
        kw["origin"] = tuple(int(v) for v in t[t.index("-d") + 1].split(","))
    if "-T" in t:   # tile grid offset; alone it also moves the image there (grk_compress.cpp:1547-1551)
        kw["tile_origin"] = tuple(int(v) for v in t[t.index("-T") + 1].split(","))
    if "-P" in t:   # grk_compress.cpp:1001-1057 with its clamps; every tile takes the list's head
        nl = len(kw.get("layer_rate") or kw.get("quality") or [0])
        nr = kw.get("numres", 6)
        pocs = []
        for e in t[t.index("-P") + 1].split("/"):
            m = re.match(r"T(\d+)=(\d+),(\d+),(\d+),(\d+),(\d+),(\w{4})", e)
            rs, cs, le, re_, ce = (int(v) for v in m.groups()[1:6])
            pocs.append((m.group(1), rs, cs, min(le, nl), re_ if re_ <= nr else nr - 1, ce, m.group(7)))
        k = sum(1 for q in pocs if q[0] == "0")
        if k > 1:
            kw["pocs"] = [q[1:] for q in pocs[:k]]
    if "-L" in t:
        kw["plt"] = True
    if "-u" in t:   # tile-part divider (grk_compress -u L|R|C)
        kw["tile_parts"] = t[t.index("-u") + 1]
    return kw


class Fixture:
    def __init__(self, path):
        z = np.load(path)
        self.name = os.path.basename(path)[:-4]
        self.img = z["img"].astype(np.int32)
        self.bits = int(z["bits"])
        self.flags = str(z["flags"])
        self.cs = z["cs"].tobytes()
        self.grok_decoded = z["grok_decoded"].astype(np.int32)
        self.kw = parse_flags(self.flags)

    @property
    def lossless(self):
        return "-I" not in self.flags

    @property
    def ht(self):
        return "-M" in self.flags

    @property
    def tiled(self):
        return "-t" in self.flags

    def __repr__(self):
        return self.name


def load_fixtures():
    return [Fixture(p) for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))]


FIXTURES = load_fixtures()


def fixture_ids(fx):
    return [f.name for f in fx]
