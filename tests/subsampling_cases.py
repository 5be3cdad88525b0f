"""Streams with subsampled components (SIZ XRsiz / YRsiz; grk_image_comp::dx / dy), shared by the
CPU tests (tests/test_subsampling.py: the oracle against OpenJPEG 2.5.4) and the GPU tests
(tests/test_gpu_subsampling.py: the HIP engine against the oracle).

Grok restates subsampling in TileProcessor.cpp:116-131 (tile-components = tiles / (dx, dy), rounded
up), PacketIter.cpp:287-388 (precinct positions scaled by dx), CodeStreamCompress.cpp:501-512 (no MCT
unless the first three components share a grid) and :961 (rate budget bits_empty = 8 dx0 dy0).
No Grok-produced subsampled stream exists in the reference or the review records, so the pin is
OpenJPEG: it decodes the oracle's streams sample for sample (test_subsampling.py)."""
import numpy as np

# name -> (W, H, subsampling, prec, oracle/engine keyword parameters)
CASES = {
    "420_53": (67, 45, [(1, 1), (2, 2), (2, 2)], 8, dict(numres=3)),
    "420_53_r6": (130, 97, [(1, 1), (2, 2), (2, 2)], 8, dict(numres=6)),
    "422_97": (96, 64, [(1, 1), (2, 1), (2, 1)], 8, dict(numres=4, irreversible=True)),
    "mixed4": (64, 48, [(1, 1), (1, 1), (2, 2), (2, 1)], 8, dict(numres=3)),
    "offset_odd": (67, 45, [(1, 1), (2, 2)], 8, dict(numres=3, origin=(3, 5))),
    "tiled_pcrl": (130, 70, [(1, 1), (2, 2), (2, 2)], 8,
                   dict(numres=3, tiles=(64, 32), prog_order="PCRL", precincts=[(16, 16)])),
    "tiled_rpcl_origin": (130, 70, [(1, 1), (2, 2), (2, 2)], 8,
                          dict(numres=3, tiles=(64, 32), tile_origin=(0, 0), origin=(1, 3), prog_order="RPCL",
                               precincts=[(8, 8)])),
    "cprl_dx3": (130, 70, [(1, 1), (2, 2), (3, 2)], 8, dict(numres=3, origin=(1, 3), prog_order="CPRL", precincts=[(8, 8)])),
    "ht_420": (96, 80, [(1, 1), (2, 2), (2, 2)], 8, dict(numres=4, cblk_sty=0x40)),
    "layers_97": (160, 120, [(1, 1), (2, 2), (2, 2)], 8, dict(numres=5, irreversible=True, layer_rate=[20, 10, 1])),
    "comp0_sub": (96, 72, [(2, 2), (1, 1), (1, 1)], 8, dict(numres=3, layer_rate=[12, 4])),
    "mono12_sub": (100, 60, [(1, 1), (4, 4)], 12, dict(numres=3, cblk=(32, 32))),
}


def comp_shape(w, h, dx, dy, origin=(0, 0)):
    x0, y0 = origin
    return -(-(y0 + h) // dy) - -(-y0 // dy), -(-(x0 + w) // dx) - -(-x0 // dx)


def planes(name, seed=7):
    """Smooth-ish random planes (a gradient plus noise) for case `name`, one per component."""
    W, H, sub, prec, kw = CASES[name]
    rng = np.random.default_rng(seed + sum(map(ord, name)))
    origin = kw.get("origin") or kw.get("tile_origin") or (0, 0)
    out = []
    for dx, dy in sub:
        h, w = comp_shape(W, H, dx, dy, origin)
        yy, xx = np.mgrid[0:h, 0:w]
        base = (xx * 3 + yy * 2) % (1 << prec)
        noise = rng.integers(0, 1 << max(1, prec - 3), size=(h, w))
        out.append(((base + noise) % (1 << prec)).astype(np.int32))
    return out


def oracle_kw(name):
    W, H, sub, prec, kw = CASES[name]
    return dict(kw, subsampling=sub)


def engine_params(name):
    """(grok_amd.default_params keyword arguments, encode origin) of case `name`."""
    W, H, sub, prec, kw = CASES[name]
    kw = dict(kw)
    origin = kw.pop("origin", None)
    if "numres" in kw:
        kw["numresolution"] = kw.pop("numres")
    return kw, origin
