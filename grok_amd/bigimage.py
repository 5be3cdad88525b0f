"""Large tiled images (BASELINE config C5: 32768x32768 RGB8 .jp2, 1024x1024 tiles,
TLM + PLT) built slab by slab on one GPU.

A 32768^2 RGB image is 3 GiB of 8-bit samples; coding it as one call would size
every per-block buffer for 3 x 1024 x 259 code-blocks at once.  Instead each
tile row is generated (seeded synthetic rows, several host threads), uploaded as
planar u8 samples and coded with gk_encode_tiles into its tile parts; the parts
are appended in a device buffer and the file is closed with the main header
(TLM filled from the part lengths, CodeStreamCompress::writeTilePart /
TileLengthMarkers::writeEnd) and the JP2 boxes (FileFormatCompress).  The
result is byte-identical to a one-call encode of the whole image.
"""
from concurrent.futures import ThreadPoolExecutor
import struct

import numpy as np

from .synth import synth_rows


def slabs(h, w, c, bits, seed, rows, threads=8):
    """Yield (y0, (c, y1 - y0, w) array) for consecutive row slabs of the seeded synthetic
    image (grok_amd.synth, 1024-row RNG chunks; `rows` a multiple of 1024), generated
    `threads` slabs ahead on a thread pool (numpy releases the GIL in the heavy loops)."""
    assert rows % 1024 == 0 or rows >= h
    dt = np.uint8 if bits <= 8 else np.uint16

    def make(y0):
        y1 = min(h, y0 + rows)
        out = np.empty((c, y1 - y0, w), dt)
        for cy in range(y0, y1, 1024):
            out[:, cy - y0:min(y1, cy + 1024) - y0] = synth_rows(cy, min(h, cy + 1024), w, c, bits, seed, h)
        return out

    starts = list(range(0, h, rows))
    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(make, y0) for y0 in starts[:threads]]
        for i, y0 in enumerate(starts):
            s = futs[i].result()
            futs[i] = None
            if i + threads < len(starts):
                futs.append(ex.submit(make, starts[i + threads]))
            yield y0, s


def encode_tiled(eng, shape, bits, params, slab_iter, device, crops=None, progress=None):
    """Encode an image delivered as tile-row slabs.  shape = (C, H, W); params carries the
    tile size (t_width/t_height) and cod_format (JP2 or raw); slab_iter yields (y0, slab)
    with slab rows aligned to tile rows.  Returns (uint8 device tensor holding the file,
    its length).  crops: optional {name: (x0, y0, x1, y1)} -> filled with the source
    samples of those windows (host copies, for checking window decodes)."""
    import torch
    C, H, W = shape
    th, tw = params.t_height, params.t_width
    ntx = (W + tw - 1) // tw
    crop_out = {}
    if crops:
        for k, (x0, y0, x1, y1) in crops.items():
            crop_out[k] = np.empty((C, y1 - y0, x1 - x0), np.uint8 if bits <= 8 else np.uint16)
    parts, lens, total = [], [], 0
    cap = None
    buf = None
    for y0, slab in slab_iter:
        rows = slab.shape[1]
        assert y0 % th == 0 and (rows % th == 0 or y0 + rows == H)
        for k, (x0, wy0, x1, wy1) in (crops or {}).items():
            a, b = max(y0, wy0), min(y0 + rows, wy1)
            if a < b:
                crop_out[k][:, a - wy0:b - wy0] = slab[:, a - y0:b - y0, x0:x1]
        x = torch.from_numpy(slab.view(np.int16) if slab.dtype == np.uint16 else slab).to(device)
        if buf is None:
            cap = x.numel() * x.element_size() * 2 + (16 << 20)
            buf = torch.empty(cap, dtype=torch.uint8, device=device)
        tb, te = (y0 // th) * ntx, ((y0 + rows + th - 1) // th) * ntx
        n, ln = eng.encode_tiles(x, bits, tb, te, image_hw=(H, W), row0=y0, params=params, out=buf)
        parts.append(buf[:n].clone())
        lens += ln
        total += n
        if progress:
            progress(y0 + rows, H)
    raw = int(params.cod_format)
    params.cod_format = 0
    try:
        hdr, tlm, nt = eng.main_header(shape, bits, params=params)
    finally:
        params.cod_format = raw
    assert nt == len(lens)
    h = bytearray(hdr)
    if tlm:
        for t, n in enumerate(lens):
            h[tlm + 6 * t:tlm + 6 * t + 6] = struct.pack(">HI", t, n)
    cs_len = len(h) + total + 2
    pre = eng.jp2_header(shape, bits, cs_len) if raw == 2 else b""
    out = torch.empty(len(pre) + cs_len, dtype=torch.uint8, device=device)
    head = torch.frombuffer(bytearray(pre) + h, dtype=torch.uint8).to(device)
    out[:head.numel()] = head
    o = head.numel()
    for p in parts:
        out[o:o + p.numel()] = p
        o += p.numel()
    out[o:o + 2] = torch.tensor([0xFF, 0xD9], dtype=torch.uint8, device=device)
    return out, out.numel(), crop_out
