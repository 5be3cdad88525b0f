"""Seeded synthetic test images.

Per component k:
  v = clip(maxv * (0.5 + 0.25*sin(2pi(x/(W/3) + 0.3k)) * cos(2pi(y/(H/2) - 0.2k))
               + 0.15*((x + (k+1)y) mod 257)/257) + N(0, 0.03*maxv), 0, maxv)
noise from numpy default_rng(seed*100003 + row_chunk_start) in 1024-row chunks,
float32 arithmetic, truncation to integer.  Seeds: C1=1, C2=10, C3=11, C4=20, C5=30.
"""
import numpy as np

SEEDS = {"C1": 1, "C2": 10, "C3": 11, "C4": 20, "C5": 30}


def synth_rows(y0, y1, w, c, bits, seed, h):
    rng = np.random.default_rng(seed * 100003 + y0)
    y, x = np.mgrid[y0:y1, 0:w].astype(np.float32)
    maxv = (1 << bits) - 1
    chans = []
    for k in range(c):
        base = 0.5 + 0.25 * np.sin(2 * np.pi * (x / (w / 3.0) + k * 0.3)) * np.cos(2 * np.pi * (y / (h / 2.0) - k * 0.2))
        base += 0.15 * ((x + y * (k + 1)) % 257) / 257.0
        v = np.clip(base * maxv + rng.normal(0, maxv * 0.03, size=(y1 - y0, w)).astype(np.float32), 0, maxv)
        chans.append(v.astype(np.uint16))
    return np.stack(chans, 0)


def synth_image(h, w, c, bits, seed, chunk=1024):
    """Return a (c, h, w) uint16 array identical to the survey's PNM generator."""
    out = np.empty((c, h, w), np.uint16)
    for y0 in range(0, h, chunk):
        y1 = min(h, y0 + chunk)
        out[:, y0:y1, :] = synth_rows(y0, y1, w, c, bits, seed, h)
    return out


def write_pnm(path, img, bits):
    c, h, w = img.shape
    maxv = (1 << bits) - 1
    with open(path, "wb") as f:
        f.write((b"P6" if c == 3 else b"P5") + b"\n%d %d\n%d\n" % (w, h, maxv))
        a = np.ascontiguousarray(img.transpose(1, 2, 0))
        f.write(a.astype(np.uint8).tobytes() if maxv < 256 else a.astype(">u2").tobytes())


def synth_slab(y0, y1, h, w, c, bits, seed, chunk=1024):
    """Rows [y0, y1) of synth_image(h, w, c, bits, seed) without building the rest
    (each rank of a tile-sharded run generates only its own tile rows)."""
    out = np.empty((c, y1 - y0, w), np.uint16)
    for cy in range((y0 // chunk) * chunk, y1, chunk):
        cy1 = min(h, cy + chunk)
        rows = synth_rows(cy, cy1, w, c, bits, seed, h)
        a, b = max(cy, y0), min(cy1, y1)
        out[:, a - y0:b - y0, :] = rows[:, a - cy:b - cy, :]
    return out
