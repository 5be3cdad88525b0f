"""Tile sharding across ranks: one process per GPU, tile rows
split into contiguous ranges, no collective on the coding path.

Encode: every rank codes its tiles (gk_encode_tiles) into tile parts; rank 0
gathers (lengths, then payload) and writes main header + TLM + tile parts in
tile order + EOC — the codestream is byte-identical to a one-GPU encode.
Decode: rank 0 splits the codestream into tile parts (SOT/Psot walk, what TLM
records) and scatters to each rank the main header (TLM rewritten to that rank's
parts) + its tile parts; each rank decodes only those tile rows; rank 0 gathers
the decoded row slabs as tensors.

The collectives are plain torch.distributed calls (RCCL on MI355X, gloo on CPU
for the world-size-2 tests); the codestream logic here is pure Python.
"""
import struct

import numpy as np

SOT, SOD, EOC, TLM = 0xFF90, 0xFF93, 0xFFD9, 0xFF55


def tile_grid(h, w, th, tw):
    """(tiles across, tiles down) for nominal tile size (tw, th)."""
    return (w + tw - 1) // tw, (h + th - 1) // th


def rank_tiles(ntx, nty, rank, world):
    """Contiguous tile-row range of this rank: (tile_begin, tile_end, row_begin, row_end)."""
    per, extra = divmod(nty, world)
    j0 = rank * per + min(rank, extra)
    j1 = j0 + per + (1 if rank < extra else 0)
    return j0 * ntx, j1 * ntx, j0, j1


def split_codestream(cs):
    """Main header bytes and [(tile index, tile-part bytes)] of a codestream
    (CodeStreamDecompress SOT handling: Isot, Psot)."""
    cs = bytes(cs)
    i = 2
    while i + 4 <= len(cs):
        m = struct.unpack(">H", cs[i:i + 2])[0]
        if m == SOT:
            break
        i += 2 + struct.unpack(">H", cs[i + 2:i + 4])[0]
    header, parts = cs[:i], []
    while i + 12 <= len(cs) and struct.unpack(">H", cs[i:i + 2])[0] == SOT:
        isot, psot = struct.unpack(">HI", cs[i + 4:i + 10])
        end = i + psot if psot else len(cs) - 2
        parts.append((isot, cs[i:end]))
        i = end
    return header, parts


def assemble(header, tlm_offset, parts):
    """header (from gk_main_header) + tile parts in tile order + EOC; fills the TLM
    entries (Ttlm u16, Ptlm u32, TileLengthMarkers::writeEnd) when tlm_offset != 0."""
    h = bytearray(header)
    parts = sorted(parts, key=lambda p: p[0])
    if tlm_offset:
        for k, (t, b) in enumerate(parts):
            h[tlm_offset + 6 * k:tlm_offset + 6 * k + 6] = struct.pack(">HI", t, len(b))
    return bytes(h) + b"".join(b for _, b in parts) + struct.pack(">H", EOC)


def split_parts(blob, lens, tile_begin):
    """Back-to-back tile parts (gk_encode_tiles output) -> [(tile, bytes)]."""
    out, o = [], 0
    for k, n in enumerate(lens):
        out.append((tile_begin + k, bytes(blob[o:o + n])))
        o += n
    return out


# ----------------------------------------------------------------- collectives
def gather_bytes(dist, payload, rank, world, device=None):
    """Variable-length byte strings to rank 0: lengths first, then the payload
    (padded to the longest).  payload: bytes (CPU) or a 1-D uint8 torch tensor.
    Returns a list of per-rank byte tensors on rank 0, None elsewhere."""
    import torch
    if isinstance(payload, torch.Tensor):
        t = payload
    else:
        t = torch.from_numpy(np.frombuffer(bytes(payload), np.uint8).copy()) if len(payload) else \
            torch.zeros(0, dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    mx = int(max(int(x.item()) for x in ns))
    buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=t.device)
    buf[:t.numel()] = t
    if rank == 0:
        bufs = [torch.empty(max(mx, 1), dtype=torch.uint8, device=t.device) for _ in range(world)]
        dist.gather(buf, bufs, dst=0)
        return [b[:int(k.item())] for b, k in zip(bufs, ns)]
    dist.gather(buf, None, dst=0)
    return None


def gather_lens(dist, lens, rank, world, device=None):
    """Per-rank lists of tile-part lengths to rank 0."""
    raw = np.asarray(list(lens), dtype="<i8").tobytes()
    out = gather_bytes(dist, raw, rank, world, device)
    if out is None:
        return None
    return [np.frombuffer(o.cpu().numpy().tobytes(), "<i8").tolist() for o in out]


def encode_sharded(dist, rank, world, encode_tiles, main_header, ntx, nty, device=None):
    """encode_tiles(tile_begin, tile_end) -> (blob, lens) for this rank's tiles;
    main_header() -> (header, tlm_offset).  Returns the full codestream on rank 0."""
    tb, te, _, _ = rank_tiles(ntx, nty, rank, world)
    blob, lens = encode_tiles(tb, te) if te > tb else (b"", [])
    blobs = gather_bytes(dist, blob, rank, world, device)
    all_lens = gather_lens(dist, lens, rank, world, device)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        rtb = rank_tiles(ntx, nty, r, world)[0]
        parts += split_parts(blobs[r].cpu().numpy().tobytes(), all_lens[r], rtb)
    header, tlm = main_header()
    return assemble(header, tlm, parts)


def retlm(header, entries):
    """The main header with its TLM marker rewritten to list exactly `entries` [(tile, Psot)]
    (Ttlm u16, Ptlm u32: Stlm = 0x60, TileLengthMarkers::writeBegin).  A rank's sub-stream
    (main header + its own tile parts) then carries a TLM that matches it.  Headers without
    TLM are returned unchanged."""
    h = bytes(header)
    i = 2
    while i + 4 <= len(h):
        m, L = struct.unpack(">HH", h[i:i + 4])
        if m == TLM:
            seg = struct.pack(">HHBB", TLM, 4 + 6 * len(entries), 0, 0x60) + \
                b"".join(struct.pack(">HI", t, n) for t, n in entries)
            return h[:i] + seg + h[i + 2 + L:]
        i += 2 + L
    return h


def _scatter_bytes(dist, rank, world, payloads, device):
    """Rank 0's per-rank byte strings to every rank (lengths, then payloads padded to the
    longest) with two scatter collectives.  Returns this rank's bytes as a uint8 tensor."""
    import torch
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == 0:
        ns = [torch.tensor([len(p)], dtype=torch.int64, device=device) for p in payloads]
        dist.scatter(n, ns, src=0)
    else:
        dist.scatter(n, None, src=0)
    mx = torch.tensor([int(n.item())], dtype=torch.int64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mx = max(int(mx.item()), 1)
    buf = torch.empty(mx, dtype=torch.uint8, device=device)
    if rank == 0:
        srcs = []
        for p in payloads:
            t = torch.zeros(mx, dtype=torch.uint8)
            if len(p):
                t[:len(p)] = torch.frombuffer(bytearray(p), dtype=torch.uint8)
            srcs.append(t.to(device))
        dist.scatter(buf, srcs, src=0)
    else:
        dist.scatter(buf, None, src=0)
    return buf[:int(n.item())]


def decode_sharded(dist, rank, world, cs, decode, ntx, nty, th, shape, device=None):
    """Rank 0 holds the codestream (host bytes).  It cuts the tile parts (SOT walk) and
    scatters to every rank its main header (TLM rewritten to its own parts) + tile parts +
    EOC; each rank decodes its tile rows with decode(sub_tensor, y0, y1) -> (C, y1-y0, W)
    tensor; rank 0 gathers the row slabs (padded to the tallest) and returns the (C, H, W)
    image.  Every transfer is a torch.distributed collective on uint8 / sample tensors
    (RCCL over xGMI with device tensors; gloo with CPU tensors in the tests)."""
    import torch
    C, H, W = shape
    device = device or torch.device("cpu")
    subs = None
    if rank == 0:
        header, parts = split_codestream(cs)
        pl = dict(parts)
        subs = []
        for r in range(world):
            tb, te, _, _ = rank_tiles(ntx, nty, r, world)
            mine = [(t, pl[t]) for t in range(tb, te) if t in pl]
            subs.append(retlm(header, [(t, len(b)) for t, b in mine]) + b"".join(b for _, b in mine) +
                        struct.pack(">H", EOC) if mine else b"")
    sub = _scatter_bytes(dist, rank, world, subs, device)
    _, _, j0, j1 = rank_tiles(ntx, nty, rank, world)
    y0, y1 = min(H, j0 * th), min(H, j1 * th)
    rows_max = max(min(H, rank_tiles(ntx, nty, r, world)[3] * th) - min(H, rank_tiles(ntx, nty, r, world)[2] * th)
                   for r in range(world))
    slab = None
    if y1 > y0:
        slab = decode(sub, y0, y1)
        if not isinstance(slab, torch.Tensor):
            slab = torch.from_numpy(np.ascontiguousarray(slab))
    dtype = slab.dtype if slab is not None else torch.int32
    pad = torch.zeros((C, max(rows_max, 1), W), dtype=dtype, device=device)
    if slab is not None:
        pad[:, :y1 - y0] = slab.to(device)
    if rank == 0:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.gather(pad, bufs, dst=0)
        full = torch.empty((C, H, W), dtype=dtype, device=device)
        for r in range(world):
            _, _, a, b = rank_tiles(ntx, nty, r, world)
            ry0, ry1 = min(H, a * th), min(H, b * th)
            if ry1 > ry0:
                full[:, ry0:ry1] = bufs[r][:, :ry1 - ry0]
        return full
    dist.gather(pad, None, dst=0)
    return None
