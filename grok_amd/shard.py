"""Tile sharding across ranks: one process per GPU, tile rows
split into contiguous ranges, no collective on the coding path.

Encode: every rank codes its tiles (gk_encode_tiles) into tile parts; rank 0
gathers (lengths, then payload) and writes main header + TLM + tile parts in
tile order + EOC — the codestream is byte-identical to a one-GPU encode.
Decode: rank 0 splits the codestream into tile parts (SOT/Psot walk, what TLM
records), each rank receives the main header + its tile parts and decodes only
those tile rows; rank 0 gathers the decoded rows.

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


def decode_sharded(dist, rank, world, cs, decode, ntx, nty, th):
    """Rank 0 holds the codestream; every rank decodes header + its tile parts with
    decode(substream) -> (C, H, W) array (rows of other tiles untouched / zero).
    Returns the full decoded image on rank 0 (rows gathered per rank)."""
    import torch
    objs = [None]
    if rank == 0:
        header, parts = split_codestream(cs)
        per_rank = []
        for r in range(world):
            tb, te, _, _ = rank_tiles(ntx, nty, r, world)
            per_rank.append(header + b"".join(b for t, b in parts if tb <= t < te) + struct.pack(">H", EOC))
        objs = [per_rank]
    dist.broadcast_object_list(objs, src=0)
    tb, te, _, _ = rank_tiles(ntx, nty, rank, world)
    img = decode(objs[0][rank]) if te > tb else None   # ranks without tiles stay idle
    out = [None] * world if rank == 0 else None
    dist.gather_object(img, out, dst=0)
    if rank != 0:
        return None
    full = np.zeros_like(next(o for o in out if o is not None))
    for r in range(world):
        _, _, j0, j1 = rank_tiles(ntx, nty, r, world)
        if j1 <= j0:
            continue
        y0, y1 = j0 * th, min(full.shape[1], j1 * th)
        full[:, y0:y1] = out[r][:, y0:y1]
    return full
