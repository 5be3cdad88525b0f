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


TLM_MAX_ENTRIES = (0xFFFF - 4) // 6   # Ltlm is 16 bits: 10,921 six-byte entries per marker


def retlm(header, entries):
    """The main header with its TLM markers replaced by ones listing exactly `entries`
    [(tile, Psot)] (Ttlm u16, Ptlm u32: Stlm = 0x60, TileLengthMarkers::writeBegin), split over
    consecutive markers (Ztlm 0, 1, ...) of at most 10,921 entries each.  A rank's sub-stream
    (main header + its own tile parts) then carries a TLM that matches it.  Headers without
    TLM are returned unchanged."""
    h = bytes(header)
    i, first, out = 2, None, [h[:2]]
    while i + 4 <= len(h):
        m, L = struct.unpack(">HH", h[i:i + 4])
        if m == SOT:
            break
        if m == TLM:
            if first is None:
                first = len(out)
                out.append(b"")   # the new markers go where the first one was
        else:
            out.append(h[i:i + 2 + L])
        i += 2 + L
    out.append(h[i:])
    if first is None:
        return h
    segs = []
    for z, k in enumerate(range(0, max(len(entries), 1), TLM_MAX_ENTRIES)):
        chunk = entries[k:k + TLM_MAX_ENTRIES]
        if z > 255:
            raise ValueError("more than 256 TLM markers")
        segs.append(struct.pack(">HHBB", TLM, 4 + 6 * len(chunk), z, 0x60) +
                    b"".join(struct.pack(">HI", t, n) for t, n in chunk))
    out[first] = b"".join(segs)
    return b"".join(out)


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


# ------------------------------------------------------- device-resident sharding (bench / drop-in)
# The classes below keep every byte in device tensors (torch uint8 on the rank's GPU, or CPU
# tensors under gloo in the tests): collectives move tensors, and only a codestream's main
# header (a few KiB) is read on the host.  A "coder" does the per-rank coding:
#   main_header() -> (header bytes, TLM entry offset or 0)
#   encode_tiles(x_slab, tile_begin, tile_end, row0, out) -> (bytes written to out, [Psot per tile])
#   decode_rows(sub, n, out_slab, row0)        sub: header + the rank's tile parts + EOC
#   decode_window(cs, n, window, out)          window = (x0, y0, x1, y1)
# EngineCoder (below) runs the HIP engine; tests/test_shard.py drives the same classes with the
# CPU oracle standing in.
SIZ = 0xFF51


def parse_main_header(head):
    """A codestream's main header from its first bytes: (length = offset of the first SOT,
    SIZ fields {w, h, tw, th, nc}, [(tile, Psot)] from its TLM markers in order).
    TLM field widths follow Stlm (TileLengthMarkers::read, cache/LengthCache.cpp): ST = 0
    (tiles in order), 1 (u8) or 2 (u16) tile indices; SP = 0 (u16) or 1 (u32) lengths."""
    h = bytes(head)
    i, siz, entries = 2, None, []
    while i + 4 <= len(h):
        m, L = struct.unpack(">HH", h[i:i + 4])
        if m == SOT:
            if siz is None:
                raise ValueError("main header without SIZ")
            return i, siz, entries
        if i + 2 + L > len(h):
            break
        if m == SIZ:
            w, hh, x0, y0, tw, th, tx0, ty0, nc = struct.unpack(">IIIIIIIIH", h[i + 6:i + 40])
            # the image area [x0, w) x [y0, hh) of the canvas, the tile grid anchored at (tx0, ty0)
            siz = dict(w=w - x0, h=hh - y0, tw=tw, th=th, nc=nc, x0=x0, y0=y0, tx0=tx0, ty0=ty0)
        elif m == TLM:
            stlm = h[i + 5]
            st, sp = (stlm >> 4) & 3, (stlm >> 6) & 1
            j, tnext = i + 6, entries[-1][0] + 1 if entries else 0
            while j < i + 2 + L:
                if st == 0:
                    t = tnext
                elif st == 1:
                    t = h[j]
                    j += 1
                else:
                    t = struct.unpack(">H", h[j:j + 2])[0]
                    j += 2
                if sp:
                    n = struct.unpack(">I", h[j:j + 4])[0]
                    j += 4
                else:
                    n = struct.unpack(">H", h[j:j + 2])[0]
                    j += 2
                entries.append((t, n))
                tnext = t + 1
        i += 2 + L
    raise ValueError("the main header does not end within %d bytes" % len(h))


def codestream_start(head):
    """Offset of the codestream in a .jp2 (the jp2c box contents) or 0 for a raw codestream."""
    h = bytes(head)
    if h[:2] == b"\xff\x4f":
        return 0
    i = 0
    while i + 8 <= len(h):
        lbox, tbox = struct.unpack(">I4s", h[i:i + 8])
        hl = 8
        if lbox == 1:
            lbox, hl = struct.unpack(">Q", h[i + 8:i + 16])[0], 16
        if tbox == b"jp2c":
            return i + hl
        if lbox == 0:
            break
        i += lbox
    raise ValueError("no jp2c box in the first %d bytes" % len(h))


def _read_header(cs, n):
    """(codestream offset, header length, SIZ, TLM entries, header bytes) of the stream held in
    the uint8 tensor cs[:n]; only the header bytes are copied to the host."""
    k = min(n, 1 << 16)
    while True:
        head = cs[:k].cpu().numpy().tobytes()
        try:
            off = codestream_start(head)
            hl, siz, ent = parse_main_header(head[off:])
            return off, hl, siz, ent, head[off:off + hl]
        except (ValueError, struct.error):
            if k >= n:
                raise
            k = min(n, 4 * k)


def _tensor(b, device):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(device)


def _scatter_tensors(dist, rank, world, parts, device, error=None):
    """Rank 0's list of per-rank uint8 tensors to every rank (lengths, then the payloads padded
    to the longest): returns (this rank's buffer, its length).  error (rank 0): an exception
    rank 0 met while building `parts`: every rank then raises it (the lengths carry -1), so no
    rank waits in a collective rank 0 never enters."""
    import torch
    n = torch.zeros(1, dtype=torch.int64, device=device)
    ns = None
    if rank == 0:
        ns = [torch.tensor([-1 if error is not None else int(p.numel())], dtype=torch.int64, device=device)
              for p in (parts if error is None else range(world))]
    dist.scatter(n, ns, src=0)
    if int(n.item()) < 0:
        raise error if error is not None else RuntimeError("rank 0 could not build the sub-streams")
    mx = n.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mx = max(int(mx.item()), 1)
    buf = torch.empty(mx, dtype=torch.uint8, device=device)
    if rank == 0:
        srcs = []
        for p in parts:
            if p.numel() == mx:
                srcs.append(p.contiguous())
            else:
                t = torch.zeros(mx, dtype=torch.uint8, device=device)
                t[:p.numel()] = p
                srcs.append(t)
        dist.scatter(buf, srcs, src=0)
    else:
        dist.scatter(buf, None, src=0)
    return buf, int(n.item())


def _as_bytes(t):
    """A sample tensor viewed as bytes along its last axis: the collectives move uint8 (RCCL has
    no 16-bit integer type; gloo none either)."""
    import torch
    return t if t is None or t.element_size() == 1 else t.view(torch.uint8)


def _gather_rows(dist, rank, world, slab, rows, bands, full):
    """Each rank's (C, rows, W) slab into rank 0's `full` at its row band [a, b) (padded to the
    tallest band for the collective)."""
    import torch
    slab, full = _as_bytes(slab), _as_bytes(full)
    hmax = max(max(b - a for a, b in bands), 1)
    if rows == hmax and slab.shape[1] == hmax:
        pad = slab.contiguous()
    else:
        pad = torch.zeros((slab.shape[0], hmax, slab.shape[2]), dtype=slab.dtype, device=slab.device)
        if rows:
            pad[:, :rows] = slab[:, :rows]
    if rank == 0:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.gather(pad, bufs, dst=0)
        y0 = bands[0][0]
        for r, (a, b) in enumerate(bands):
            if b > a and (r or full.data_ptr() != slab.data_ptr()):
                full[:, a - y0:b - y0] = bufs[r][:, :b - a]
    else:
        dist.gather(pad, None, dst=0)


class TileRowShard:
    """A tiled image (single tile-part tiles) coded on `world` ranks, tile rows split into
    contiguous ranges.

    encode(x_slab): every rank codes its tiles from its row slab; the tile-part lengths are
    all-gathered and rank 0 gathers the payloads and writes main header (TLM filled) + tile
    parts in tile order + EOC: the codestream equals a one-GPU encode byte for byte.
    decode(cs, n, out_slab, full): rank 0 reads the main header of its codestream, locates
    every tile part through TLM (no SOT walk), and scatters to each rank a sub-stream (main
    header with a TLM of just its parts + those parts + EOC); each rank decodes its rows into
    out_slab and rank 0 gathers the row slabs into `full`.
    scatter_input(full, slab): rank 0's image rows to every rank's slab."""

    def __init__(self, dist, rank, world, coder, shape, tile_hw, device):
        import torch
        self.dist, self.rank, self.world, self.coder, self.device = dist, rank, world, coder, device
        self.C, self.H, self.W = shape
        self.tw, self.th = tile_hw
        self.ntx, self.nty = tile_grid(self.H, self.W, self.th, self.tw)
        self.ranges = [rank_tiles(self.ntx, self.nty, r, world) for r in range(world)]
        self.tb, self.te = self.ranges[rank][:2]
        self.bands = [(min(self.H, j0 * self.th), min(self.H, j1 * self.th)) for _, _, j0, j1 in self.ranges]
        self.y0, self.y1 = self.bands[rank]
        self.maxt = max(max(te - tb for tb, te, _, _ in self.ranges), 1)
        self.hdr, self.tlm = coder.main_header()
        self.hdr_t = _tensor(self.hdr, device)
        self.eoc = torch.tensor([0xFF, 0xD9], dtype=torch.uint8, device=device)

    def scatter_input(self, full, slab):
        """full: rank 0's (C, H, W) image; slab: this rank's (C, y1-y0, W) rows."""
        import torch
        if self.world == 1:
            if slab.data_ptr() != full.data_ptr():
                slab.copy_(full)
            return
        hmax = max(max(b - a for a, b in self.bands), 1)
        slab, full = _as_bytes(slab), _as_bytes(full)
        buf = torch.empty((self.C, hmax, slab.shape[2]), dtype=torch.uint8, device=self.device)
        srcs = None
        if self.rank == 0:
            srcs = []
            for a, b in self.bands:
                t = torch.zeros_like(buf)
                t[:, :b - a] = full[:, a:b]
                srcs.append(t)
        self.dist.scatter(buf, srcs, src=0)
        slab.copy_(buf[:, :self.y1 - self.y0])

    def encode(self, x_slab, parts):
        """Returns (codestream tensor, length) on rank 0, (None, length) elsewhere."""
        import torch
        n, lens = self.coder.encode_tiles(x_slab, self.tb, self.te, self.y0, parts) if self.te > self.tb else (0, [])
        if self.world == 1:
            h = bytearray(self.hdr)
            if self.tlm:
                for k, v in enumerate(lens):
                    h[self.tlm + 6 * (self.tb + k):self.tlm + 6 * (self.tb + k) + 6] = struct.pack(">HI", self.tb + k, int(v))
            cs = torch.cat([_tensor(h, self.device), parts[:n], self.eoc])
            return cs, int(cs.numel())
        ln = torch.zeros(self.maxt + 1, dtype=torch.int64, device=self.device)
        ln[0] = n
        if lens:
            ln[1:1 + len(lens)] = torch.tensor(lens, dtype=torch.int64)
        lns = [torch.zeros_like(ln) for _ in range(self.world)]
        self.dist.all_gather(lns, ln)
        lns = [v.cpu().tolist() for v in lns]
        mx = max(int(max(v[0] for v in lns)), 1)
        payload = parts[:mx]
        if self.rank != 0:
            self.dist.gather(payload, None, dst=0)
            return None, 0
        bufs = [torch.empty(mx, dtype=torch.uint8, device=self.device) for _ in range(self.world)]
        self.dist.gather(payload, bufs, dst=0)
        h = bytearray(self.hdr)
        if self.tlm:
            for r, (tb, te, _, _) in enumerate(self.ranges):
                for k in range(te - tb):
                    h[self.tlm + 6 * (tb + k):self.tlm + 6 * (tb + k) + 6] = struct.pack(">HI", tb + k, int(lns[r][1 + k]))
        cs = torch.cat([_tensor(h, self.device)] + [b[:int(v[0])] for b, v in zip(bufs, lns)] + [self.eoc])
        return cs, int(cs.numel())

    def substreams(self, cs, n):
        """Rank 0: per-rank sub-streams of the codestream cs[:n], located through its TLM: the
        main header with a TLM of the rank's tile parts, those parts in stream order (each
        located on its own, so tile parts that interleave across tiles stay right), EOC."""
        off, hl, siz, ent, hdr = _read_header(cs, n)
        if not ent:
            raise ValueError("sharded decode needs a TLM marker to locate the tile parts")
        if siz["x0"] or siz["y0"] or siz["tx0"] or siz["ty0"]:
            raise ValueError("tile-row sharding of a stream with image / tile-grid offsets is not supported")
        owner = {t: r for r, (tb, te, _, _) in enumerate(self.ranges) for t in range(tb, te)}
        pos, mine_of = off + hl, [[] for _ in self.ranges]
        for t, L in ent:
            if t in owner:
                mine_of[owner[t]].append((t, pos, L))
            pos += L
        if pos > n:
            raise ValueError("TLM lengths run past the codestream")
        subs = []
        for mine in mine_of:
            if not mine:
                subs.append(cs[:0])
                continue
            subs.append(torch_cat([_tensor(retlm(hdr, [(t, L) for t, _, L in mine]), cs.device)] +
                                  [cs[p:p + L] for _, p, L in mine] + [self.eoc]))
        return subs

    def decode(self, cs, n, out_slab, full=None, gather=True):
        """cs[:n] on rank 0 (ignored elsewhere); out_slab: this rank's (C, y1-y0, W) rows;
        gather (the same on every rank): rank 0 collects the slabs into full, its (C, H, W)."""
        if self.world == 1:
            self.coder.decode_rows(cs, n, out_slab, self.y0)
            if gather and full is not None and full.data_ptr() != out_slab.data_ptr():
                full.copy_(out_slab)
            return
        subs, err = None, None
        if self.rank == 0:
            try:
                subs = self.substreams(cs, n)
            except Exception as e:   # any failure: every rank raises in the scatter, none waits
                err = e
        sub, m = _scatter_tensors(self.dist, self.rank, self.world, subs, self.device, err)
        if self.y1 > self.y0:
            self.coder.decode_rows(sub, m, out_slab, self.y0)
        if gather:
            _gather_rows(self.dist, self.rank, self.world, out_slab, self.y1 - self.y0, self.bands, full)


def torch_cat(ts):
    import torch
    return torch.cat(ts)


class WindowShard:
    """Random-access window decode of a tiled codestream / .jp2 held on rank 0 (C5): the window's
    tile rows are split into contiguous bands, one per rank; rank 0 locates the tile parts each
    band needs through TLM and scatters them (main header with a TLM of just those parts + the
    parts + EOC) — no rank holds the whole file; each rank decodes its band of the window
    (PLT finds the packets, out-of-reach code-blocks are skipped) and rank 0 gathers the bands."""

    def __init__(self, dist, rank, world, coder, device, file=None, n=0):
        import torch
        self.dist, self.rank, self.world, self.coder, self.device = dist, rank, world, coder, device
        self.file, self.n = file, n
        self.eoc = torch.tensor([0xFF, 0xD9], dtype=torch.uint8, device=device)
        meta = torch.zeros(8, dtype=torch.int64, device=device)
        err = None
        if rank == 0:
            try:
                off, hl, siz, ent, hdr = _read_header(file, n)
                if not ent:
                    raise ValueError("window sharding needs a TLM marker")
                self.hdr, self.siz = hdr, siz
                pos, self.where = off + hl, {}
                for t, L in ent:
                    self.where.setdefault(t, []).append((pos, L))
                    pos += L
                meta[:7] = torch.tensor([siz[k] for k in ("tw", "th", "w", "x0", "y0", "tx0", "ty0")])
                meta[7] = 1
            except Exception as e:   # every rank raises below, none waits
                err = e
        if world > 1:
            dist.broadcast(meta, 0)
        if not int(meta[7].item()):
            raise err if err is not None else RuntimeError("rank 0 could not read the window stream's header")
        self.tw, self.th, self.W, self.X0, self.Y0, self.TX0, self.TY0 = (int(v) for v in meta[:7].tolist())

    def bands(self, win):
        """The window's rows [y0, y1) (image coordinates) split into per-rank bands along tile
        rows of the canvas grid: tile row j covers canvas rows [TY0 + j th, TY0 + (j+1) th)."""
        x0, y0, x1, y1 = win
        j0 = (y0 + self.Y0 - self.TY0) // self.th
        j1 = (y1 - 1 + self.Y0 - self.TY0) // self.th + 1
        edge = lambda j: self.TY0 + j * self.th - self.Y0   # image row where tile row j starts
        per, extra = divmod(j1 - j0, self.world)
        out = []
        for r in range(self.world):
            a = j0 + r * per + min(r, extra)
            b = a + per + (1 if r < extra else 0)
            out.append((max(y0, edge(a)), min(y1, edge(b))) if b > a else (y0, y0))
        return out

    def _band_streams(self, win, bands):
        """Rank 0: each band's sub-stream (main header with a TLM of its tile parts, the parts, EOC)."""
        x0, y0, x1, y1 = win
        # canvas tile grid (B.3): ntx columns from TX0 to the image's right edge X0 + W
        ntx = (self.X0 + self.W - self.TX0 + self.tw - 1) // self.tw
        cx, cy = self.X0 - self.TX0, self.Y0 - self.TY0   # image -> grid coordinates
        i0, i1 = (x0 + cx) // self.tw, (x1 - 1 + cx) // self.tw + 1
        subs = []
        for a, b in bands:
            if b <= a:
                subs.append(self.file[:0])
                continue
            tiles = [j * ntx + i for j in range((a + cy) // self.th, (b - 1 + cy) // self.th + 1)
                     for i in range(i0, i1)]
            mine = [(t, p, L) for t in tiles for p, L in self.where.get(t, [])]
            subs.append(torch_cat([_tensor(retlm(self.hdr, [(t, L) for t, _, L in mine]), self.device)] +
                                  [self.file[p:p + L] for _, p, L in mine] + [self.eoc]))
        return subs

    def decode(self, win, out, band_buf=None):
        """out: rank 0's (C, y1-y0, x1-x0) window; band_buf: a (C, >= tallest band, x1-x0) buffer
        on the other ranks (rank 0 decodes its band straight into out)."""
        x0, y0, x1, y1 = win
        if self.world == 1:
            self.coder.decode_window(self.file, self.n, win, out)
            return
        bands = self.bands(win)
        subs, err = None, None
        if self.rank == 0:
            try:
                subs = self._band_streams(win, bands)
            except Exception as e:   # (e.g. retlm: more than 256 TLM entries) every rank raises
                err = e
        sub, m = _scatter_tensors(self.dist, self.rank, self.world, subs, self.device, err)
        a, b = bands[self.rank]
        dst = out[:, a - y0:b - y0] if self.rank == 0 else band_buf[:, :b - a]
        if b > a:
            self.coder.decode_window(sub, m, (x0, a, x1, b), dst)
        slab = out[:, a - y0:b - y0] if self.rank == 0 else band_buf
        _gather_rows(self.dist, self.rank, self.world, slab, b - a, bands, out if self.rank == 0 else None)


class EngineCoder:
    """The coder interface over a grok_amd.Engine (one per rank / GPU)."""

    def __init__(self, engine, image_shape, prec, params):
        self.eng, self.shape, self.prec, self.params = engine, image_shape, prec, params

    def main_header(self):
        h, tlm, _ = self.eng.main_header(self.shape, self.prec, params=self.params)
        return h, tlm

    def encode_tiles(self, x, tb, te, row0, out):
        return self.eng.encode_tiles(x, self.prec, tb, te, image_hw=self.shape[1:], row0=row0, params=self.params,
                                     out=out)

    def decode_rows(self, sub, n, out, row0):
        self.eng.decode(sub, length=n, out=out, row0=row0)

    def decode_window(self, cs, n, win, out):
        self.eng.decode_window(cs, win, length=n, out=out)
