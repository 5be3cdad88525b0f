"""grok_amd/shard.py on streams its own encoder does not write (CPU, gloo world size 2, the
oracle standing in for the per-rank engine as in test_bench_shard.py):

  * tile parts that interleave across tiles (every tile's part 0, then every part 1): each
    rank's sub-stream is cut part by part through TLM, not as one slice;
  * image and tile-grid offsets (-d / -T): WindowShard maps windows to canvas tile rows;
  * errors rank 0 meets before a collective (no TLM) reach every rank instead of leaving the
    others waiting;
  * TLM rewritten over several markers when a sub-stream has more than 10,921 tile parts.
"""
import os
import socket
import struct
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O
from conftest import ROOT
from grok_amd import shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def interleave_parts(cs):
    """A tiled stream with tile parts (-u) rewritten so every tile's part k precedes any part
    k+1 (TLM entries in the new stream order)."""
    header, parts = shard.split_codestream(cs)
    order = sorted(range(len(parts)), key=lambda i: (parts[i][1][10], parts[i][0]))   # (TPsot, tile)
    new = [parts[i] for i in order]
    return shard.retlm(header, [(t, len(b)) for t, b in new]) + b"".join(b for _, b in new) + b"\xff\xd9"


def _run(target, args, nres=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, 2, port, q) + args) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [q.get(timeout=5) for _ in range(nres)]


def _init(rank, world, port):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _w_interleaved(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from test_bench_shard import OracleCoder
        rng = np.random.default_rng(5)
        C, H, W = 3, 160, 192
        img = rng.integers(0, 256, size=(C, H, W)).astype(np.int32)
        kw = dict(tiles=(64, 64), tlm=True, nlayers=2, tile_parts="L")
        cs = interleave_parts(O.encode(img, 8, **kw))
        dev = torch.device("cpu")
        sh = shard.TileRowShard(dist, rank, world, OracleCoder((C, H, W), 8, kw), (C, H, W), (64, 64), dev)
        slab = torch.zeros((C, sh.y1 - sh.y0, W), dtype=torch.uint8)
        full = torch.zeros((C, H, W), dtype=torch.uint8) if rank == 0 else None
        src = torch.frombuffer(bytearray(cs), dtype=torch.uint8) if rank == 0 else None
        sh.decode(src, len(cs) if rank == 0 else 0, slab, full)
        if rank == 0:
            q.put(bool((full.numpy().astype(np.int32) == img).all()))
    finally:
        dist.destroy_process_group()


def test_tilerow_shard_interleaved_tile_parts():
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(3, 160, 192)).astype(np.int32)
    cs = interleave_parts(O.encode(img, 8, tiles=(64, 64), tlm=True, nlayers=2, tile_parts="L"))
    np.testing.assert_array_equal(O.decode(cs)[0], img)   # the rewritten stream is valid
    assert _run(_w_interleaved, ()) == [True]


def _w_offsets(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from test_bench_shard import OracleCoder
        from grok_amd.synth import synth_image
        C, H, W = 3, 150, 170
        img = synth_image(H, W, C, 8, 31).astype(np.int32)
        kw = dict(tiles=(48, 40), tlm=True, plt=True, origin=(17, 9), tile_origin=(5, 2))
        cs = O.encode(img, 8, **kw)
        file = torch.frombuffer(bytearray(cs), dtype=torch.uint8) if rank == 0 else None
        dev = torch.device("cpu")
        ws = shard.WindowShard(dist, rank, world, OracleCoder((C, H, W), 8, kw), dev, file=file,
                               n=len(cs) if rank == 0 else 0)
        ok = True
        for win in [(0, 0, 170, 150), (3, 31, 90, 107), (100, 60, 170, 150), (40, 0, 41, 150)]:
            x0, y0, x1, y1 = win
            out = torch.zeros((C, y1 - y0, x1 - x0), dtype=torch.uint8) if rank == 0 else None
            band = torch.zeros((C, y1 - y0, x1 - x0), dtype=torch.uint8)
            ws.decode(win, out, band)
            if rank == 0:
                ok &= bool((out.numpy().astype(np.int32) == img[:, y0:y1, x0:x1]).all())
        if rank == 0:
            q.put(ok)
    finally:
        dist.destroy_process_group()


def test_window_shard_canvas_offsets():
    assert _run(_w_offsets, ()) == [True]


def _w_errors(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from test_bench_shard import OracleCoder
        rng = np.random.default_rng(6)
        C, H, W = 1, 128, 128
        img = rng.integers(0, 256, size=(C, H, W)).astype(np.int32)
        kw = dict(tiles=(64, 64))   # no TLM
        cs = O.encode(img, 8, **kw)
        dev = torch.device("cpu")
        src = torch.frombuffer(bytearray(cs), dtype=torch.uint8) if rank == 0 else None
        got = []
        try:
            shard.WindowShard(dist, rank, world, OracleCoder((C, H, W), 8, kw), dev, file=src,
                              n=len(cs) if rank == 0 else 0)
        except (ValueError, RuntimeError) as e:
            got.append(type(e).__name__)
        sh = shard.TileRowShard(dist, rank, world, OracleCoder((C, H, W), 8, kw), (C, H, W), (64, 64), dev)
        slab = torch.zeros((C, sh.y1 - sh.y0, W), dtype=torch.uint8)
        try:
            sh.decode(src, len(cs) if rank == 0 else 0, slab, None, gather=False)
        except (ValueError, RuntimeError) as e:
            got.append(type(e).__name__)
        q.put((rank, len(got)))
    finally:
        dist.destroy_process_group()


def test_rank0_errors_reach_every_rank():
    res = sorted(_run(_w_errors, (), nres=2))
    # both ranks raised both times (none of them hung in a collective)
    assert res == [(0, 2), (1, 2)]


def test_retlm_splits_over_markers():
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(1, 64, 64)).astype(np.int32)
    header, _ = shard.split_codestream(O.encode(img, 8, tiles=(32, 32), tlm=True))
    entries = [(t % 65535, 100 + t) for t in range(25000)]
    h = shard.retlm(header, entries)
    i, seen, zs = 2, [], []
    while i + 4 <= len(h):
        m, L = struct.unpack(">HH", h[i:i + 4])
        if m == 0xFF55:
            zs.append(h[i + 4])
            assert L <= 0xFFFF
            seen += [struct.unpack(">HI", h[j:j + 6]) for j in range(i + 6, i + 2 + L, 6)]
        i += 2 + L
    assert zs == [0, 1, 2] and seen == entries
    assert shard.parse_main_header(h + b"\xff\x90\x00\x0a")[2] == entries


def _w_window_errors(rank, world, port, q):
    # rank 0 failing while it cuts a window's band sub-streams (any exception type: an IndexError
    # from a bad TLM offset here) reaches every rank through the scatter
    dist = _init(rank, world, port)
    try:
        from test_bench_shard import OracleCoder
        rng = np.random.default_rng(8)
        C, H, W = 1, 128, 128
        img = rng.integers(0, 256, size=(C, H, W)).astype(np.int32)
        kw = dict(tiles=(32, 32), tlm=True)
        cs = O.encode(img, 8, **kw)
        dev = torch.device("cpu")
        src = torch.frombuffer(bytearray(cs), dtype=torch.uint8) if rank == 0 else None
        ws = shard.WindowShard(dist, rank, world, OracleCoder((C, H, W), 8, kw), dev, file=src,
                               n=len(cs) if rank == 0 else 0)
        if rank == 0:
            def bad(win, bands):
                raise IndexError("tile part offset past the file")
            ws._band_streams = bad
        out = torch.zeros((C, H, W), dtype=torch.uint8) if rank == 0 else None
        band = torch.zeros((C, H, W), dtype=torch.uint8)
        got = None
        try:
            ws.decode((0, 0, W, H), out, band)
        except (IndexError, RuntimeError) as e:
            got = type(e).__name__
        # the group is still usable afterwards: a clean window decodes
        if rank == 0:
            del ws._band_streams
        ws.decode((0, 0, W, H), out, band)
        ok = bool((out.numpy().astype(np.int32) == img).all()) if rank == 0 else True
        q.put((rank, got, ok))
    finally:
        dist.destroy_process_group()


def test_window_band_errors_reach_every_rank():
    res = sorted(_run(_w_window_errors, (), nres=2))
    assert res == [(0, "IndexError", True), (1, "RuntimeError", True)]
