"""bench.py's multi-GPU runners on CPU: world size 2 over gloo, with the CPU oracle standing in
for the per-rank engine (the coder interface of grok_amd.shard).  ShardRunner (C4: rank 0's
image -> scattered tile rows -> per-rank tile parts -> codestream assembled on rank 0 ->
TLM-located parts scattered -> per-rank decode -> rows gathered on rank 0) and C5Runner
(random windows of a .jp2 held by rank 0: each rank receives only the tile parts of its band
of the window) run their real step() code; the assembled codestream must equal the
one-process oracle encode byte for byte and every gathered image / window must equal the
source."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O
from conftest import ROOT


class OracleCoder:
    """grok_amd.shard's coder interface over the CPU oracle (CPU tensors)."""

    def __init__(self, shape, bits, kw):
        self.shape, self.bits, self.kw = shape, bits, kw

    def main_header(self):
        C, H, W = self.shape
        return O.main_header(W, H, C, self.bits, **self.kw)

    def encode_tiles(self, x, tb, te, row0, out):
        blob, lens = O.encode_tile_parts(x.numpy().view(np.uint16) if x.dtype == torch.int16 else x.numpy(), row0,
                                         self.shape[1:], self.bits, tb, te, **self.kw)
        out[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        return len(blob), lens

    def _decode(self, cs, n):
        d, _ = O.decode(cs[:n].numpy().tobytes())
        return d

    def decode_rows(self, sub, n, out, row0):
        d = self._decode(sub, n)[:, row0:row0 + out.shape[1]]
        out.copy_(torch.from_numpy(d.astype(np.uint16).view(np.int16) if out.dtype == torch.int16 else d.astype(np.uint8)))

    def decode_window(self, cs, n, win, out):
        x0, y0, x1, y1 = win
        out.copy_(torch.from_numpy(self._decode(cs, n)[:, y0:y1, x0:x1].astype(np.uint8)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, what, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from grok_amd.synth import synth_image
        dev = torch.device("cpu")
        if what == "c4":
            size, tiles = 256, (64, 64)
            bench.CONFIGS["C4"] = dict(bench.CONFIGS["C4"], params=dict(bench.CONFIGS["C4"]["params"], tiles=tiles))
            cfg = bench.CONFIGS["C4"]
            kw = dict(cblk_sty=0x40, tiles=tiles, tlm=True, plt=True)
            r = bench.ShardRunner("C4", size, rank, world, dev, dist, coder=OracleCoder((1, size, size), 16, kw))
            r.check()
            r.step()
            if rank == 0:
                img = synth_image(size, size, 1, 16, cfg["seed"]).astype(np.int32)
                full = O.encode(img, 16, **kw)
                got = r.cs[:r.n].numpy().tobytes()
                dec = r.y_full.numpy().view(np.uint16).astype(np.int32)
                q.put((got == full, bool((dec == img).all())))
        else:
            size, tiles = 192, (64, 64)
            kw = dict(tiles=tiles, tlm=True, plt=True, jp2=True)
            img = synth_image(size, size, 3, 8, 30).astype(np.int32)
            file = n = None
            if rank == 0:
                cs = O.encode(img, 8, **kw)
                file, n = torch.frombuffer(bytearray(cs), dtype=torch.uint8), len(cs)
            wins = [(0, 0, 64, 64), (37, 50, 161, 150), (150, 170, 192, 192), (10, 5, 190, 187)]
            r = bench.C5Runner(rank, world, dev, dist, size=size, windows=wins,
                               coder=OracleCoder((3, size, size), 8, kw), file=file, n=n)
            r.check()
            r.step()
            if rank == 0:
                ok = all(np.array_equal(o.numpy(), img[:, y0:y1, x0:x1]) for o, (x0, y0, x1, y1) in zip(r.outs, wins))
                q.put((True, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("what", ["c4", "c5"])
def test_bench_runner_world2_gloo(what):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, what, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    same_cs, exact = q.get(timeout=5)
    assert same_cs, "assembled codestream differs from the one-process encode"
    assert exact, "gathered decode differs from the source"
