"""Benchmark: Mpixels/s encode+decode, JPEG 2000 tile pipeline on MI355X.

Headline workload = BASELINE.json's metric as named, "8K RGB 5/3 lossless + 9/7 lossy": one
step encodes and decodes one image of each of
  C2  configs[1]: 8192x8192 8-bit RGB, 5/3 reversible lossless + RCT, 64x64 code-blocks,
      6 resolutions, single tile, one quality layer (Grok's default coding parameters), and
  C3  configs[2]: 8192x8192 12-bit RGB, 9/7 irreversible + ICT, 3 quality layers -r 40,20,10
      (PCRD rate control),
synthetic input from the survey's seeded generator (grok_amd/synth.py, seeds 10 / 11 + rank).
Encode = image resident in HBM -> codestream resident in HBM; decode = codestream in HBM ->
image in HBM; host T2 (packet headers, rate allocation) runs inside the step.  value = pixels
of all ranks (2 x 8192^2 per rank per step) / max-over-ranks wall time.  Single-tile configs run
as replicas (one C2 + C3 pair per GPU, no collective on the data path): scaling = "weak".  The
line also carries C2 and C3 timed alone (`per_config`).

The same JSON line carries auxiliary measurements:
  C4  configs[3]: 16384^2 16-bit mono, HTJ2K, 1024^2 tiles, TLM + PLT — with N > 1
      ranks tile rows are sharded (strong scaling): each rank codes its tile rows,
      rank 0 gathers the tile parts over RCCL, each rank decodes its own parts;
  C5  configs[4]: decode-only random windows of a 32768^2 RGB8 tiled .jp2 (1024^2
      tiles, TLM + PLT): the four SURVEY windows per step; with N > 1 ranks each
      window's tile rows are split over the ranks and rank 0 gathers the rows;
  C2_batch2: two C2 images in flight per GPU (serving throughput, never `value`).
  C3_batch2: two C3 images in flight per GPU (host PCRD overlapped with GPU work).

`cpu_baseline`: the oracle (CPU restatement, byte-exact with Grok by the fixtures)
on bounded crops of C2 / C3 / C4, median of 3 runs, at 1 and N host threads.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4] [--no-aux]
With --gpus N > 1 and no WORLD_SIZE in the environment the script starts N rank
processes itself (torch.distributed.run) before touching the GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak
CLOCK_GHZ = 2.4            # MI355X max engine clock (MI355X_MICROARCH.md)
METRIC = "Mpixels/s encode+decode, 8K RGB 5/3 lossless + 9/7 lossy, 1/2/4/8 GPU"
# Grok 9.2.0 on the survey container (8 vCPU), enc+dec Mpix/s
GROK_CPU = {"C2p_8t": 5.99, "C2p_1t": 1.11, "C3p_8t": 2.87, "C3p_1t": 0.93, "C4_8t": 51.9, "C4_1t": 19.3,
            "C5_w16k_8t": 12.8}

CONFIGS = {
    "C2": dict(size=8192, comps=3, bits=8, seed=10, params=dict(),
               desc="8192x8192 8-bit RGB, 5/3 lossless + RCT, 64x64 code-blocks, 6 resolutions, single tile, 1 layer"),
    "C3": dict(size=8192, comps=3, bits=12, seed=11, params=dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0]),
               desc="8192x8192 12-bit RGB, 9/7 + ICT, 64x64 code-blocks, 6 resolutions, single tile, "
                    "3 layers -r 40,20,10 (PCRD)"),
    "C4": dict(size=16384, comps=1, bits=16, seed=20,
               params=dict(cblk_sty=0x40, tiles=(1024, 1024), tlm=True, plt=True),
               desc="16384x16384 16-bit mono, HTJ2K, 5/3 lossless, 1024x1024 tiles, TLM + PLT (-M 64 -t 1024,1024 -X -L)"),
    "C5": dict(size=32768, comps=3, bits=8, seed=30, params=dict(tiles=(1024, 1024), tlm=True, plt=True, jp2=True),
               desc="decode-only random windows of a 32768x32768 8-bit RGB tiled .jp2 (5/3, 1024x1024 tiles, TLM + "
                    "PLT; -t 1024,1024 -X -L): windows 0,0,1024,1024 / 12345,23456,16441,27552 / "
                    "30000,30000,32768,32768 / 8000,8000,24384,24384, decoded to u8 planes in HBM"),
}
C5_WINDOWS = [(0, 0, 1024, 1024), (12345, 23456, 16441, 27552), (30000, 30000, 32768, 32768),
              (8000, 8000, 24384, 24384)]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=0, help="override the config's image side")
    ap.add_argument("--config", default="C2+C3", choices=["C2+C3", "C2", "C3", "C4"],
                    help="C2+C3: the headline metric (one 5/3 and one 9/7 image per step)")
    ap.add_argument("--no-aux", action="store_true", help="skip the auxiliary C3/C4/C5/batch measurements")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 window-decode measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="N for the N-thread CPU baseline (0: the host share)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group / timing plumbing only (CPU, gloo, no engine): for tests")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """Start --gpus rank processes (one per GPU) with torch.distributed.run and return its
    exit code.  Called before this process touches the GPU; the ranks find WORLD_SIZE set."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def host_threads(args):
    """Threads of the N-thread CPU baseline: the host CPU share this process may use.  The GPU
    box gives one GPU's job a 16-CPU share (it exports OMP_NUM_THREADS=16) while os.cpu_count()
    reports the whole machine, so the share, not os.cpu_count(), is what the baseline can use."""
    if args.cpu_threads:
        return args.cpu_threads
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
    return max(1, min(share, aff, os.cpu_count() or 1))


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(nthreads):
    """The oracle (CPU restatement, byte-exact with Grok by the committed fixtures) timed on
    bounded crops of the same synthetic images: encode + decode, median of 3 runs, at 1 and
    nthreads threads (code-blocks / tiles on worker threads)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from grok_amd.synth import synth_image
    cases = {
        "C2": (synth_image(2048, 2048, 3, 8, 10).astype(np.int32), 8, dict(), "2048x2048 crop of C2 (RGB8 5/3)"),
        "C3": (synth_image(1024, 1024, 3, 12, 11).astype(np.int32), 12,
               dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0]), "1024x1024 crop of C3 (RGB12 9/7 -r 40,20,10)"),
        "C4": (synth_image(2048, 2048, 1, 16, 20).astype(np.int32), 16,
               dict(cblk_sty=0x40, tiles=(1024, 1024), tlm=True, plt=True), "2048x2048 crop of C4 (mono16 HT tiles)"),
    }
    per = {}
    for name, (img, bits, kw, desc) in cases.items():
        c, h, w = img.shape
        per[name] = {"sample": desc}
        for th in sorted({1, nthreads}):
            O.set_threads(th)
            runs = []
            for _ in range(3):
                t0 = time.perf_counter()
                cs = O.encode(img, bits, **kw)
                dec, _ = O.decode(cs)
                runs.append(time.perf_counter() - t0)
            if not kw.get("irreversible"):
                assert (dec == img).all()
            per[name]["%dt" % th] = round(h * w / 1e6 / float(np.median(runs)), 4)
    O.set_threads(1)
    # the headline's unit of work: one C2 pixel and one C3 pixel (harmonic mean of the two rates)
    comb = lambda t: round(2.0 / (1.0 / per["C2"][t] + 1.0 / per["C3"][t]), 4)
    return {"value": comb("%dt" % nthreads), "unit": "Mpixels/s", "cores": nthreads,
            "cores_list": sorted({1, nthreads}), "value_1t": comb("1t"),
            "host_cpu_count": os.cpu_count(),
            "cores_note": "threads = the CPU share of this GPU's job (OMP_NUM_THREADS / affinity); os.cpu_count() "
                          "reports the whole host, which the box shares between GPUs",
            "kind": "port",
            "sample": "oracle/j2k_oracle.cpp encode+decode, median of 3, on crops: C2 2048^2, C3 1024^2, C4 2048^2; "
                      "value = C2 + C3 crops combined as the headline (one 5/3 and one 9/7 pixel per unit) at %d "
                      "threads" % nthreads,
            "per_config": per,
            "grok_container_8vcpu": {"note": "BASELINE.md section 2, Grok 9.2.0 CLI on the survey container (8 vCPU), "
                                             "enc+dec Mpix/s; C2p/C3p = -c [256,256] variants (Grok cannot decode the "
                                             "single-precinct 8K streams)", **GROK_CPU}}


def profile_file(config, kind):
    """The committed counter summary bench.py reports for (config, kind = "pmc" | "sq"): the file
    named in profiles/current.json ({"C2_pmc": "r05_C2_pmc.json", ...}, written with the profiles
    of the build they were measured on), else None.  An explicit manifest, not the newest-sorting
    name, so adding a profile never silently changes which counters a bench line carries."""
    man = os.path.join(ROOT, "profiles", "current.json")
    try:
        name = json.load(open(man)).get("%s_%s" % (config, kind))
    except (OSError, ValueError):
        return None
    f = os.path.join(ROOT, "profiles", name) if name else None
    return f if f and os.path.exists(f) else None


def ht_issue_roofline(stages, config="C4"):
    """Issue roofline of the HTJ2K coders (one lane per code-block, branchy per-lane chains):
    instructions issued per wave (VALU + SALU + LDS) from the committed SQ counter summary of this
    config named in profiles/current.json (tools/sq_counters.sh + tools/sq_summary.py),
    times 4 cycles (a lone wave issues one instruction per 4 cycles), times the waves a SIMD
    holds (ceil(waves / 1,024)), over the live coder time.  None if no summary exists."""
    f = profile_file(config, "sq")
    if not f:
        return None
    d = json.load(open(f))
    out = {}
    for kern, ms_key in (("k_ht_dec", "dec_t1_coder_ms"), ("k_ht_enc", "enc_t1_coder_ms")):
        if kern not in d or not stages.get(ms_key):
            continue
        k = d[kern]
        insts = sum(k["insts_per_wave"].get(t, 0.0) for t in ("valu", "salu", "lds"))
        per_simd = -(-int(k["waves"]) // 1024)
        floor_ms = per_simd * insts * 4 / (CLOCK_GHZ * 1e6)
        out[kern] = {"bound": "instruction issue of the longest chain (one lane per block)",
                     "instructions_per_wave": round(insts), "waves": int(k["waves"]), "waves_per_simd": per_simd,
                     "floor_ms": round(floor_ms, 3), "measured_ms": round(stages[ms_key], 3),
                     "frac": round(floor_ms / stages[ms_key], 3),
                     "wait_any": round(k["wait_any"], 3), "source": os.path.basename(f)}
    return out or None


def pmc_traffic(kernels, config="C2"):
    """HBM bytes per launch of `kernels` from the committed PMC summary of this config named in
    profiles/current.json (written by tools/pmc_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this benchmark, tools/gpu_profile_all.sh; FETCH_SIZE
    doubled per MI355X_MICROARCH.md's gfx950 note).  (None, None) if no summary exists."""
    f = profile_file(config, "pmc")
    if not f:
        return None, None
    d = json.load(open(f))
    tot = 0.0
    for k in kernels:
        if k not in d:
            return None, None
        tot += d[k]["hbm_bytes_per_launch"]
    return tot, os.path.basename(f)


# ----------------------------------------------------------------------------- runners
class Runner:
    def __init__(self, name, size, rank, device):
        import torch
        import grok_amd as G
        from grok_amd.synth import synth_image
        cfg = CONFIGS[name]
        size = size or cfg["size"]
        self.name, self.cfg, self.size = name, cfg, size
        self.img = synth_image(size, size, cfg["comps"], cfg["bits"], cfg["seed"] + rank)
        self.x = torch.from_numpy(self.img.astype(np.int32)).to(device).contiguous()
        self.out = torch.empty(self.x.numel() * 4 + (1 << 24), dtype=torch.uint8, device=device)
        self.y = torch.empty_like(self.x)
        self.eng = G.Engine(device.index or 0)
        self.params = G.default_params(**cfg["params"])
        self.n = 0
        self.pixels = size * size

    def step(self):
        self.n = self.eng.encode(self.x, self.cfg["bits"], params=self.params, out=self.out)
        te = self.eng.timings()
        self.eng.decode(self.out, length=self.n, out=self.y)
        td = self.eng.timings()
        return te, td

    def check(self):
        import torch
        self.step()
        torch.cuda.synchronize()
        if not self.cfg["params"].get("irreversible"):
            if not torch.equal(self.x, self.y):
                raise SystemExit("lossless round trip FAILED (%s)" % self.name)
        else:
            d = (self.y - self.x).double()
            mse = float((d * d).mean())
            psnr = 10 * np.log10(((1 << self.cfg["bits"]) - 1) ** 2 / mse)
            if psnr < 30.0:
                raise SystemExit("9/7 round trip PSNR %.2f dB too low (%s)" % (psnr, self.name))
            return psnr
        return None

    def close(self):
        self.eng.close()


class InFlightRunner:
    """Runners driven concurrently, each from its own host thread with its own engine (HIP stream
    and buffers): one step = every runner's step once.  With the headline pair (one C2 and one
    C3 image) the host phases of one image (PCRD, packet headers) overlap the other's kernels."""

    def __init__(self, runners):
        from concurrent.futures import ThreadPoolExecutor
        self.rs = runners
        self.pixels = sum(r.pixels for r in runners)
        self.n = sum(r.n for r in runners)
        self.pool = ThreadPoolExecutor(len(runners))

    def step(self):
        for f in [self.pool.submit(r.step) for r in self.rs]:
            f.result()
        self.n = sum(r.n for r in self.rs)
        return {}

    def check(self):
        for r in self.rs:
            r.check()
        self.n = sum(r.n for r in self.rs)

    def close(self):
        self.pool.shutdown()
        for r in self.rs:
            r.close()


class BatchRunner:
    """`nimg` images in flight on one GPU: each has its own engine (own HIP stream and
    buffers) and is driven from its own host thread, so one image's host T2 and
    chain-bound T1 kernels overlap with the other's (ctypes releases the GIL).  One
    step = every image encoded and decoded once.  Image i uses seed cfg.seed + rank
    + 1000 * i (same generator, same statistics)."""

    def __init__(self, name, nimg, rank, device):
        from concurrent.futures import ThreadPoolExecutor
        self.rs = [Runner(name, 0, rank + 1000 * i, device) for i in range(nimg)]
        self.size, self.cfg, self.name = self.rs[0].size, self.rs[0].cfg, name
        self.n = self.rs[0].n
        self.pool = ThreadPoolExecutor(nimg)

    def step(self):
        res = [f.result() for f in [self.pool.submit(r.step) for r in self.rs]]
        self.n = self.rs[0].n
        return res[0]

    def check(self):
        for r in self.rs:
            r.check()
        self.n = self.rs[0].n

    def close(self):
        self.pool.shutdown()
        for r in self.rs:
            r.eng.close()


class ShardRunner:
    """C4 on N ranks through grok_amd.shard.TileRowShard: rank 0 holds the
    16-bit image in HBM.  One step = rank 0 scatters the tile rows (RCCL) -> every rank
    encodes its tiles -> rank 0 gathers the tile parts and assembles the codestream (main
    header, TLM filled) -> rank 0 locates each rank's tile parts through TLM and scatters them
    -> every rank decodes its rows -> rank 0 gathers the decoded rows.  Samples travel as
    16-bit (u16 held in int16 tensors, the engine's 2-byte sample type).
    coder: per-rank coder (grok_amd.shard.EngineCoder by default; tests pass the CPU oracle)."""

    def __init__(self, name, size, rank, world, device, dist, coder=None):
        import torch
        from grok_amd import shard
        from grok_amd.synth import synth_slab
        cfg = CONFIGS[name]
        size = size or cfg["size"]
        self.name, self.cfg, self.size, self.rank, self.world, self.dist = name, cfg, size, rank, world, dist
        self.device = device
        C, bits = cfg["comps"], cfg["bits"]
        shape = (C, size, size)
        if coder is None:
            import grok_amd as G
            self.eng = G.Engine(device.index or 0)
            coder = shard.EngineCoder(self.eng, shape, bits, G.default_params(**cfg["params"]))
        else:
            self.eng = None
        self.coder = coder
        self.sh = shard.TileRowShard(dist, rank, world, coder, shape, cfg["params"]["tiles"], device)
        dt = torch.int16 if bits > 8 else torch.uint8
        self.full = self.y_full = None
        if rank == 0:
            self.full = torch.empty(shape, dtype=dt, device=device)
            th = cfg["params"]["tiles"][1]
            for y0 in range(0, size, th):   # rank 0's image, generated by tile rows
                y1 = min(size, y0 + th)
                sl = synth_slab(y0, y1, size, size, C, bits, cfg["seed"])
                sl = sl.view(np.int16) if bits > 8 else sl.astype(np.uint8)
                self.full[:, y0:y1] = torch.from_numpy(np.ascontiguousarray(sl)).to(device)
            self.y_full = torch.empty_like(self.full)
        self.y0, self.y1 = self.sh.y0, self.sh.y1
        self.x = torch.empty((C, self.y1 - self.y0, size), dtype=dt, device=device)
        self.y = torch.empty_like(self.x)
        self.parts = torch.empty(max(self.x.numel() * 4, 1) + (1 << 22), dtype=torch.uint8, device=device)
        self.n = 0
        self.cs = None
        self.pixels = size * size

    def _timings(self):
        return self.eng.timings() if self.eng is not None else None

    def step(self):
        self.sh.scatter_input(self.full, self.x)
        self.cs, self.n = self.sh.encode(self.x, self.parts)
        te = self._timings()
        self.sh.decode(self.cs, self.n, self.y, self.y_full)
        td = self._timings()
        return (te, td) if te is not None else {}

    def check(self):
        import torch
        self.step()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        if not torch.equal(self.x, self.y):
            raise SystemExit("sharded lossless round trip FAILED (%s, rank %d rows)" % (self.name, self.rank))
        if self.rank == 0 and not torch.equal(self.full, self.y_full):
            raise SystemExit("sharded lossless round trip FAILED (%s, gathered image)" % self.name)
        return None

    def close(self):
        if self.eng is not None:
            self.eng.close()


class C5Runner:
    """C5: decode-only random windows of a tiled RGB8 .jp2 held in rank 0's HBM (built on its
    GPU from tile-row slabs, grok_amd.bigimage).  One step decodes the four SURVEY windows
    through grok_amd.shard.WindowShard: with N ranks each window's tile rows are split into
    bands, rank 0 scatters to each rank the tile parts its band needs (located through TLM;
    no rank holds the whole file), every rank decodes its band into u8 planes and rank 0
    gathers the bands.  size / windows / coder / file: overrides for the CPU tests."""

    def __init__(self, rank, world, device, dist, size=None, windows=None, coder=None, file=None, n=0):
        import torch
        from grok_amd import shard
        cfg = CONFIGS["C5"]
        self.cfg, self.rank, self.world, self.device, self.dist = cfg, rank, world, device, dist
        S = size or cfg["size"]
        self.windows = windows or C5_WINDOWS
        self.crops = None
        self.eng = None
        t0 = time.perf_counter()
        if coder is None:
            import grok_amd as G
            from grok_amd import bigimage
            self.eng = G.Engine(device.index or 0)
            p = G.default_params(**cfg["params"])
            coder = shard.EngineCoder(self.eng, (cfg["comps"], S, S), cfg["bits"], p)
            if rank == 0:
                it = bigimage.slabs(S, S, cfg["comps"], cfg["bits"], cfg["seed"], 1024, threads=16)
                crops = {k: w for k, w in enumerate(self.windows)}
                file, n, self.crops = bigimage.encode_tiled(self.eng, (cfg["comps"], S, S), cfg["bits"], p, it,
                                                            device, crops=crops)
        self.file, self.n = file, n
        self.build_s = time.perf_counter() - t0
        self.ws = shard.WindowShard(dist, rank, world, coder, device, file if rank == 0 else None, n)
        nb = torch.zeros(1, dtype=torch.int64, device=device)
        if rank == 0:
            nb[0] = n
        if world > 1:
            dist.broadcast(nb, 0)
        self.n = int(nb.item())
        self.pixels = sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in self.windows)
        self.outs, self.bufs = [], []
        for w in self.windows:
            x0, y0, x1, y1 = w
            hmax = max(b - a for a, b in self.ws.bands(w))
            self.outs.append(torch.empty((3, y1 - y0, x1 - x0), dtype=torch.uint8, device=device) if rank == 0 else None)
            self.bufs.append(torch.empty((3, max(hmax, 1), x1 - x0), dtype=torch.uint8, device=device)
                             if rank != 0 else None)

    def step(self):
        acc = {}
        for k, w in enumerate(self.windows):
            self.ws.decode(w, self.outs[k], self.bufs[k])
            if self.eng is not None:
                t = self.eng.timings()
                for f in ("t1_ms", "dwt_ms", "mct_ms", "t2_ms", "total_ms"):
                    acc["dec_" + f] = acc.get("dec_" + f, 0.0) + float(getattr(t, f))
        return acc

    def check(self):
        import torch
        self.step()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        if self.rank == 0 and self.crops is not None:
            for k, o in enumerate(self.outs):
                if not np.array_equal(o.cpu().numpy(), self.crops[k]):
                    raise SystemExit("C5 window %s decode differs from the source" % (self.windows[k],))

    def close(self):
        if self.eng is not None:
            self.eng.close()


class PairRunner:
    """The headline step: one C2 image (5/3 lossless) and one C3 image (9/7 lossy) encoded and
    decoded, one after the other on one engine each.  Stage timings are reported per config
    (keys prefixed "C2_" / "C3_")."""

    def __init__(self, r2, r3):
        self.rs = (("C2", r2), ("C3", r3))
        self.pixels = r2.pixels + r3.pixels
        self.n = r2.n
        self.name = "C2+C3"

    def step(self):
        acc = {}
        for name, r in self.rs:
            te, td = r.step()
            for pre, t in (("enc", te), ("dec", td)):
                for f, _ in t._fields_:
                    acc["%s_%s_%s" % (name, pre, f)] = float(getattr(t, f))
        self.n = self.rs[0][1].n + self.rs[1][1].n
        return acc

    def check(self):
        self.rs[0][1].check()
        psnr = self.rs[1][1].check()
        self.n = self.rs[0][1].n + self.rs[1][1].n
        return psnr

    def close(self):
        for _, r in self.rs:
            r.close()


def stage_rooflines(name, m, cfg, size=0):
    """HBM roofline candidates of one config's timed stages (per step averages of the engine's
    HIP-event timings m): T1 decode (compressed bytes + 4 B/sample), T1 encode (4 B/sample +
    compressed bytes), DWT (the engine's per-level algorithmic bytes)."""
    cp = cfg["params"]
    samples = cfg["comps"] * (size or cfg["size"]) ** 2
    if cp.get("cblk_sty"):   # HTJ2K: one cleanup-pass coder kernel each way
        dec_k, enc_k = ("T1 decode (k_ht_dec)", ["k_ht_dec"]), ("T1 encode (k_ht_enc)", ["k_ht_enc"])
    else:
        dec_k = ("T1 decode (k_t1_dec2 + k_t1_recon)", ["void k_t1_dec2<0, 4>", "k_t1_recon"])
        cm = "void k_t1_cm<true>" if cp.get("irreversible") else "void k_t1_cm<false>"
        enc_k = ("T1 encode (k_t1_cm + k_t1_mq)", [cm, "k_t1_mq"])
    dw = "97" if cp.get("irreversible") else "53"
    return [
        {"config": name, "stage": "%s %s" % (name, dec_k[0]), "avg_ms": m["dec_t1_ms"],
         "bytes_per_launch": m["dec_t1_bytes"] + 4.0 * samples, "kernels": dec_k[1]},
        {"config": name, "stage": "%s %s" % (name, enc_k[0]), "avg_ms": m["enc_t1_ms"],
         "bytes_per_launch": 4.0 * samples + m["enc_t1_bytes"], "kernels": enc_k[1]},
        {"config": name, "stage": "%s DWT %s fwd+inv (all levels)" % (name, "9/7" if dw == "97" else "5/3"),
         "avg_ms": m["enc_dwt_ms"] + m["dec_dwt_ms"], "bytes_per_launch": m["enc_dwt_bytes"] + m["dec_dwt_bytes"],
         "kernels": ["k_dwt%s_fwd_level" % dw, "k_dwt%s_inv_level" % dw]},
    ]


def timed(r, steps, warmup, world, dist, device, sync=True):
    import torch
    for _ in range(warmup):
        r.step()
    if world > 1:
        dist.barrier()
    if sync:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = {}
    for _ in range(steps):
        out = r.step()
        if isinstance(out, dict):
            for k, v in out.items():
                acc[k] = acc.get(k, 0.0) + v
            continue
        te, td = out
        for pre, t in (("enc", te), ("dec", td)):
            for f, _ in t._fields_:
                acc[pre + "_" + f] = acc.get(pre + "_" + f, 0.0) + float(getattr(t, f))
    if sync:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, {k: v / steps for k, v in acc.items()}


class DryRunner:
    """--dry-run: a fixed host computation per step, no engine (launcher/timing plumbing)."""
    pixels = 1 << 20

    def step(self):
        a = np.arange(1 << 16, dtype=np.float64)
        return {"work": float(np.sqrt(a).sum()) * 0.0}


def dry_main(args, world, rank, dist):
    import torch
    el, _ = timed(DryRunner(), args.steps, args.warmup, world, dist, torch.device("cpu"), sync=False)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "value": round(DryRunner.pixels / 1e6 * world * args.steps / el, 3),
                          "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el * 1000.0 / args.steps, 3), "higher_is_better": True,
                          "scaling": "weak"}), flush=True)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch(args))   # this process has not touched the GPU
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo" if args.dry_run else "nccl")
    if args.dry_run:
        dry_main(args, world, rank, dist)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    if args.config == "C2+C3":
        r2 = Runner("C2", args.size, rank, device)
        r3 = Runner("C3", args.size, rank, device)
        r = PairRunner(r2, r3)
    elif args.config != "C4" or world == 1:
        r = Runner(args.config, args.size, rank, device)
    else:
        r = ShardRunner("C4", args.size, rank, world, device, dist)
    psnr = r.check()
    el, m = timed(r, args.steps, args.warmup, world, dist, device)
    ms = el * 1000.0 / args.steps
    per_rank = world if not isinstance(r, ShardRunner) else 1   # replicas: every rank codes its own images
    value = r.pixels / 1e6 * per_rank * args.steps / el
    r_pixels = int(r.pixels)
    per_config = None
    if isinstance(r, PairRunner):
        # each config of the pair timed alone as well (same engines, same images)
        per_config = {}
        for name, rr in (("C2", r2), ("C3", r3)):
            elx, _ = timed(rr, args.steps, 1, world, dist, device)
            per_config[name] = {"config": "%s: %s" % (name, CONFIGS[name]["desc"]),
                                "value": round(rr.pixels / 1e6 * world * args.steps / elx, 3), "unit": "Mpixels/s",
                                "ms_per_step": round(elx * 1000.0 / args.steps, 3),
                                "codestream_bytes": int(rr.n),
                                "stages_ms": {k[3:]: round(v, 3) for k, v in m.items()
                                              if k.startswith(name + "_") and k.endswith("_ms") and v > 0}}
        per_config["C3"]["psnr_db"] = round(psnr, 3)
        per_config["C3"]["psnr_note"] = "decode vs source, 12-bit peak (tolerance check: >= 30 dB in bench)"
    codestream_bytes = int(r.n)
    # the T1 decoder's chain length: one more (untimed) decode with the step counters on
    dec_steps = None
    rs = r2 if isinstance(r, PairRunner) else r
    if isinstance(rs, Runner) and not rs.cfg["params"].get("cblk_sty"):
        os.environ["GK_T1_STATS"] = "1"
        try:
            rs.eng.decode(rs.out, length=rs.n, out=rs.y)
            t = rs.eng.timings()
            dec_steps = (int(t.t1_steps_max), int(t.t1_steps_total), int(t.t1_symbols), int(t.t1_solo_blocks),
                         int(t.t1_solo_decisions), int(t.t1_solo_decisions_max))
        finally:
            del os.environ["GK_T1_STATS"]
    r.close()
    del r, rs
    if args.config == "C2+C3":
        del r2, r3
    torch.cuda.empty_cache()

    aux = None
    if not args.no_aux and args.config == "C2+C3":
        aux = {}
        # the headline pair with both images in flight (one host thread and engine each)
        rp = InFlightRunner([Runner("C2", args.size, rank, device), Runner("C3", args.size, rank, device)])
        rp.check()
        elp, _ = timed(rp, 3, 1, world, dist, device)
        aux["C2+C3_inflight"] = {"config": "the headline step (one C2 and one C3 image encoded + decoded) with both images "
                                           "in flight on the GPU (2 engines / HIP streams, one host thread each: the "
                                           "host PCRD and packet phases of one image overlap the other's kernels)",
                                 "value": round(rp.pixels / 1e6 * world * 3 / elp, 3), "unit": "Mpixels/s",
                                 "ms_per_step": round(elp * 1000.0 / 3, 3), "parallelism": "replicas x%d" % world}
        rp.close()
        del rp
        torch.cuda.empty_cache()
        # C2 with two images in flight per GPU (throughput of overlapped independent jobs)
        rb = BatchRunner("C2", 2, rank, device)
        rb.check()
        elb, mb = timed(rb, 3, 1, world, dist, device)
        Sb = rb.size
        aux["C2_batch2"] = {"config": "C2 with 2 images in flight per GPU (2 engines / HIP streams, one host thread "
                                      "each); one step = 2 images encoded + decoded",
                            "value": round(2 * Sb * Sb / 1e6 * world * 3 / elb, 3), "unit": "Mpixels/s",
                            "ms_per_step": round(elb * 1000.0 / 3, 3), "images_per_step": 2,
                            "parallelism": "replicas x%d" % world}
        rb.close()
        del rb
        torch.cuda.empty_cache()
        # C3 with two images in flight: one image's host PCRD + T2 runs while the other's
        # DWT / T1 kernels occupy the GPU
        rb3 = BatchRunner("C3", 2, rank, device)
        rb3.check()
        elb3, _ = timed(rb3, 2, 1, world, dist, device)
        Sb3 = rb3.size
        aux["C3_batch2"] = {"config": "C3 with 2 images in flight per GPU (2 engines / HIP streams, one host thread "
                                      "each: host PCRD of one image overlaps the other's GPU stages); one step = 2 "
                                      "images encoded + decoded",
                            "value": round(2 * Sb3 * Sb3 / 1e6 * world * 2 / elb3, 3), "unit": "Mpixels/s",
                            "ms_per_step": round(elb3 * 1000.0 / 2, 3), "images_per_step": 2,
                            "parallelism": "replicas x%d" % world}
        rb3.close()
        del rb3
        torch.cuda.empty_cache()
        r4 = ShardRunner("C4", 0, rank, world, device, dist) if world > 1 else Runner("C4", 0, rank, device)
        r4.check()
        el4, m4 = timed(r4, 3, 1, world, dist, device)
        S4 = r4.size
        aux["C4"] = {"config": "C4: " + CONFIGS["C4"]["desc"], "value": round(S4 * S4 / 1e6 * 3 / el4, 3),
                     "unit": "Mpixels/s", "ms_per_step": round(el4 * 1000.0 / 3, 3),
                     "codestream_bytes": int(r4.n),
                     "parallelism": ("tile rows sharded over %d ranks (grok_amd.shard.TileRowShard): RCCL scatter of "
                                     "the 16-bit rows from rank 0, gather of the tile parts, scatter of the "
                                     "TLM-located parts, gather of the decoded rows" % world)
                     if world > 1 else "1 GPU, all 256 tiles batched",
                     "scaling": "strong",
                     "stages_ms": {k: round(v, 3) for k, v in m4.items() if k.endswith("_ms") and v > 0},
                     "t1_blocks": int(m4.get("enc_t1_blocks", 0)),
                     "issue_roofline": ht_issue_roofline(m4)}
        r4.close()
        del r4
        torch.cuda.empty_cache()
        if not args.no_c5:
            r5 = C5Runner(rank, world, device, dist)
            r5.check()
            el5, m5 = timed(r5, 3, 1, world, dist, device)
            aux["C5"] = {"config": "C5: " + CONFIGS["C5"]["desc"], "value": round(r5.pixels / 1e6 * 3 / el5, 3),
                         "unit": "Mpixels/s (window output samples)", "ms_per_step": round(el5 * 1000.0 / 3, 3),
                         "window_mpix_per_step": round(r5.pixels / 1e6, 3), "file_bytes": int(r5.n),
                         "parallelism": ("each window's tile rows split over %d ranks (grok_amd.shard.WindowShard): "
                                         "RCCL scatter of the TLM-located tile parts each band needs, gather of the "
                                         "decoded rows" % world)
                         if world > 1 else "1 GPU",
                         "scaling": "strong", "build_s": round(r5.build_s, 1),
                         "stages_ms_rank0": {k: round(v, 3) for k, v in m5.items() if v > 0},
                         "vs_grok_8vcpu_w16k": "Grok -H 8 decodes the 16384^2 window at %.1f Mpix/s (BASELINE.md)"
                                               % GROK_CPU["C5_w16k_8t"]}
            r5.close()
            del r5
            torch.cuda.empty_cache()

    if rank == 0:
        # dominant kernel: the T1 / DWT stage with the largest average duration per step, measured
        # with HIP events on the engine stream, over the configs of the step
        names = ["C2", "C3"] if args.config == "C2+C3" else [args.config]
        cands = []
        for name in names:
            mm = {k[3:]: v for k, v in m.items() if k.startswith(name + "_")} if len(names) > 1 else m
            cands += stage_rooflines(name, mm, CONFIGS[name], args.size)
        dom = max(cands, key=lambda c: c["avg_ms"])
        achieved = dom["bytes_per_launch"] / 1e9 / (dom["avg_ms"] / 1e3)
        traffic, traffic_src = pmc_traffic(dom["kernels"], dom["config"])
        dwt = {}
        for name in names:
            mm = {k[3:]: v for k, v in m.items() if k.startswith(name + "_")} if len(names) > 1 else m
            smp = CONFIGS[name]["comps"] * (args.size or CONFIGS[name]["size"]) ** 2
            gbs = (mm["enc_dwt_bytes"] + mm["dec_dwt_bytes"]) / 1e9 / ((mm["enc_dwt_ms"] + mm["dec_dwt_ms"]) / 1e3)
            dwt[name] = {"stage": "DC shift + MCT + DWT (%s), encode and decode (level 1 fused with the sample stage, "
                                  "all levels)" % ("9/7 + ICT" if CONFIGS[name]["params"].get("irreversible") else
                                                   "5/3 + RCT"),
                         "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "ms": round(mm["enc_dwt_ms"] + mm["dec_dwt_ms"], 3),
                         "bytes_per_sample": round((mm["enc_dwt_bytes"] + mm["dec_dwt_bytes"]) / (2.0 * smp), 3)}
        grok_ref = GROK_CPU["C2p_8t"] if args.config == "C2" else (
            2.0 / (1.0 / GROK_CPU["C2p_8t"] + 1.0 / GROK_CPU["C3p_8t"]) if args.config == "C2+C3" else None)
        res = {
            "metric": METRIC,
            "value": round(value, 3), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak" if args.config != "C4" else "strong",
            # the reference publishes no number for this metric
            "vs_baseline": None,
            "dtype": "int32 (5/3) + f32 (9/7)" if args.config == "C2+C3" else
                     ("f32" if CONFIGS[args.config]["params"].get("irreversible") else "int32"),
            "data": "synthetic (seeded survey generator grok_amd/synth.py, seeds %s + rank)" % (
                "10 (C2) / 11 (C3)" if args.config == "C2+C3" else str(CONFIGS[args.config]["seed"])),
            "config": {"workload": ("C2+C3: one 8192x8192 8-bit RGB 5/3 lossless image (C2: %s) and one 8192x8192 "
                                    "12-bit RGB 9/7 lossy image (C3: %s) encoded + decoded per step, images and "
                                    "codestreams resident in HBM" % (CONFIGS["C2"]["desc"], CONFIGS["C3"]["desc"]))
                                   if args.config == "C2+C3" else
                                   "%s: %s; encode+decode, image and codestream resident in HBM" % (
                                       args.config, CONFIGS[args.config]["desc"]),
                       "parallelism": "replicas x%d (one image per GPU)" % world if args.config != "C4" or world == 1
                       else "C4 tile rows sharded over %d ranks" % world,
                       "pixels_per_step_per_rank": r_pixels,
                       "codestream_bytes": codestream_bytes},
            "roofline": {"bound": "hbm", "kernel": dom["stage"], "config": dom["config"], "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None if traffic is None else round(traffic), "traffic_source": traffic_src,
                         "bytes_per_launch": round(dom["bytes_per_launch"]), "avg_ms": round(dom["avg_ms"], 3),
                         "note": "T1 is a serial MQ chain per code-block; bytes = compressed bytes + 4 B/sample"},
            "dwt_roofline": dwt[names[0]] if len(names) == 1 else dwt,
            "stages_ms": {k: round(v, 3) for k, v in m.items() if k.endswith("_ms") and v > 0},
        }
        if per_config:
            res["per_config"] = per_config
        if grok_ref:
            res["vs_grok_cpu_container"] = {"ratio": round(value / grok_ref, 1), "grok_mpix_s": round(grok_ref, 3),
                                            "ref": "Grok 9.2.0 CPU enc+dec on the survey container (8 vCPU), BASELINE.md "
                                                   "section 2 (C2' / C3' -c [256,256] variants: Grok cannot decode its "
                                                   "single-precinct 8K streams); not a published number"}
        t1m = {k[3:]: v for k, v in m.items() if k.startswith("C2_")} if args.config == "C2+C3" else m
        if "enc_t1_blocks" in t1m:
            res["t1"] = {"blocks": int(t1m["enc_t1_blocks"]),
                         "enc_blocks_per_s": round(t1m["enc_t1_blocks"] / (t1m["enc_t1_ms"] / 1e3)),
                         "dec_blocks_per_s": round(t1m["dec_t1_blocks"] / (t1m["dec_t1_ms"] / 1e3))}
        cp = CONFIGS[args.config]["params"] if args.config in CONFIGS else {}
        if cp.get("cblk_sty"):   # HTJ2K coders: issue roofline from the committed SQ counter summary
            res["issue_roofline"] = ht_issue_roofline(m, args.config)
        if dec_steps and dec_steps[0]:
            # issue roofline of the chain-bound decoder: one wave per SIMD issues one instruction
            # per 4 cycles, so the kernel takes at least (steps of its longest wave) x
            # (instructions per step) x 4 cycles; instructions per step read from the loaded
            # library's gfx950 code object (tools/isa_step_count.py, ROCm llvm-objdump)
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import isa_step_count
            import grok_amd as G
            _, dec_ips, dec_by = isa_step_count.count_so(G.LIB_PATH)
            dec_ips = int(dec_ips)
            floor_ms = dec_steps[0] * dec_ips * 4 / (CLOCK_GHZ * 1e6)
            dec2_ms = t1m.get("dec_t1_coder_ms", t1m["dec_t1_ms"])
            res["issue_roofline"] = {
                "kernel": "k_t1_dec2 (T1 decode chain, C2)", "bound": "instruction issue of the longest wave",
                "max_steps_per_wave": dec_steps[0], "instructions_per_step": dec_ips,
                "instructions_per_step_source": "llvm-objdump of %s (k_t1_dec2<0, 4> step bodies: %s)" % (
                    os.path.relpath(G.LIB_PATH, ROOT), ", ".join("%s %d" % kv for kv in dec_by.items())),
                "clock_ghz": CLOCK_GHZ, "floor_ms": round(floor_ms, 3), "measured_ms": round(dec2_ms, 3),
                "frac": round(floor_ms / dec2_ms, 3), "steps_total": dec_steps[1], "symbols": dec_steps[2],
                "lane_efficiency": round(dec_steps[2] / (64.0 * dec_steps[1]), 3) if dec_steps[1] else None,
                "solo": {"blocks": dec_steps[3], "decisions": dec_steps[4], "max_decisions_per_wave": dec_steps[5],
                         "note": "heaviest blocks decoded one per wave on the SIMDs the lane-parallel waves leave "
                                 "(gk_t1dec.hip solo_block); the steps above are the lane-parallel waves'"}}
        if aux:
            res["aux"] = aux
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(host_threads(args))
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
