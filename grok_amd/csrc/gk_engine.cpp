// gk_engine.cpp — host orchestration of the MI355X JPEG 2000 tile pipeline.
//
// Encode (TileProcessor::doCompress, TileProcessor.cpp:202-260):
//   H2D (optional) -> DC shift + MCT -> 5/3 DWT levels -> T1 encode (one wave
//   per code-block) -> D2H of per-block (numbps, passes, length) -> host T2
//   packet headers (T2Compress.cpp:113-240) -> device gather of headers and
//   code-block bytes into the codestream (-> D2H if the caller wants host bytes).
// Decode (TileProcessor::decompressT2T1, TileProcessor.cpp:384-408):
//   host T2 parse of packet headers (device-resident codestreams are read
//   through a paged D2H reader) -> T1 decode -> inverse DWT -> inverse MCT.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <tuple>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>
#include <queue>
#include <map>
#include <climits>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/grok_amd.h"
#include "gk_common.h"
#include "gk_bitio.h"
#include "gk_launch.h"

namespace {

static inline uint32_t ceildivpow2(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + (1ull << b) - 1) >> b); }
static inline uint32_t ceildiv(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b - 1) / b); }
static inline int floorlog2(uint32_t a) { return a > 1 ? 31 - __builtin_clz(a) : 0; }
static inline uint32_t align_up(uint32_t v, uint32_t a) { return (v + a - 1) / a * a; }

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { throw GkError(std::string(#x) + ": " + hipGetErrorString(e_)); } } while (0)

struct GkError {
    std::string msg;
    explicit GkError(std::string m) : msg(std::move(m)) {}
};
// Kernel launches report a bad configuration only through hipGetLastError: each stage of an
// encode / decode ends with this check, so such an error fails the call that made it (with the
// engine source line of the stage) instead of surfacing in a later, unrelated HIP call.
static void launch_check(int line) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        throw GkError("kernel launch before gk_engine.cpp:" + std::to_string(line) + ": " + hipGetErrorString(e));
}

// Engines alive per device in this process.  Solo T1 waves use the SIMDs a decode leaves idle;
// when several engines share a device their kernels overlap and no SIMD is idle, so solo waves
// only stretch the tail (C2 with two images in flight: 2,555 -> 2,394 Mpix/s with them).
static std::mutex g_dev_mu;
static std::map<int, int> g_dev_engines;
// Engines of a device inside an encode / decode call right now (every call returns after its
// stream has drained): a second one means another image's kernels share the chip with this one
static std::map<int, int> g_dev_busy;
static int engines_busy(int dev) {
    std::lock_guard<std::mutex> g(g_dev_mu);
    auto it = g_dev_busy.find(dev);
    return it == g_dev_busy.end() ? 0 : it->second;
}
struct DevBusy {
    int dev;
    explicit DevBusy(int d) : dev(d) { std::lock_guard<std::mutex> g(g_dev_mu); ++g_dev_busy[dev]; }
    ~DevBusy() { std::lock_guard<std::mutex> g(g_dev_mu); if (--g_dev_busy[dev] <= 0) g_dev_busy.erase(dev); }
};


// Persistent host worker pool for the T2 stages (tiles, precinct chains, blocks).
// run(n, f) calls f(0..n-1) across the workers and the caller, and returns when all
// calls finished; the first GkError thrown by any call is rethrown.  Host phases are short (a
// rate-control bisection step is ~100 us on 16 threads), so a dispatch must cost little:
//  * items are claimed from one word holding (generation, item count, next item) and run()
//    waits for the items to finish, not for every worker to have woken; a worker reads the job
//    only after a successful claim, when no later job can have replaced it (a worker that
//    wakes after its generation's items are all claimed never touches that job);
//  * workers sleep on the generation word itself (futex), so a wake-up takes no mutex: with a
//    mutex and a condition variable, 15 woken workers queued on the mutex the next dispatch
//    needed.  Empty dispatch on the GPU box (tools/pcrd_bench.cpp): ~30 us with
//    notify_all and a wait for every worker, ~5 us now.
class HostPool {
    std::vector<std::thread> th_;
    // (the claim word and the finished count on lines of their own: every item touches both,
    // from every thread)
    std::atomic<const std::function<void(size_t)>*> job_{nullptr};   // written before the claim word
    std::atomic<uint32_t> gen_{0};           // futex word: a new job
    std::atomic<uint32_t> fin_{0};           // futex word: the caller sleeps until done_ == items
    alignas(128) std::atomic<uint64_t> claim_{0};   // generation (16 bits) | items (24) | next item (24)
    alignas(128) std::atomic<size_t> done_{0};      // items of the current generation finished
    char pad_[128 - sizeof(std::atomic<size_t>)];
    std::atomic<bool> stop_{false}, has_err_{false};
    std::mutex err_m_;
    std::string err_;
    std::mutex run_m_;
    static constexpr uint64_t kMaxItems = (1u << 24) - 1;
    static void fwait(std::atomic<uint32_t>& w, uint32_t v) {
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
    }
    static void fwake(std::atomic<uint32_t>& w) {
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
    }
    // an item of generation g: its index and the generation's item count, or false
    bool claim(uint32_t g, size_t& i, size_t& n) {
        uint64_t c = claim_.load(std::memory_order_acquire);
        for (;;) {
            if ((uint32_t)(c >> 48) != (g & 0xffffu)) return false;
            n = (size_t)((c >> 24) & kMaxItems);
            i = (size_t)(c & kMaxItems);
            if (i >= n) return false;
            if (claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel)) return true;
        }
    }
    void fail(const std::string& e) {
        std::lock_guard<std::mutex> lk(err_m_);
        if (err_.empty()) err_ = e;
        has_err_ = true;
    }
    // A thread counts the items it ran and adds them to done_ once it finds nothing left to
    // claim (the job stays alive until done_ reaches the item count, so the count is added
    // before this thread lets go of it).
    void work(uint32_t g) {
        size_t ran = 0, n = 0;
        for (size_t i; claim(g, i, n);) {
            // (the claim synchronises with the caller's publication, and this item keeps the job alive)
            const std::function<void(size_t)>& f = *job_.load(std::memory_order_relaxed);
            try { f(i); } catch (const GkError& e) {
                fail(e.msg);
            } catch (const std::exception& e) {   // e.g. std::bad_alloc: recorded, never escapes a worker
                fail(std::string("host worker: ") + e.what());
            } catch (...) {
                fail("host worker: unknown exception");
            }
            ++ran;
        }
        if (ran && done_.fetch_add(ran, std::memory_order_acq_rel) + ran == n) {   // the last items
            fin_.fetch_add(1, std::memory_order_release);
            fwake(fin_);
        }
    }
    void worker() {
        uint32_t seen = 0;
        for (;;) {
            uint32_t g;
            while ((g = gen_.load(std::memory_order_acquire)) == seen && !stop_.load(std::memory_order_acquire)) fwait(gen_, seen);
            if (stop_.load(std::memory_order_acquire)) return;
            seen = g;
            work(g);
        }
    }

public:
    explicit HostPool(unsigned k) { for (unsigned i = 0; i < k; ++i) th_.emplace_back([this] { worker(); }); }
    ~HostPool() {
        stop_.store(true, std::memory_order_release);
        gen_.fetch_add(1, std::memory_order_release);
        fwake(gen_);
        for (auto& t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    // One job at a time: a caller that finds the pool busy (another engine context on
    // another host thread) runs its items inline.
    void run(size_t n, const std::function<void(size_t)>& f) {
        if (n == 0) return;
        std::unique_lock<std::mutex> own(run_m_, std::try_to_lock);
        if (n == 1 || th_.empty() || !own.owns_lock() || n > kMaxItems) { for (size_t i = 0; i < n; ++i) f(i); return; }
        { std::lock_guard<std::mutex> lk(err_m_); err_.clear(); }
        has_err_ = false;
        job_.store(&f, std::memory_order_relaxed);
        done_.store(0, std::memory_order_relaxed);
        const uint32_t g = gen_.load(std::memory_order_relaxed) + 1;
        claim_.store(((uint64_t)(g & 0xffffu) << 48) | ((uint64_t)n << 24), std::memory_order_release);
        gen_.store(g, std::memory_order_release);
        fwake(gen_);
        work(g);
        for (uint32_t v; done_.load(std::memory_order_acquire) != n;) {   // items still running on workers
            v = fin_.load(std::memory_order_acquire);
            if (done_.load(std::memory_order_acquire) == n) break;
            fwait(fin_, v);
        }
        if (has_err_.load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(err_m_);
            throw GkError(err_);
        }
    }
};
static HostPool& host_pool() {   // one pool per process, sized to the CPU share (at most 16 threads)
    static HostPool pool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
    return pool;
}

// ---------------------------------------------------------------------------
// Tile geometry (ISO 15444-1 Annex B; Grok Resolution.h:37-72,
// Precinct.h:59-68).  Single tile anchored at the image origin.
// ---------------------------------------------------------------------------
// One progression order change (POC marker, A.6.6): layers [0, lye), resolutions [rs, re),
// components [cs, ce) in progression prog.
struct Poc { uint32_t rs = 0, cs = 0, lye = 0, re = 0, ce = 0, prog = 0; };

struct Params {
    uint32_t numres = 6, cbw = 6, cbh = 6, irrev = 0, mct = 1, numgbits = 2, nlayers = 1, write_com = 1;
    uint32_t prcw[GK_MAXRLVLS], prch[GK_MAXRLVLS];
    bool custom_prc = false;
    double rates[GK_MAX_LAYERS] = {0};   // compression ratio per layer (0 = remaining passes)
    uint32_t cblk_sty = 0;               // Part-1 mode switches or GRK_CBLKSTY_HT (0x40, grok.h:98-104)
    uint32_t prog = 0;                   // progression order: GRK_LRCP 0, RLCP 1, RPCL 2, PCRL 3, CPRL 4
    char tp_div = 0;                     // tile-part divider 'L' / 'R' / 'C' (grk_compress -u), 0 = one part per tile
    std::vector<Poc> pocs;               // progression order changes (every tile; empty = prog)
    std::vector<uint8_t> roishift;       // per component ROI shift (RGN, maxshift; empty = none)
    // the caller's COM markers (Rcom 0 binary / 1 text, bytes) written instead of the default one
    std::vector<std::pair<uint32_t, std::string>> comments;
    uint32_t roi(uint32_t c) const { return c < roishift.size() ? roishift[c] : 0u; }
    bool ht() const { return (cblk_sty & 0x40) != 0; }
    // a code-block side above 64 (128 x 32 ... 1024 x 4): Part-1 blocks take the lane-per-block
    // coders of gk_t1ms.hip, whose state is sized by the block (T1::alloc, T1.cpp:337-398), HT
    // blocks the wide-line HT kernels; the headline kernels keep their 64-column layouts
    bool wide() const { return cbw > 6 || cbh > 6; }
    bool t1_generic() const { return (cblk_sty & 0x3f) != 0 || (wide() && !ht()); }
    uint32_t tw = 0, th = 0;             // nominal tile size (grk_cparameters::t_width/t_height; 0 = image)
    bool tlm = false, plt = false;       // grk_cparameters::writeTLM / writePLT
    bool jp2 = false;                    // grk_cparameters::cod_format == GRK_CODEC_JP2 (file format boxes)
    uint32_t sop_eph = 0;                // Scod bits: 2 = SOP before every packet (-S), 4 = EPH after its header (-E)
    bool quality = false;                // fixed-quality layers (grk_cparameters::allocationByQuality, -q)
    double dist[GK_MAX_LAYERS] = {0};    // PSNR target per layer (0 = the remaining passes)
    bool layer_rc(uint32_t l) const {    // TileProcessor::layerNeedsRateControl (TileProcessor.cpp:952-957)
        return quality ? dist[l] > 0.0 : rates[l] > 0.0;
    }
    bool rate_control() const {          // TileProcessor::needsRateControl (TileProcessor.cpp:958-966)
        for (uint32_t l = 0; l < nlayers; ++l) if (layer_rc(l)) return true;
        return false;
    }
    // Per-component coding from main-header COC markers (A.6.2; CodeStreamDecompress read_coc):
    // decomposition levels, code-block size and style, transform, precincts.  Empty: every
    // component takes the COD's (always so on encode: grk_cparameters has one coding style).
    struct CompCod {
        uint32_t numres = 6, cbw = 6, cbh = 6, cblk_sty = 0, irrev = 0;
        uint32_t prcw[GK_MAXRLVLS], prch[GK_MAXRLVLS];
    };
    std::vector<CompCod> cc;
    uint32_t c_numres(uint32_t c) const { return cc.empty() ? numres : cc[c].numres; }
    uint32_t c_cbw(uint32_t c) const { return cc.empty() ? cbw : cc[c].cbw; }
    uint32_t c_cbh(uint32_t c) const { return cc.empty() ? cbh : cc[c].cbh; }
    uint32_t c_sty(uint32_t c) const { return cc.empty() ? cblk_sty : cc[c].cblk_sty; }
    uint32_t c_irrev(uint32_t c) const { return cc.empty() ? irrev : cc[c].irrev; }
    uint32_t c_prcw(uint32_t c, uint32_t r) const { return cc.empty() ? prcw[r] : cc[c].prcw[r]; }
    uint32_t c_prch(uint32_t c, uint32_t r) const { return cc.empty() ? prch[r] : cc[c].prch[r]; }
    bool c_ht(uint32_t c) const { return (c_sty(c) & 0x40) != 0; }
    bool c_wide(uint32_t c) const { return c_cbw(c) > 6 || c_cbh(c) > 6; }
    // T1 kernel class of a component's blocks: 0 the headline Part-1 coders, 1 the lane-per-block
    // coders of gk_t1ms.hip (mode switches or wide blocks), 2 HTJ2K; with the style bits and width
    uint32_t c_class(uint32_t c) const {
        const uint32_t k = c_ht(c) ? 2u : ((c_sty(c) & 0x3f) || c_wide(c)) ? 1u : 0u;
        return k | (c_sty(c) & 0x3f) << 2 | (c_wide(c) ? 1u << 8 : 0u);
    }
};

struct BandG {
    uint32_t orient, x0, y0, x1, y1;
    uint32_t level;       // decomposition level (1..L), 0 for the final LL
    uint32_t expn, mant, numbps;
    float step_enc, step_dec;
    uint32_t plane;       // 0 = A, 1 = B
    uint32_t offx, offy;  // placement inside that plane
    bool empty() const { return x1 <= x0 || y1 <= y0; }
};
struct PrecG {
    uint32_t cw = 0, ch = 0;
    uint32_t first_block = 0;   // index into Plan::blocks (canonical order)
    uint32_t tree = 0;          // index of this precinct-band's tag trees
};
struct ResG {
    uint32_t x0, y0;      // resolution origin on the reference grid (B.5)
    uint32_t w, h, pw, ph, cbw, cbh;
    uint32_t px0, py0;    // precinct grid origin (resolution coordinates)
    std::vector<BandG> bands;
    std::vector<std::vector<PrecG>> prc;   // [band][precinct]
};
struct CompG {
    std::vector<ResG> res;
};

// One tile (B.3).  Its samples live in the tile's rectangle of the image-sized
// work planes, so DC/MCT run once over the image and every tile's DWT levels
// and code-blocks are windows of the same planes.
struct TileG {
    uint32_t x0, y0, x1, y1;             // image coordinates
    std::vector<CompG> comps;
    uint32_t b0 = 0, b1 = 0;             // code-block range in Plan::blocks
};
// A class of tiles with the same geometry at every level (size, and resolution origins of the
// same parity): one DWT launch per level (grid.z = tile).  On a grid whose tile sizes are
// multiples of 2^L there are at most four (interior / last column x interior / last row); other
// sizes split the columns (rows) by tile origin modulo 2^L, so a class is the tile columns
// ci + k * si (rows cj + k * sj), k < tb.nx (tb.ny), and tb.dx = si * tw.
struct ShapeG {
    uint32_t w, h;
    std::vector<uint32_t> resw, resh;    // resolution sizes by level l = 0..L (l=0: full tile)
    std::vector<uint8_t> parx, pary;     // parity of the resolution origins by level (odd: cas1 lifting)
    uint32_t ci = 0, cj = 0, si = 1, sj = 1;
    uint32_t px0 = 0, py0 = 0;           // plane position of the first member's top-left
    GkTiles tb;
};

// Components sampled on one grid (SIZ XRsiz / YRsiz; grk_image_comp::dx / dy) and transformed
// alike (levels, 5/3 or 9/7: COD / COC): their tile-components are the tiles divided by
// (dx, dy), rounded up (TileProcessor.cpp:116-131), so they share one set of tile classes and DWT
// launches.  Without subsampling or COC there is one group holding every component.
struct SGroup {
    uint32_t dx = 1, dy = 1;
    uint32_t numres = 1, irrev = 0;      // the components' decomposition levels + 1 and transform (COD / COC)
    uint32_t ox = 0, oy = 0;             // the image area's origin on the group's grid: ceil(x0 / dx), ceil(y0 / dy)
    uint32_t w = 0, h = 0;               // its extent there (grk_image_comp w / h): a component plane's size
    std::vector<ShapeG> shapes;          // tile classes on the group's grid
    std::vector<int> shape_of;           // tile -> class
    std::vector<std::pair<uint32_t, uint32_t>> runs;   // its components as contiguous ranges [c0, c1)
};

struct Plan {
    uint32_t w = 0, h = 0, nc = 0, prec = 0, sgnd = 0;
    std::vector<uint8_t> cdx, cdy;       // per component subsampling (empty: none)
    // decode: per-component precision and signedness (SIZ Ssiz) when they differ (empty: prec /
    // sgnd for every component; prec is then the largest)
    std::vector<uint8_t> cprec, csgnd;
    uint32_t c_prec(uint32_t c) const { return c < cprec.size() ? cprec[c] : prec; }
    uint32_t c_sgnd(uint32_t c) const { return c < csgnd.size() ? csgnd[c] : sgnd; }
    uint32_t sx(uint32_t c) const { return c < cdx.size() ? cdx[c] : 1u; }
    uint32_t sy(uint32_t c) const { return c < cdy.size() ? cdy[c] : 1u; }
    bool subsampled() const {
        for (uint32_t c = 0; c < nc; ++c) if (sx(c) != 1 || sy(c) != 1) return true;
        return false;
    }
    // the inverse / forward MCT: COD's flag, three components or more, the first three on one
    // grid (Grok's encoder clears the flag otherwise, CodeStreamCompress.cpp:501-512; its decoder
    // skips the transform, TileProcessor::needsMctDecompress :432-456)
    bool mct3() const {
        return p.mct && nc >= 3 && sx(1) == sx(0) && sx(2) == sx(0) && sy(1) == sy(0) && sy(2) == sy(0);
    }
    // canvas (B.2-B.3): the image area starts at (x0, y0), the tile grid at (gx0, gy0) <= (x0, y0).
    // Tile and band geometry are canvas coordinates; work planes hold the image area, so a plane
    // position is a canvas position less (x0, y0).
    uint32_t x0 = 0, y0 = 0, gx0 = 0, gy0 = 0;
    Params p;
    uint32_t stride = 0;                 // work-plane stride (samples)
    size_t plane_elems = 0;              // per plane
    uint32_t ntx = 1, nty = 1, tw = 0, th = 0;   // tile grid
    std::vector<TileG> tiles;            // raster order
    std::vector<SGroup> groups;          // sampling grids (one without subsampling)
    std::vector<uint32_t> group_of;      // component -> group
    uint32_t max_numres() const { uint32_t m = 0; for (const SGroup& G : groups) m = std::max(m, G.numres); return m; }
    uint32_t min_numres() const { uint32_t m = 64; for (const SGroup& G : groups) m = std::min(m, G.numres); return m; }
    bool l1_fusable = true;              // every tile(-component) origin even: level 1 fuses with DC shift / MCT
    std::vector<GkBlock> blocks;         // tile order, then canonical: comp, res, band, precinct, cblk
    std::vector<uint32_t> bxy;           // per block: top-left (x, y) in its band's coordinates
    uint64_t slot_bytes = 0;
    std::vector<uint64_t> sym_off;       // T1 symbol-stream offsets (nblocks + 1)
    uint32_t ntrees = 0;                 // precinct-bands with code-blocks
};

// Caller sample type (GkSample) of planes described by (sample_bytes, sgnd).
static int sample_type(uint32_t sample_bytes, uint32_t prec, bool sgnd) {
    if (sample_bytes == 0 || sample_bytes == 4) return GK_S32;
    if (sample_bytes != (prec + 7) / 8) throw GkError("sample_bytes must be 4 or (prec + 7) / 8");
    if (sample_bytes == 1) return sgnd ? GK_S8 : GK_U8;
    return sgnd ? GK_S16 : GK_U16;
}

// The image rectangle the work planes hold during one call.  A plan's block offsets
// (GkBlock::band_off) address planes covering the whole image; a call that touches only
// some tiles (tile-range encode, sharded or windowed decode) allocates planes for the
// rectangle of those tiles alone and relocates the offsets of the blocks it codes.
struct Region {
    uint32_t x0 = 0, y0 = 0, w = 0, h = 0, stride = 0;
    size_t plane = 0;                    // elements per work plane
};
static Region make_region(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    Region R;
    R.x0 = x0; R.y0 = y0; R.w = x1 - x0; R.h = y1 - y0;
    R.stride = align_up(std::max(R.w, 1u), 64);
    R.plane = (size_t)R.stride * R.h;
    return R;
}
static inline uint64_t relocate(const Plan& P, const Region& R, uint64_t band_off) {
    const uint64_t q = band_off / P.plane_elems, rem = band_off % P.plane_elems;
    const uint64_t y = rem / P.stride, x = rem % P.stride;
    return q * R.plane + (y - R.y0) * R.stride + (x - R.x0);
}
// The region R (image-relative, full-resolution canvas grid) on sampling group G's grid: its
// canvas edges divided by (dx, dy), rounded up, less the group's image origin; the work planes
// keep R's stride and size (a subsampled grid is never larger).  Without subsampling R itself.
static inline Region group_region(const Plan& P, const Region& R, const SGroup& G) {
    Region g = R;
    g.x0 = ceildiv(R.x0 + P.x0, G.dx) - G.ox; g.y0 = ceildiv(R.y0 + P.y0, G.dy) - G.oy;
    g.w = ceildiv(R.x0 + R.w + P.x0, G.dx) - G.ox - g.x0; g.h = ceildiv(R.y0 + R.h + P.y0, G.dy) - G.oy - g.y0;
    return g;
}

// DWT basis-function norms (T1.cpp:264-277 getnorm_53 / getnorm_97; ISO 15444-1 Annex E)
static double band_norm(uint32_t level, uint32_t orient, bool rev) {
    static const double n53[4][10] = {
        {1.000, 1.500, 2.750, 5.375, 10.68, 21.34, 42.67, 85.33, 170.7, 341.3},
        {1.038, 1.592, 2.919, 5.703, 11.33, 22.64, 45.25, 90.48, 180.9},
        {1.038, 1.592, 2.919, 5.703, 11.33, 22.64, 45.25, 90.48, 180.9},
        {.7186, .9218, 1.586, 3.043, 6.019, 12.01, 24.00, 47.97, 95.93}};
    static const double n97[4][10] = {
        {1.000, 1.965, 4.177, 8.403, 16.90, 33.84, 67.69, 135.3, 270.6, 540.9},
        {2.022, 3.989, 8.355, 17.04, 34.27, 68.63, 137.3, 274.6, 549.0},
        {2.022, 3.989, 8.355, 17.04, 34.27, 68.63, 137.3, 274.6, 549.0},
        {2.080, 3.865, 8.307, 17.18, 34.71, 69.59, 139.3, 278.6, 557.2}};
    if (orient == 0 && level > 9) level = 9;
    else if (orient > 0 && level > 8) level = 8;
    return rev ? n53[orient][level] : n97[orient][level];
}

// HT reversible QCD: param_qcd::set_rev_quant (HTParams.cpp:253-272) —
// exponent = B + ceil(log2(bibo_gain^2 * 1.1)) with the 5/3 BIBO gains
// (HTParams.cpp:134-145).  Grok evaluates it before tcp->mct is set
// (CodeStreamCompress.cpp:382 vs :396), so B is the sample precision.
static uint32_t ht_rev_expn(uint32_t B, uint32_t ndecomp, uint32_t r, uint32_t orient) {
    static const float gl[16] = {1.0000f, 1.5000f, 1.6250f, 1.6875f, 1.6963f, 1.7067f, 1.7116f, 1.7129f,
                                 1.7141f, 1.7145f, 1.7151f, 1.7152f, 1.7155f, 1.7155f, 1.7156f, 1.7156f};
    static const float gh[16] = {2.0000f, 2.5000f, 2.7500f, 2.8047f, 2.8198f, 2.8410f, 2.8558f, 2.8601f,
                                 2.8628f, 2.8656f, 2.8662f, 2.8667f, 2.8669f, 2.8670f, 2.8671f, 2.8671f};
    auto L = [&](uint32_t i) { return gl[std::min(i, 15u)]; };
    auto H = [&](uint32_t i) { return gh[std::min(i, 15u)]; };
    auto X = [](float g) { return (int)ceil(log(g * 1.1f) / 0.69314718055994530942); };
    if (r == 0) return (uint32_t)((int)B + X(L(ndecomp) * L(ndecomp)));
    const uint32_t d = ndecomp - r;
    return (uint32_t)((int)B + (orient == 3 ? X(H(d) * H(d)) : X(H(d) * L(d + 1))));
}

// HT irreversible QCD: param_qcd::set_irrev_quant (HTParams.cpp:273-317), base_delta =
// 2^-(bit depth + signed) (:211-212), 9/7 synthesis energy gains (sqrt_energy_gains,
// HTParams.cpp:75-86: constant data of the 9/7 filter bank).
static void ht_irrev_quant(uint32_t prec, bool sgnd, uint32_t nd, uint32_t r, uint32_t orient, uint32_t& expn,
                           uint32_t& mant) {
    static const float L97[34] = {
        1.0000e+00f, 1.4021e+00f, 2.0304e+00f, 2.9012e+00f, 4.1153e+00f, 5.8245e+00f, 8.2388e+00f, 1.1652e+01f, 1.6479e+01f,
        2.3304e+01f, 3.2957e+01f, 4.6609e+01f, 6.5915e+01f, 9.3217e+01f, 1.3183e+02f, 1.8643e+02f, 2.6366e+02f, 3.7287e+02f,
        5.2732e+02f, 7.4574e+02f, 1.0546e+03f, 1.4915e+03f, 2.1093e+03f, 2.9830e+03f, 4.2185e+03f, 5.9659e+03f, 8.4371e+03f,
        1.1932e+04f, 1.6874e+04f, 2.3864e+04f, 3.3748e+04f, 4.7727e+04f, 6.7496e+04f, 9.5454e+04f};
    static const float H97[34] = {
        1.4425e+00f, 1.9669e+00f, 2.8839e+00f, 4.1475e+00f, 5.8946e+00f, 8.3472e+00f, 1.1809e+01f, 1.6701e+01f, 2.3620e+01f,
        3.3403e+01f, 4.7240e+01f, 6.6807e+01f, 9.4479e+01f, 1.3361e+02f, 1.8896e+02f, 2.6723e+02f, 3.7792e+02f, 5.3446e+02f,
        7.5583e+02f, 1.0689e+03f, 1.5117e+03f, 2.1378e+03f, 3.0233e+03f, 4.2756e+03f, 6.0467e+03f, 8.5513e+03f, 1.2093e+04f,
        1.7103e+04f, 2.4187e+04f, 3.4205e+04f, 4.8373e+04f, 6.8410e+04f, 9.6747e+04f, 1.3682e+05f};
    const float base_delta = 1.0f / (float)(1u << (prec + (sgnd ? 1 : 0)));
    float gl, gh;
    if (r == 0) { gl = L97[nd]; gh = gl; }
    else { const uint32_t d = nd - r; gl = orient == 3 ? H97[d] : L97[d + 1]; gh = H97[d]; }
    float delta_b = base_delta / (gl * gh);
    uint32_t e = 0;
    while (delta_b < 1.0f) { e++; delta_b *= 2.0f; }
    const uint32_t m = (uint32_t)round(delta_b * (float)(1 << 11)) - (1 << 11);
    mant = m < (1u << 11) ? m : 0x7ff;
    expn = e;
}

static void assign_steps_tile(Plan& P, TileG& T) {
    for (uint32_t ci = 0; ci < (uint32_t)T.comps.size(); ++ci) {
        CompG& C = T.comps[ci];
        const uint32_t nres = P.p.c_numres(ci), irrev = P.p.c_irrev(ci);
        const bool ht = P.p.c_ht(ci);
        for (uint32_t r = 0; r < nres; ++r) {
            for (auto& B : C.res[r].bands) {
                uint32_t level = nres - 1 - r;
                if (ht && !irrev) {
                    B.mant = 0;
                    B.expn = ht_rev_expn(P.prec, nres - 1, r, B.orient);
                    B.step_enc = B.step_dec = 1.0f;
                    B.numbps = (uint32_t)std::max(0, (int)B.expn + (int)P.p.numgbits - 1) + P.p.roi(ci);
                    continue;
                }
                uint32_t gain = irrev ? 0 : (B.orient == 0 ? 0 : (B.orient == 3 ? 2 : 1));
                if (ht) {
                    ht_irrev_quant(P.prec, P.sgnd != 0, nres - 1, r, B.orient, B.expn, B.mant);
                } else {
                // Part-1 QCD generation (HTParams.cpp:216-251)
                double stepsize = 1.0;
                if (irrev) stepsize = (double)(1u << gain) / band_norm(level, B.orient, false);
                uint32_t step = (uint32_t)floor(stepsize * 8192.0);
                int pp = floorlog2(step) - 13, n = 11 - floorlog2(step);
                B.mant = (n < 0 ? step >> -n : step << n) & 0x7ff;
                B.expn = (uint32_t)((int)(P.prec + gain) - pp);
                }
                // Quantizer::setBandStepSizeAndBps (Quantizer.cpp:26-66)
                uint32_t lg_enc = B.orient == 0 ? 0 : (B.orient == 3 ? 2 : 1);
                uint32_t lg_dec = irrev ? 0 : lg_enc;
                B.step_enc = (float)((1.0 + B.mant / 2048.0) * pow(2.0, (int)(P.prec + lg_enc) - (int)B.expn));
                B.step_dec = (float)((1.0 + B.mant / 2048.0) * pow(2.0, (int)(P.prec + lg_dec) - (int)B.expn));
                int v = (int)B.expn + (int)P.p.numgbits - 1;
                B.numbps = P.p.roi(ci) + (uint32_t)std::max(0, v);   // Quantizer.cpp:47: roishift + ...
            }
        }
    }
}

// A stream's quantisation per component (QCD, replaced per component by a main-header QCC, A.6.4-
// A.6.5) as one flat list: for each component a (guard bits, ~0u) entry, then the (expn, mant) of
// its bands, LL first then (HL, LH, HH) per resolution, scalar-derived steps already expanded.
typedef std::vector<std::pair<uint32_t, uint32_t>> QuantList;
static void apply_qcd(Plan& P, const QuantList& q) {
    // the start of each component's entries
    std::vector<size_t> at;
    for (size_t k = 0; k < q.size(); ++k) if (q[k].second == ~0u) at.push_back(k);
    if (at.size() != P.nc) throw GkError("quantisation list does not match the component count");
    for (auto& T : P.tiles)
    for (uint32_t ci = 0; ci < (uint32_t)T.comps.size(); ++ci) {
        CompG& C = T.comps[ci];
        const size_t k0 = at[ci] + 1, k1 = ci + 1 < at.size() ? at[ci + 1] : q.size();
        if (k1 <= k0) throw GkError("QCD / QCC without step sizes");
        const uint32_t gb = q[at[ci]].first;
        uint32_t bandno = 0;
        for (uint32_t r = 0; r < P.p.c_numres(ci); ++r)
            for (auto& B : C.res[r].bands) {
                size_t k = std::min<size_t>(k0 + bandno, k1 - 1);
                B.expn = q[k].first; B.mant = q[k].second;
                uint32_t lg_enc = B.orient == 0 ? 0 : (B.orient == 3 ? 2 : 1);
                uint32_t lg_dec = P.p.c_irrev(ci) ? 0 : lg_enc;
                const uint32_t prec = P.c_prec(ci);   // (R_b = the component's precision + gain, Quantizer.cpp:40-42)
                B.step_enc = (float)((1.0 + B.mant / 2048.0) * pow(2.0, (int)(prec + lg_enc) - (int)B.expn));
                B.step_dec = (float)((1.0 + B.mant / 2048.0) * pow(2.0, (int)(prec + lg_dec) - (int)B.expn));
                B.numbps = P.p.roi(ci) + (uint32_t)std::max(0, (int)B.expn + (int)gb - 1);
                ++bandno;
            }
    }
}
// Sqcd / Sqcc + SPqcd / SPqcc -> guard bits and band steps (Quantizer::read_SQcd_SQcc,
// Quantizer.cpp:185-334): no quantisation (one byte per band, exponent << 3), scalar expounded
// (16 bits per band), scalar derived (the LL step only; band b > 0 takes expn_0 - floor((b - 1) / 3)
// and mant_0, :319-331, i.e. E-5's epsilon_0 - N_L + n_b)
static void parse_quant(const std::vector<uint8_t>& b, uint32_t numres, QuantList& out) {
    if (b.size() < 2) throw GkError("corrupt QCD / QCC marker");
    const uint32_t sq = b[0], qt = sq & 0x1f, nb = 3 * numres - 2;
    out.push_back({sq >> 5, ~0u});
    const size_t k0 = out.size();
    if (qt == 0) for (size_t k = 1; k < b.size(); ++k) out.push_back({(uint32_t)b[k] >> 3, 0u});
    else if (qt == 1 || qt == 2) for (size_t k = 1; k + 1 < b.size(); k += 2) { uint32_t v = (uint32_t)b[k] << 8 | b[k + 1]; out.push_back({v >> 11, v & 0x7ff}); }
    else throw GkError("corrupt QCD / QCC marker (quantisation style)");
    if (out.size() == k0) throw GkError("QCD / QCC without step sizes");
    if (qt == 1) {
        const auto s0 = out[k0];
        out.resize(k0 + nb);
        for (uint32_t k = 1; k < nb; ++k) out[k0 + k] = {s0.first > (k - 1) / 3 ? s0.first - (k - 1) / 3 : 0u, s0.second};
    }
}

static void build_tile(Plan& P, TileG& T, uint32_t t) {
    T.comps.assign(P.nc, CompG());
    T.b0 = (uint32_t)P.blocks.size();
    // tile-component c: the tile divided by its component's subsampling (the tile itself without)
    std::vector<uint32_t> tcx0(P.nc), tcy0(P.nc), tcx1(P.nc), tcy1(P.nc);
    for (uint32_t c = 0; c < P.nc; ++c) {
        tcx0[c] = ceildiv(T.x0, P.sx(c)); tcy0[c] = ceildiv(T.y0, P.sy(c));
        tcx1[c] = ceildiv(T.x1, P.sx(c)); tcy1[c] = ceildiv(T.y1, P.sy(c));
    }
    for (uint32_t c = 0; c < P.nc; ++c) {
        CompG& C = T.comps[c];
        const SGroup& G = P.groups[P.group_of[c]];
        const ShapeG& S = G.shapes[G.shape_of[t]];
        const uint32_t nres = P.p.c_numres(c), L = nres - 1;   // the component's coding (COD / COC)
        C.res.assign(nres, ResG());
        for (uint32_t r = 0; r < nres; ++r) {
            ResG& R = C.res[r];
            const uint32_t nb = L - r;
            R.x0 = ceildivpow2(tcx0[c], nb); R.y0 = ceildivpow2(tcy0[c], nb);
            R.w = ceildivpow2(tcx1[c], nb) - R.x0; R.h = ceildivpow2(tcy1[c], nb) - R.y0;
            const uint32_t pwe = P.p.c_prcw(c, r), phe = P.p.c_prch(c, r);
            R.px0 = (R.x0 >> pwe) << pwe; R.py0 = (R.y0 >> phe) << phe;
            R.pw = R.w ? ((ceildivpow2(R.x0 + R.w, pwe) << pwe) - R.px0) >> pwe : 0;
            R.ph = R.h ? ((ceildivpow2(R.y0 + R.h, phe) << phe) - R.py0) >> phe : 0;
            const uint32_t bpw = r ? pwe - 1 : pwe, bph = r ? phe - 1 : phe;
            R.cbw = std::min(P.p.c_cbw(c), bpw); R.cbh = std::min(P.p.c_cbh(c), bph);
            const uint32_t nbands = r ? 3 : 1;
            R.bands.assign(nbands, BandG());
            R.prc.assign(nbands, std::vector<PrecG>(R.pw * R.ph));
            for (uint32_t bi = 0; bi < nbands; ++bi) {
                BandG& B = R.bands[bi];
                B.orient = r ? bi + 1 : 0;
                if (!r) {
                    B.x0 = R.x0; B.y0 = R.y0; B.x1 = R.x0 + R.w; B.y1 = R.y0 + R.h;
                    B.level = L; B.offx = 0; B.offy = 0;
                    B.plane = L == 0 ? 0 : ((L & 1) ? 1 : 0);
                } else {
                    const uint32_t lev = nres - r;   // decomposition level of this band (1..L)
                    const uint32_t xo = B.orient & 1, yo = B.orient >> 1;
                    const uint64_t half = 1ull << (lev - 1);
                    auto cb = [&](uint64_t t, uint32_t o) -> uint32_t {   // B-15
                        if (!o) return ceildivpow2((uint32_t)t, lev);
                        return t <= half ? 0 : ceildivpow2((uint32_t)(t - half), lev);
                    };
                    B.x0 = cb(tcx0[c], xo); B.y0 = cb(tcy0[c], yo); B.x1 = cb(tcx1[c], xo); B.y1 = cb(tcy1[c], yo);
                    B.level = lev;
                    B.plane = (lev & 1) ? 1 : 0;
                    B.offx = xo ? S.resw[lev] : 0;   // Mallat placement inside the tile rectangle
                    B.offy = yo ? S.resh[lev] : 0;
                }
            }
        }
    }
    assign_steps_tile(P, T);
    // code-blocks, canonical order (T1CompressScheduler.cpp:31-94); grids are absolute
    for (uint32_t c = 0; c < P.nc; ++c) {
        CompG& C = T.comps[c];
        const SGroup& SG = P.groups[P.group_of[c]];
        const uint32_t nres = P.p.c_numres(c), irrev = P.p.c_irrev(c);
        for (uint32_t r = 0; r < nres; ++r) {
            ResG& R = C.res[r];
            const uint32_t pwe = P.p.c_prcw(c, r), phe = P.p.c_prch(c, r);
            const uint32_t bpw = r ? pwe - 1 : pwe, bph = r ? phe - 1 : phe;
            const uint32_t tlx = r ? R.px0 >> 1 : R.px0, tly = r ? R.py0 >> 1 : R.py0;
            for (uint32_t bi = 0; bi < R.bands.size(); ++bi) {
                BandG& B = R.bands[bi];
                for (uint32_t pi = 0; pi < R.pw * R.ph; ++pi) {
                    PrecG& PG = R.prc[bi][pi];
                    PG.first_block = (uint32_t)P.blocks.size();
                    PG.tree = P.ntrees;
                    if (B.empty()) continue;
                    const uint32_t i = pi % R.pw, j = pi / R.pw;
                    const uint32_t cx0 = tlx + (i << bpw), cy0 = tly + (j << bph);
                    const uint32_t px0 = std::max(cx0, B.x0), py0 = std::max(cy0, B.y0);
                    const uint32_t px1 = std::min(cx0 + (1u << bpw), B.x1), py1 = std::min(cy0 + (1u << bph), B.y1);
                    if (px1 <= px0 || py1 <= py0) continue;
                    const uint32_t gx0 = (px0 >> R.cbw) << R.cbw, gy0 = (py0 >> R.cbh) << R.cbh;
                    PG.cw = ((ceildivpow2(px1, R.cbw) << R.cbw) - gx0) >> R.cbw;
                    PG.ch = ((ceildivpow2(py1, R.cbh) << R.cbh) - gy0) >> R.cbh;
                    ++P.ntrees;
                    for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                        const uint32_t a = k % PG.cw, b = k / PG.cw;
                        const uint32_t kx0 = gx0 + (a << R.cbw), ky0 = gy0 + (b << R.cbh);
                        const uint32_t x0 = std::max(kx0, px0), y0 = std::max(ky0, py0);
                        const uint32_t x1 = std::min(kx0 + (1u << R.cbw), px1), y1 = std::min(ky0 + (1u << R.cbh), py1);
                        GkBlock G{};
                        const size_t plane_base = ((size_t)c * 2 + B.plane) * P.plane_elems;
                        // (plane positions on the component's grid, less the image origin there)
                        G.band_off = plane_base + (size_t)(tcy0[c] - SG.oy + B.offy + y0 - B.y0) * P.stride +
                                     (tcx0[c] - SG.ox + B.offx + x0 - B.x0);
                        G.stride = P.stride;
                        G.w = (uint16_t)(x1 - x0); G.h = (uint16_t)(y1 - y0);
                        G.orient = (uint8_t)B.orient; G.comp = (uint8_t)c;
                        G.band_numbps = (uint8_t)B.numbps;
                        // bits 3..7: the component's ROI shift (RGN; RoiShiftFilter on decode)
                        // (bit 1, rate control: set when an encode uploads the table, so one plan
                        // serves the encode and the decode of a rate-controlled stream)
                        G.flags = (irrev ? 1 : 0) | (uint8_t)(P.p.roi(c) << 3);
                        G.step = B.step_enc;
                        // T1::getwmsedec weight w1 * w2 * stepsize (T1.cpp:418-436): w1 = MCT basis norm
                        // (mct.cpp:689-704) when the MCT is on, w2 = DWT band norm (T1.cpp:264-277)
                        {
                            static const double norms_irrev[3] = {1.732, 1.805, 1.573};
                            static const double norms_rev[3] = {1.732, .8292, .8292};
                            const bool mct = P.mct3();
                            double w1 = (mct && c < 3) ? (irrev ? norms_irrev[c] : norms_rev[c]) : 1.0;
                            G.wmse = w1 * band_norm(nres - 1 - r, B.orient, !irrev) * (double)B.step_enc;
                        }
                        P.blocks.push_back(G);
                        P.bxy.push_back(x0); P.bxy.push_back(y0);
                    }
                }
            }
        }
    }
    T.b1 = (uint32_t)P.blocks.size();
}

static void build_plan(Plan& P) {
    P.stride = align_up(std::max(P.w, 1u), 64);
    P.plane_elems = (size_t)P.stride * P.h;
    // canvas extent of the image: [x0, X1) x [y0, Y1); without tiling one tile from the grid origin
    // (CodeStreamCompress.cpp:352-363)
    const uint32_t X1 = P.x0 + P.w, Y1 = P.y0 + P.h;
    P.tw = P.p.tw ? std::min(P.p.tw, X1 - P.gx0) : X1 - P.gx0;
    P.th = P.p.th ? std::min(P.p.th, Y1 - P.gy0) : Y1 - P.gy0;
    P.ntx = (X1 - P.gx0 + P.tw - 1) / P.tw; P.nty = (Y1 - P.gy0 + P.th - 1) / P.th;
    if ((size_t)P.ntx * P.nty > 65535) throw GkError("too many tiles");
    // tile classes: along each axis tile k spans [max(g + k t, o), min(g + (k + 1) t, end)); the
    // last tile (and a first tile cut by the image origin) is a class of its own, the others fall
    // into classes by origin modulo 2^L (m = 2^L / gcd(t, 2^L) of them, an arithmetic progression
    // each; one class on a 2^L-aligned grid)
    struct Axis { uint32_t first, step, count, size, origin; };   // origin: canvas position of the first member
    auto classes = [&](uint32_t n, uint32_t t, uint32_t g, uint32_t o, uint32_t end, uint32_t L) {
        std::vector<Axis> v;
        auto lo = [&](uint32_t k) { return std::max(g + k * t, o); };
        auto hi = [&](uint32_t k) { return std::min(g + (k + 1) * t, end); };
        // a first tile on the grid with the nominal size joins its residue class
        const uint32_t c0 = (o == g && n > 1) ? 0 : 1;
        if (c0) v.push_back({0, 1, 1, hi(0) - lo(0), lo(0)});
        if (n == 1) return v;
        const uint32_t G = 1u << L, lb = t & (0u - t), m = G / (lb < G ? lb : G);   // gcd(t, 2^L) = lowest set bit, capped
        for (uint32_t c = c0; c < std::min(c0 + m, n - 1); ++c) v.push_back({c, m, (n - 1 - c + m - 1) / m, t, lo(c)});
        v.push_back({n - 1, 1, 1, hi(n - 1) - lo(n - 1), lo(n - 1)});
        return v;
    };
    // sampling groups: components by (XRsiz, YRsiz), in order of first appearance
    P.groups.clear();
    P.group_of.assign(P.nc, 0);
    for (uint32_t c = 0; c < P.nc; ++c) {
        uint32_t g = 0;
        auto same = [&](const SGroup& G) {
            return G.dx == P.sx(c) && G.dy == P.sy(c) && G.numres == P.p.c_numres(c) && G.irrev == P.p.c_irrev(c);
        };
        while (g < P.groups.size() && !same(P.groups[g])) ++g;
        if (g == P.groups.size()) {
            P.groups.emplace_back();
            SGroup& G = P.groups[g];
            G.dx = P.sx(c); G.dy = P.sy(c); G.numres = P.p.c_numres(c); G.irrev = P.p.c_irrev(c);
        }
        P.group_of[c] = g;
        auto& runs = P.groups[g].runs;
        if (!runs.empty() && runs.back().second == c) runs.back().second = c + 1;
        else runs.push_back({c, c + 1});
    }
    P.l1_fusable = true;
    for (SGroup& G : P.groups) {
        // the tile grid on the group's grid: tile k spans ceil(edge / d) of the canvas tile, a regular
        // grid (origin ceil(g / d), pitch t / d) when d divides the nominal tile size
        if ((P.ntx > 1 && P.tw % G.dx) || (P.nty > 1 && P.th % G.dy))
            throw GkError("a component subsampling factor that does not divide the tile size is not supported on this path");
        const uint32_t tw = P.ntx > 1 ? P.tw / G.dx : ceildiv(P.tw, G.dx), th = P.nty > 1 ? P.th / G.dy : ceildiv(P.th, G.dy);
        G.ox = ceildiv(P.x0, G.dx); G.oy = ceildiv(P.y0, G.dy);
        G.w = ceildiv(X1, G.dx) - G.ox; G.h = ceildiv(Y1, G.dy) - G.oy;
        const uint32_t L = G.numres - 1;
        const std::vector<Axis> cx = classes(P.ntx, tw, ceildiv(P.gx0, G.dx), G.ox, ceildiv(X1, G.dx), L);
        const std::vector<Axis> cy = classes(P.nty, th, ceildiv(P.gy0, G.dy), G.oy, ceildiv(Y1, G.dy), L);
        G.shapes.clear();
        G.shape_of.assign((size_t)P.ntx * P.nty, -1);
        for (const Axis& ay : cy)
            for (const Axis& ax : cx) {
                ShapeG S;
                S.w = ax.size; S.h = ay.size;
                const uint32_t x0 = ax.origin, y0 = ay.origin;   // any member: the same geometry
                S.resw.resize(L + 1); S.resh.resize(L + 1); S.parx.resize(L + 1); S.pary.resize(L + 1);
                for (uint32_t l = 0; l <= L; ++l) {
                    S.resw[l] = ceildivpow2(x0 + S.w, l) - ceildivpow2(x0, l);
                    S.resh[l] = ceildivpow2(y0 + S.h, l) - ceildivpow2(y0, l);
                    S.parx[l] = (uint8_t)(ceildivpow2(x0, l) & 1);
                    S.pary[l] = (uint8_t)(ceildivpow2(y0, l) & 1);
                }
                if (S.parx[0] || S.pary[0]) P.l1_fusable = false;
                S.ci = ax.first; S.si = ax.step; S.cj = ay.first; S.sj = ay.step;
                S.px0 = x0 - G.ox; S.py0 = y0 - G.oy;
                S.tb.nx = ax.count; S.tb.ny = ay.count; S.tb.i0 = 0; S.tb.j0 = 0;
                S.tb.dx = ax.step * tw; S.tb.dy = ay.step * th;
                for (uint32_t b = 0; b < ay.count; ++b)
                    for (uint32_t a = 0; a < ax.count; ++a)
                        G.shape_of[(size_t)(ay.first + b * ay.step) * P.ntx + ax.first + a * ax.step] = (int)G.shapes.size();
                G.shapes.push_back(S);
            }
    }
    // level 1 fuses with the sample stage when every group has a level 1 and the MCT's three
    // components share a group (COC can give them different levels)
    for (const SGroup& G : P.groups) if (G.numres < 2) P.l1_fusable = false;
    if (P.mct3() && (P.group_of[1] != P.group_of[0] || P.group_of[2] != P.group_of[0])) P.l1_fusable = false;
    P.tiles.assign((size_t)P.ntx * P.nty, TileG());
    P.blocks.clear();
    P.bxy.clear();
    P.ntrees = 0;
    for (uint32_t t = 0; t < P.tiles.size(); ++t) {
        TileG& T = P.tiles[t];
        const uint32_t i = t % P.ntx, j = t / P.ntx;
        T.x0 = std::max(P.gx0 + i * P.tw, P.x0); T.y0 = std::max(P.gy0 + j * P.th, P.y0);
        T.x1 = std::min(P.gx0 + (i + 1) * P.tw, X1); T.y1 = std::min(P.gy0 + (j + 1) * P.th, Y1);
        build_tile(P, T, t);
    }
    // encode slots: w*h*4 + 64 bytes each, 64-byte aligned (the MQ coder stores whole 64-byte lines)
    uint64_t off = 0;
    for (auto& G : P.blocks) {
        uint32_t cap = (uint32_t)G.w * G.h * 4 + 64;
        G.data_off = off;
        G.data_cap = cap;
        off += align_up(cap, 64);
    }
    P.slot_bytes = off;
    // symbol streams for the parallel context modeller: band numbps planes x 11264 symbols
    P.sym_off.resize(P.blocks.size() + 1);
    uint64_t so = 0;
    for (size_t i = 0; i < P.blocks.size(); ++i) {
        P.sym_off[i] = so;
        so += (uint64_t)(P.blocks[i].band_numbps + 1) * 11264u;
        so = (so + 255) & ~255ull;
    }
    P.sym_off[P.blocks.size()] = so;
}

// ---------------------------------------------------------------------------
// Packet-header bit writer / reader (t2/BitIO.cpp) and tag trees (t2/TagTree.h)
// ---------------------------------------------------------------------------
// bit-stuffed writer (gk_bitio.h)
using BitWriter = PktBitWriter;
// one header coded into two writers at once
template <class A, class B> struct TeeWriter {
    A& a; B& b;
    inline void put(uint32_t v, uint32_t k) { a.put(v, k); b.put(v, k); }
    inline void putbit(uint32_t v) { a.putbit(v); b.putbit(v); }
    inline void write(uint32_t v, int n) { a.write(v, n); b.write(v, n); }
    void flush() { a.flush(); b.flush(); }
    void commacode(uint32_t n) { a.commacode(n); b.commacode(n); }
    void numpasses(uint32_t n) { a.numpasses(n); b.numpasses(n); }
};

struct TagTree {
    std::vector<int32_t> parent;
    std::vector<uint32_t> value, low;
    std::vector<uint8_t> known;
    void build(uint32_t nw, uint32_t nh) {
        std::vector<uint32_t> lw{nw}, lh{nh};
        size_t total = 0;
        while (true) {
            total += (size_t)lw.back() * lh.back();
            if ((size_t)lw.back() * lh.back() <= 1) break;
            lw.push_back((lw.back() + 1) / 2); lh.push_back((lh.back() + 1) / 2);
        }
        parent.assign(total, -1);
        size_t base = 0;
        for (size_t l = 0; l + 1 < lw.size(); ++l) {
            size_t nbase = base + (size_t)lw[l] * lh[l];
            for (uint32_t y = 0; y < lh[l]; ++y)
                for (uint32_t x = 0; x < lw[l]; ++x)
                    parent[base + (size_t)y * lw[l] + x] = (int32_t)(nbase + (size_t)(y / 2) * lw[l + 1] + x / 2);
            base = nbase;
        }
        value.assign(total, 0xffffffffu); low.assign(total, 0); known.assign(total, 0);
    }
    void reset() {
        std::fill(value.begin(), value.end(), 0xffffffffu);
        std::fill(low.begin(), low.end(), 0u);
        std::fill(known.begin(), known.end(), 0);
    }
    void setvalue(uint32_t leaf, uint32_t v) {
        int32_t n = (int32_t)leaf;
        while (n >= 0 && value[n] > v) { value[n] = v; n = parent[n]; }
    }
    // TagTree::encode (TagTree.h): from the root to the leaf, each node emits a 0 per unit its
    // low rises below min(value, threshold) and a 1 when it reaches a value below the
    // threshold the first time.  A node with nothing left to emit (low >= min(value,
    // threshold), and known if value < threshold) only has such nodes above it, and its low
    // bounds theirs, so the walk starts below the first one met going up from the leaf
    // (usually the leaf's parent, visited by the previous leaf); runs of bits go out at once.
    template <class W> void encode(W& bw, uint32_t leaf, uint32_t threshold) {
        uint32_t* lw = low.data();
        uint8_t* kn = known.data();
        int32_t stk[40]; int sp = 0; int32_t n = (int32_t)leaf;
        uint32_t lo = 0;
        while (true) {
            const uint32_t v = value[n];
            if (lw[n] >= std::min(v, threshold) && (v >= threshold || kn[n])) { lo = lw[n]; break; }
            stk[sp++] = n;
            if (parent[n] < 0) break;
            n = parent[n];
        }
        while (sp) {
            n = stk[--sp];
            if (lw[n] < lo) lw[n] = lo; else lo = lw[n];
            const uint32_t v = value[n];
            if (v < threshold) {
                const uint32_t z = v > lo ? v - lo : 0;
                const uint32_t one = kn[n] ? 0u : 1u;
                put_run(bw, z, one);
                kn[n] = 1;
                if (lo < v) lo = v;
            } else if (lo < threshold) {
                put_run(bw, threshold - lo, 0);
                lo = threshold;
            }
            lw[n] = lo;
        }
    }
    // z zero bits, then a 1 if one
    template <class W> static inline void put_run(W& bw, uint32_t z, uint32_t one) {
        for (; z >= 31; z -= 31) bw.put(0u, 31);
        if (z + one) bw.put(one, z + one);
    }
};

// Raw (unstuffed) packet-header bits, MSB first in left-aligned 64-bit words, with BitWriter's
// interface: the rate-control simulation codes each band of a packet on its own and counts
// the stuffed length of the concatenation afterwards (T2Enc::stuffed_len).
struct RawBits {
    std::vector<uint64_t> w;
    uint64_t acc = 0;   // pending bits, right-aligned
    uint32_t nacc = 0;
    uint64_t n = 0;     // bits written
    void clear() { w.clear(); acc = 0; nacc = 0; n = 0; }
    inline void put(uint32_t v, uint32_t k) {   // the low k <= 32 bits of v (higher bits zero)
        n += k;
        if (nacc + k < 64) { acc = (acc << k) | v; nacc += k; return; }
        const uint32_t k1 = 64 - nacc, k2 = k - k1;   // k1 in 1..32, k2 in 0..31
        w.push_back((acc << k1) | ((uint64_t)v >> k2));
        acc = (uint64_t)v & ((1ull << k2) - 1);
        nacc = k2;
    }
    void finish() { if (nacc) w.push_back(acc << (64 - nacc)); acc = 0; nacc = 0; }
    inline void putbit(uint32_t b) { put(b, 1); }
    inline void write(uint32_t v, int k) {
        if (k > 32) { put(0, (uint32_t)k - 32); k = 32; }
        put(k == 32 ? v : (v & ((1u << k) - 1)), (uint32_t)k);
    }
    void commacode(uint32_t c) {
        while (c >= 31) { put(0x7fffffffu, 31); c -= 31; }
        put(((1u << c) - 1) << 1, c + 1);
    }
    void numpasses(uint32_t np) {
        if (np == 1) put(0, 1);
        else if (np == 2) put(2, 2);
        else if (np <= 5) put(0xc | (np - 3), 4);
        else if (np <= 36) put(0x1e0 | (np - 6), 9);
        else put(0xff80 | (np - 37), 16);
    }
};

// Random-access byte source for decode: host memory, or device memory read
// through 64 KiB D2H pages.
struct ByteSrc {
    const uint8_t* host = nullptr;
    const uint8_t* dev = nullptr;
    size_t len = 0;
    hipStream_t st = nullptr;
    static const size_t PG = 1 << 16;
    // pages in pinned host memory from a process-wide pool (a pageable destination made each
    // synchronous 64 KiB fetch go through the runtime's bounce buffer).  At most kLive pinned
    // pages exist at once (256 MiB; past that a page is ordinary heap memory) and at most kKeep
    // of them stay pooled between decodes (64 MiB; the rest are freed when returned)
    struct PinnedPages {
        static const size_t kLive = 4096, kKeep = 1024;
        std::mutex m;
        std::vector<uint8_t*> free;
        size_t live = 0;
        uint8_t* get(bool& pinned) {
            {
                std::lock_guard<std::mutex> lk(m);
                if (!free.empty()) { uint8_t* p = free.back(); free.pop_back(); pinned = true; return p; }
                if (live >= kLive) { pinned = false; return (uint8_t*)malloc(PG); }
                ++live;
            }
            void* p = nullptr;
            if (hipHostMalloc(&p, PG, hipHostMallocDefault) != hipSuccess) {
                std::lock_guard<std::mutex> lk(m);
                --live;
                pinned = false;
                return (uint8_t*)malloc(PG);
            }
            pinned = true;
            return (uint8_t*)p;
        }
        void put(uint8_t* p) {
            {
                std::lock_guard<std::mutex> lk(m);
                if (free.size() < kKeep) { free.push_back(p); return; }
                --live;
            }
            (void)hipHostFree(p);
        }
    };
    static PinnedPages& pinned() { static PinnedPages* pp = new PinnedPages(); return *pp; }   // (never destroyed)
    struct PageDel {
        bool pin = true;
        void operator()(uint8_t* p) const { if (!p) return; if (pin) pinned().put(p); else ::free(p); }
    };
    std::unordered_map<size_t, std::unique_ptr<uint8_t, PageDel>> pages;
    size_t last_pg = ~(size_t)0;             // fast path: the page of the previous access
    const uint8_t* last = nullptr;
    // host copies of scattered ranges fetched in one batch (tile-part and packet headers),
    // sorted by start; a read outside them falls back to a page fetch
    struct Region { size_t start, len; const uint8_t* p; };
    std::shared_ptr<std::vector<Region>> regp = std::make_shared<std::vector<Region>>();
    size_t last_reg = ~(size_t)0;
    void add_regions(const std::vector<Region>& rs) {
        auto& regs = *regp;
        regs.insert(regs.end(), rs.begin(), rs.end());
        std::sort(regs.begin(), regs.end(), [](const Region& a, const Region& b) { return a.start < b.start; });
        last_reg = ~(size_t)0;
    }
    // a reader for another thread: shares the (read-only) regions, has its own page cache
    ByteSrc fork() const {
        ByteSrc b;
        b.host = host; b.dev = dev; b.len = len; b.st = st; b.regp = regp;
        return b;
    }
    inline bool from_region(size_t i, uint8_t& v) {
        const auto& regs = *regp;
        if (last_reg < regs.size() && i - regs[last_reg].start < regs[last_reg].len) {
            v = regs[last_reg].p[i - regs[last_reg].start];
            return true;
        }
        size_t lo = 0, hi = regs.size();
        while (lo < hi) { size_t m = (lo + hi) / 2; if (regs[m].start <= i) lo = m + 1; else hi = m; }
        for (size_t k = lo; k > 0 && k + 2 > lo; --k) {   // the last two regions starting at or before i
            const Region& R = regs[k - 1];
            if (i - R.start < R.len) { last_reg = k - 1; v = R.p[i - R.start]; return true; }
        }
        return false;
    }
    static std::atomic<uint64_t> fetch_ns, fetch_cnt;   // GK_PROFILE: synchronous page fetches
    const uint8_t* page(size_t pg) {
        auto it = pages.find(pg);
        if (it == pages.end()) {
            const auto t0 = std::chrono::steady_clock::now();
            size_t o = pg * PG, n = std::min(PG, len - o);
            bool pin = true;
            uint8_t* v = pinned().get(pin);
            if (!v) throw GkError("out of host memory for codestream pages");
            std::unique_ptr<uint8_t, PageDel> hold(v, PageDel{pin});
            HIPCHK(hipMemcpyAsync(v, dev + o, n, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            it = pages.emplace(pg, std::move(hold)).first;
            fetch_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
            ++fetch_cnt;
        }
        return it->second.get();
    }
    inline uint8_t at(size_t i) {
        if (i >= len) return 0;
        if (host) return host[i];
        const size_t pg = i / PG;
        if (pg == last_pg) return last[i - pg * PG];
        uint8_t v;
        if (!regp->empty() && from_region(i, v)) return v;
        last = page(pg); last_pg = pg;
        return last[i - pg * PG];
    }
    uint32_t be16(size_t i) { return ((uint32_t)at(i) << 8) | at(i + 1); }
    uint32_t be32(size_t i) { return (be16(i) << 16) | be16(i + 2); }
    // contiguous bytes [lo, hi) around i, for readers that scan forward (packet headers)
    const uint8_t* span(size_t i, size_t& lo, size_t& hi) {
        if (host) { lo = 0; hi = len; return host; }
        if (!regp->empty()) {
            uint8_t v;
            if (from_region(i, v)) {
                const Region& R = (*regp)[last_reg];
                lo = R.start; hi = R.start + R.len; return R.p;
            }
        }
        const size_t pg = i / PG;
        if (pg != last_pg) { last = page(pg); last_pg = pg; }
        lo = pg * PG; hi = std::min(len, lo + PG);
        return last;
    }
};
std::atomic<uint64_t> ByteSrc::fetch_ns{0}, ByteSrc::fetch_cnt{0};
// Packet-header bit reader (T2Decompress / BitIO: a byte after 0xFF carries 7 bits): up to 64
// unread bits in one register (gk_bitio.h), bytes from the source's cached windows.
using BitReader = PktBitReader<ByteSrc>;

struct DecTree {   // decoder-side tag tree
    std::vector<int32_t> parent;
    std::vector<uint32_t> value, low;
    void build(uint32_t nw, uint32_t nh) {
        TagTree t; t.build(nw, nh);
        parent = t.parent; value.assign(parent.size(), 0xffffffffu); low.assign(parent.size(), 0);
    }
    // TagTree::decode (TagTree.h): walk from the root to the leaf reading bits until each
    // node's value or the threshold is reached.  A node with nothing left to read at this
    // threshold (low >= min(threshold, value)) has only such nodes above it — a node is
    // processed only after its parent, and thresholds never decrease — and its final `lo` is
    // its `low`, so the walk starts below the first such node met going up from the leaf
    // (for raster-order leaves that is usually the leaf's parent).
    uint32_t decode(BitReader& br, uint32_t leaf, uint32_t threshold) {
        int32_t stk[40]; int sp = 0; int32_t n = (int32_t)leaf;
        uint32_t lo = 0;
        while (true) {
            if (low[n] >= std::min(threshold, value[n])) { lo = low[n]; break; }
            stk[sp++] = n;
            if (parent[n] < 0) break;
            n = parent[n];
        }
        while (sp) {
            n = stk[--sp];
            if (low[n] < lo) low[n] = lo; else lo = low[n];
            const uint32_t lim = std::min(threshold, value[n]);
            if (lo < lim) {   // zeros up to the node's value (a 1) or the threshold
                bool one;
                lo += br.run(0, lim - lo, one);
                if (one) value[n] = lo;
            }
            low[n] = lo;
        }
        return value[leaf];
    }
};

// ---------------------------------------------------------------------------
// T2 packet encoding with quality layers and PCRD rate allocation.
//   write_packet  — T2Compress::compressHeader + body (T2Compress.cpp:114-260,
//                   compressPacketSimulate :347-430 for the byte budget);
//   simulate      — compressPacketsSimulate (:59-112), LRCP;
//   make_layer    — makeLayerSimple / makeLayerFinal (TileProcessor.cpp:1367-1515);
//   allocate      — pcrdBisectSimple (:1196-1365) with updateRates
//                   (CodeStreamCompress.cpp:951-1025).
// Block k of the plan contributes lnp[k * nlayers + l] passes to layer l.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Packet order of one tile (ISO 15444-1 B.12; PacketIter::next_lrcp .. next_cprl,
// PacketIter.cpp:100-266).  For the position-driven orders the iterator walks x, y over the
// tile in steps of the smallest precinct (reference grid), starting at the tile origin and
// then at multiples of the step, and emits a precinct where the position is its first
// sample (generatePrecinctIndex, :287-335): with tile origins on the 2^levels grid that is
// the tile origin for a resolution's first precinct column / row and the precinct's own
// origin (a multiple of 2^(PP + level)) for the others.  So the walk is a sort by (anchor
// y, anchor x) with the order's other indices around it.
// ---------------------------------------------------------------------------
struct PacketRef { uint32_t l, r, c, pi; };
// One progression over layers [0, L), resolutions [r0, r1), components [c0, c1).
static void order_ranges(const Plan& P, const TileG& T, uint32_t prog, uint32_t L, uint32_t r0, uint32_t r1, uint32_t c0,
                         uint32_t c1, std::vector<PacketRef>& out) {
    // (a component coded with fewer resolutions (COC) has no packets at the higher ones,
    // PacketIter.cpp:160-162)
    auto np = [&](uint32_t c, uint32_t r) {
        if (r >= T.comps[c].res.size()) return 0u;
        const ResG& R = T.comps[c].res[r];
        return R.w && R.h ? R.pw * R.ph : 0u;
    };
    if (prog == 0 || prog == 1) {   // LRCP / RLCP
        for (uint32_t a = (prog == 0 ? 0 : r0); a < (prog == 0 ? L : r1); ++a)
            for (uint32_t b = (prog == 0 ? r0 : 0); b < (prog == 0 ? r1 : L); ++b)
                for (uint32_t c = c0; c < c1; ++c) {
                    const uint32_t l = prog == 0 ? a : b, r = prog == 0 ? b : a;
                    for (uint32_t pi = 0; pi < np(c, r); ++pi) out.push_back({l, r, c, pi});
                }
        return;
    }
    struct Pr { uint64_t ay, ax; uint32_t r, c, pi; };
    std::vector<Pr> v;
    for (uint32_t c = c0; c < c1; ++c)
        for (uint32_t r = r0; r < std::min<uint32_t>(r1, (uint32_t)T.comps[c].res.size()); ++r) {
            const ResG& R = T.comps[c].res[r];
            const uint32_t nr = (uint32_t)T.comps[c].res.size();
            const uint32_t n = np(c, r), lv = nr - 1 - r, pwe = P.p.c_prcw(c, r), phe = P.p.c_prch(c, r);
            // where Grok's walk (PacketIter::generatePrecinctIndex, PacketIter.cpp:287-335) first
            // meets precinct (i, j): the canvas position XRsiz * 2^(PPx + level) * (its grid index),
            // except a first precinct whose resolution starts off its precinct grid, which the
            // walk takes at the tile origin (that test without XRsiz, as there)
            const uint64_t sxc = P.sx(c), syc = P.sy(c);
            const bool offx = (((uint64_t)R.x0 << lv) & ((1ull << (pwe + lv)) - 1)) != 0;
            const bool offy = (((uint64_t)R.y0 << lv) & ((1ull << (phe + lv)) - 1)) != 0;
            for (uint32_t pi = 0; pi < n; ++pi) {
                const uint32_t i = pi % R.pw, j = pi / R.pw;
                const uint64_t ax = (i || !offx) ? sxc * (((uint64_t)(R.px0 >> pwe) + i) << (pwe + lv)) : T.x0;
                const uint64_t ay = (j || !offy) ? syc * (((uint64_t)(R.py0 >> phe) + j) << (phe + lv)) : T.y0;
                v.push_back({ay, ax, r, c, pi});
            }
        }
    auto key = [&](const Pr& a) {
        // RPCL: r, y, x, c; PCRL: y, x, c, r; CPRL: c, y, x, r (layers innermost)
        if (prog == 2) return std::make_tuple((uint64_t)a.r, a.ay, a.ax, (uint64_t)a.c);
        if (prog == 3) return std::make_tuple(a.ay, a.ax, (uint64_t)a.c, (uint64_t)a.r);
        return std::make_tuple((uint64_t)a.c, a.ay, a.ax, (uint64_t)a.r);
    };
    std::stable_sort(v.begin(), v.end(), [&](const Pr& a, const Pr& b) { return key(a) < key(b); });
    for (const Pr& q : v)
        for (uint32_t l = 0; l < L; ++l) out.push_back({l, q.r, q.c, q.pi});
}

// The tile's packet order: its progression, or with progression order changes (POC marker,
// A.6.6; PacketIter over the tile's progressions, each packet at most once: update_include)
// the concatenation of every entry's progression over its ranges, clamped to the stream's
// layers / resolutions / components, skipping packets an earlier entry already emitted.
// entry (optional) receives per packet the emitting entry and the packet's position in the
// entries' concatenated sequences, skipped packets counted: Grok's final pass runs each
// entry's iterator afresh, skips a packet written before through the tile's packet tracker
// (T2Compress.cpp:46-54, 278-280) and still counts it in tile->numProcessedPackets (SOP's Nsop).
static std::vector<PacketRef> packet_order(const Plan& P, const TileG& T, uint32_t L,
                                           const std::vector<Poc>* pocs = nullptr,
                                           std::vector<uint32_t>* entry = nullptr) {
    std::vector<PacketRef> out;
    const uint32_t NR = P.max_numres();   // (COC: components may have fewer)
    if (!pocs || pocs->empty()) {
        order_ranges(P, T, P.p.prog, L, 0, NR, 0, P.nc, out);
        return out;
    }
    // packet id: ((c * NR + r) * maxprc + pi) * L + l
    uint32_t maxprc = 1;
    for (uint32_t c = 0; c < P.nc; ++c)
        for (const ResG& R : T.comps[c].res) maxprc = std::max(maxprc, R.pw * R.ph);
    std::vector<uint8_t> seen((size_t)P.nc * NR * maxprc * L, 0);
    std::vector<PacketRef> sub;
    uint32_t iter = 0;
    for (uint32_t ei = 0; ei < (uint32_t)pocs->size(); ++ei) {
        const Poc& q = (*pocs)[ei];
        sub.clear();
        const uint32_t le = std::min(q.lye, L), r1 = std::min(q.re, NR), c1 = std::min(q.ce, P.nc);
        if (q.rs >= r1 || q.cs >= c1 || !le) continue;
        order_ranges(P, T, q.prog, le, q.rs, r1, q.cs, c1, sub);
        for (const PacketRef& pr : sub) {
            uint8_t& sflag = seen[(((size_t)pr.c * NR + pr.r) * maxprc + pr.pi) * L + pr.l];
            const uint32_t it = iter++;
            if (sflag) continue;
            sflag = 1;
            out.push_back(pr);
            if (entry) { entry->push_back(ei); entry->push_back(it); }
        }
    }
    return out;
}

// Tile parts per tile (CodeStreamCompress::getNumTilePartsForProgression,
// CodeStreamCompress.cpp:1899-1958): with divider D the indices of the progression string up
// to D (layers L, resolutions R, components C) each start a new tile part, so a tile has the
// product of their ranges and part k holds the packets whose leading indices form the k-th
// combination; those are contiguous in the packet order.  A divider behind the position
// index (P) is refused.  tp_key(pr) = the part of packet pr.
struct TilePartSplit {
    uint32_t n = 1;
    bool poc = false;   // one part per progression order change (part = the entry that emits the packet)
    int depth = -1;   // last progression-string position that splits
    const char* prog = "LRCP";
    uint32_t L = 1, R = 1, C = 1;
    uint32_t key(const PacketRef& pr) const {
        uint32_t k = 0;
        for (int j = 0; j <= depth; ++j) {
            const char ch = prog[j];
            if (ch == 'L') k = k * L + pr.l;
            else if (ch == 'R') k = k * R + pr.r;
            else k = k * C + pr.c;
        }
        return k;
    }
};
static TilePartSplit tile_part_split(const Plan& P) {
    static const char* names[5] = {"LRCP", "RLCP", "RPCL", "PCRL", "CPRL"};
    TilePartSplit S;
    S.prog = names[P.p.prog]; S.L = P.p.nlayers; S.R = P.p.numres; S.C = P.nc;
    if (!P.p.pocs.empty()) {
        // CodeStreamCompress::writeTileParts (:902-946): without a divider every progression
        // is a tile part of its own (getNumTilePartsForProgression returns 1 for each)
        if (P.p.tp_div) throw GkError("tile-part generation with progression order changes is not supported");
        S.n = (uint32_t)P.p.pocs.size(); S.poc = true;
        return S;
    }
    if (!P.p.tp_div) return S;
    for (int j = 0; j < 4; ++j) {
        const char ch = S.prog[j];
        if (ch == 'P') throw GkError("a tile-part divider behind the position index is not supported");
        S.n *= ch == 'L' ? S.L : ch == 'R' ? S.R : S.C;
        if (ch == P.p.tp_div) { S.depth = j; break; }
    }
    if (S.n > 255) throw GkError("more than 255 tile parts per tile");
    return S;
}

// Code-block style bits (grok.h:98-104) and T1::enc_is_term_pass (T1.cpp:437-458) for pass q
// of a block with nbp bit-planes: pass 0 is the first cleanup pass, then SP, MR, CL per plane.
enum { GK_STY_LAZY = 0x01, GK_STY_RESET = 0x02, GK_STY_TERMALL = 0x04, GK_STY_VSC = 0x08, GK_STY_PTERM = 0x10,
       GK_STY_SEGSYM = 0x20, GK_STY_HT = 0x40 };
static inline bool term_pass(uint32_t sty, uint32_t nbp, uint32_t q) {
    const int bpno = q == 0 ? (int)nbp - 1 : (int)nbp - 2 - (int)(q - 1) / 3;
    const int type = q == 0 ? 2 : (int)(q - 1) % 3;
    if (type == 2 && bpno == 0) return true;
    if (sty & GK_STY_TERMALL) return true;
    if (sty & GK_STY_LAZY) {
        if (bpno == (int)nbp - 4 && type == 2) return true;
        if (bpno < (int)nbp - 4 && type > 0) return true;
    }
    return false;
}

#ifdef PCRD_TRACE
static std::atomic<uint64_t> g_scans{0}, g_scan_passes{0};
#endif
struct T2Enc {
    const Plan& P;
    const uint32_t* info;        // 4 u32 per block: numbps, npasses, bytes, pass offset
    const GkPass* passes;        // packed pass records (only needed when passes split across layers)
    uint32_t L;                  // layers
    std::vector<uint16_t> lnp;   // passes per (block, layer)
    std::vector<uint16_t> inprev;   // T2 state: passes already in packets (numPassesInPacket)
    std::vector<uint8_t> nlb;       // T2 state: numlenbits
    std::vector<TagTree> incl, imsb;
    std::vector<uint8_t> hdr;
    uint32_t b0 = 0, b1 = 0;     // code-blocks of the tiles being written (tiles [tb, te))
    uint32_t t0 = 0, t1 = 0;     // those tiles; rate control runs on one tile (t1 == t0 + 1)
    bool serial = false;         // run on the calling thread (tiles allocated in parallel)
    template <class F> void prun(size_t n, const F& f) {
        if (serial) { for (size_t i = 0; i < n; ++i) f(i); return; }
        host_pool().run(n, f);
    }
    T2Enc(const Plan& plan, const uint32_t* inf, const GkPass* ps, uint32_t tb, uint32_t te)
        : P(plan), info(inf), passes(ps), L(plan.p.nlayers) {
        size_t nb = P.blocks.size();
        t0 = tb; t1 = te;
        b0 = P.tiles[tb].b0; b1 = P.tiles[te - 1].b1;
        lnp.assign(nb * L, 0); inprev.assign(nb, 0); nlb.assign(nb, 0);
        incl.resize(P.ntrees); imsb.resize(P.ntrees);
        // the tiles' tag trees are disjoint: many tiles (C4: 256 x ~18 trees) build in parallel
        auto build_tile = [&](size_t q) {
            for (auto& C : P.tiles[tb + (uint32_t)q].comps)
                for (auto& R : C.res)
                    for (size_t bi = 0; bi < R.bands.size(); ++bi)
                        for (auto& PG : R.prc[bi])
                            if (PG.cw && PG.ch) { incl[PG.tree].build(PG.cw, PG.ch); imsb[PG.tree].build(PG.cw, PG.ch); }
        };
        if (te - tb > 1) host_pool().run(te - tb, build_tile);
        else build_tile(0);
    }
    uint32_t npasses(uint32_t b) const { return info[4 * (size_t)b + 1]; }
    uint32_t rate(uint32_t b, uint32_t q) const {   // cumulative bytes after pass q (q < npasses)
        if (q + 1 == npasses(b)) return info[4 * (size_t)b + 2];
        return passes[info[4 * (size_t)b + 3] + q].rate;
    }
    // HT code-blocks have one pass and no distortion record (T1HT::compress sets only its
    // rate; CodePass zero-initialises distortiondec, Codeblock.h:47)
    double dist(uint32_t b, uint32_t q) const { return passes ? passes[info[4 * (size_t)b + 3] + q].dist : 0.0; }
    // The pass records (tens of MB) are read one or two per code-block in block order, each
    // a cache miss: prefetch those of the block PF ahead (its first pass not yet in packets
    // and the last one layer l would take).
    static constexpr uint32_t PF = 8;
    inline void prefetch_rates(uint32_t b, uint32_t l) const {
        const GkPass* p = passes + info[4 * (size_t)b + 3] + inprev[b];
        __builtin_prefetch(p - 1);
        __builtin_prefetch(p + lnp[(size_t)b * L + l] - 1);
    }

    // l == 0: fresh tag trees, every code-block's zero-bit-plane count in its tree
    void band_init(const PrecG& PG, uint32_t bnb) {
        incl[PG.tree].reset(); imsb[PG.tree].reset();
        for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
            const uint32_t b = PG.first_block + k;
            inprev[b] = 0;
            imsb[PG.tree].setvalue(k, bnb - info[4 * (size_t)b]);
        }
    }
    // one band's part of a packet header (T2Compress::compressHeader, T2Compress.cpp:114-240)
    template <class W> void band_header(const PrecG& PG, uint32_t l, W& bw) {
        const uint32_t n = PG.cw * PG.ch;
        TagTree& IT = incl[PG.tree];
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t b = PG.first_block + k;
            if (!inprev[b] && lnp[(size_t)b * L + l]) IT.setvalue(k, l);
        }
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t b = PG.first_block + k;
            if (passes && k + PF < n) prefetch_rates(b + PF, l);
            uint32_t np = lnp[(size_t)b * L + l];
            if (!inprev[b]) IT.encode(bw, k, l + 1);
            else bw.putbit(np != 0);
            if (!np) continue;
            if (!inprev[b]) { nlb[b] = 3; imsb[PG.tree].encode(bw, k, 0xffffffffu); }
            bw.numpasses(np);
            uint32_t r0 = inprev[b] ? rate(b, inprev[b] - 1) : 0;
            if (!(P.p.cblk_sty & (GK_STY_LAZY | GK_STY_TERMALL))) {
                // default style: one segment per contribution (only the last pass is terminated)
                uint32_t len = rate(b, inprev[b] + np - 1) - r0;
                int inc = std::max(0, floorlog2(len) + 1 - ((int)nlb[b] + floorlog2(np)));
                bw.commacode((uint32_t)inc);
                nlb[b] = (uint8_t)(nlb[b] + inc);
                bw.write(len, (int)nlb[b] + floorlog2(np));
                continue;
            }
            // one length per codeword segment: a segment ends at a terminated pass or at the
            // contribution's last pass (T2Compress.cpp:210-248)
            const uint32_t q0 = inprev[b], q1 = q0 + np, nbp = info[4 * (size_t)b];
            int inc = 0;
            for (uint32_t q = q0, s0 = q0, rs = r0; q < q1; ++q)
                if (term_pass(P.p.cblk_sty, nbp, q) || q + 1 == q1) {
                    const uint32_t re = rate(b, q);
                    inc = std::max(inc, floorlog2(re - rs) + 1 - ((int)nlb[b] + floorlog2(q + 1 - s0)));
                    s0 = q + 1; rs = re;
                }
            bw.commacode((uint32_t)inc);
            nlb[b] = (uint8_t)(nlb[b] + inc);
            for (uint32_t q = q0, s0 = q0, rs = r0; q < q1; ++q)
                if (term_pass(P.p.cblk_sty, nbp, q) || q + 1 == q1) {
                    const uint32_t re = rate(b, q);
                    bw.write(re - rs, (int)nlb[b] + floorlog2(q + 1 - s0));
                    s0 = q + 1; rs = re;
                }
        }
    }
    // one band's packet body bytes; advances its code-blocks' pass counts
    uint64_t band_body(const PrecG& PG, uint32_t l) {
        uint64_t sum = 0;
        for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
            const uint32_t b = PG.first_block + k;
            const uint32_t np = lnp[(size_t)b * L + l];
            if (!np) continue;
            const uint32_t r0 = inprev[b] ? rate(b, inprev[b] - 1) : 0;
            sum += rate(b, inprev[b] + np - 1) - r0;
            inprev[b] = (uint16_t)(inprev[b] + np);
        }
        return sum;
    }

    // One packet.  budget: remaining bytes (nullptr = unbounded).  seg (optional) receives
    // (block, first byte, length) body segments.  Returns false when the budget is exceeded.
    bool write_packet(const ResG& R, uint32_t pi, uint32_t l, uint64_t* budget,
                      std::vector<uint32_t>* seg) {
        return write_packet(R, pi, l, budget, seg, hdr);
    }
    // hdr_out: the packet header bytes (a per-thread buffer when tiles are written in parallel;
    // all other state touched is per code-block / per precinct, i.e. disjoint across tiles).
    // With a budget the header is only counted, as compressPacketSimulate (T2Compress.cpp:
    // 347-434) does in its uint32 arithmetic: M, the packet's bytes left, loses SOP's 6 bytes
    // untested, the header goes through Grok's bounded BitIO (GrkSimWriter: fails when its count
    // reaches M - never with none left, so such a packet passes and the subtraction wraps - and
    // misses a budget reached inside a number-of-passes or comma code), EPH's 2 bytes untested,
    // then each body must fit; M is not decremented once it is UINT_MAX.  The caller's budget
    // (compressPacketsSimulate's maxBytes) takes the packet's counted bytes, under the same
    // guard.  *sw (optional) reports a swallowed failure: the packet's counted header bytes.
    bool write_packet(const ResG& R, uint32_t pi, uint32_t l, uint64_t* budget,
                      std::vector<uint32_t>* seg, std::vector<uint8_t>& hdr, uint64_t* body_bytes = nullptr,
                      uint64_t* hdr_count = nullptr, bool* swallowed = nullptr) {
        if (l == 0)
            for (size_t bi = 0; bi < R.bands.size(); ++bi) {
                const PrecG& PG = R.prc[bi][pi];
                if (PG.cw && PG.ch) band_init(PG, R.bands[bi].numbps);
            }
        hdr.clear();
        constexpr uint32_t UMAX = 0xffffffffu;
        uint32_t M = 0;
        uint64_t counted = 0;
        if (budget) {
            M = (uint32_t)*budget;
            if (P.p.sop_eph & 2) { if (M != UMAX) M -= 6; counted += 6; }
            GrkSimWriter sw(M);
            BitWriter bw(hdr);   // the real header too (its length when a failure is swallowed)
            TeeWriter<GrkSimWriter, BitWriter> tw{sw, bw};
            tw.putbit(1);
            for (size_t bi = 0; bi < R.bands.size(); ++bi) {
                const PrecG& PG = R.prc[bi][pi];
                if (PG.cw && PG.ch) band_header(PG, l, tw);
            }
            tw.flush();
            if (sw.failed) return false;
            if (hdr_count) *hdr_count = sw.offset;
            if (swallowed) *swallowed = sw.swallowed;
            if (M != UMAX) M -= (uint32_t)sw.offset;
            counted += sw.offset;
            if (P.p.sop_eph & 4) { if (M != UMAX) M -= 2; counted += 2; }
        } else {
            BitWriter bw(hdr);
            bw.putbit(1);
            for (size_t bi = 0; bi < R.bands.size(); ++bi) {
                const PrecG& PG = R.prc[bi][pi];
                if (PG.cw && PG.ch) band_header(PG, l, bw);
            }
            bw.flush();
        }
        for (size_t bi = 0; bi < R.bands.size(); ++bi) {
            const PrecG& PG = R.prc[bi][pi];
            for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                uint32_t b = PG.first_block + k;
                uint32_t np = lnp[(size_t)b * L + l];
                if (!np) continue;
                uint32_t r0 = inprev[b] ? rate(b, inprev[b] - 1) : 0;
                uint32_t r1 = rate(b, inprev[b] + np - 1);
                if (budget) {
                    if (r1 - r0 > M) return false;
                    if (M != UMAX) M -= r1 - r0;
                    counted += r1 - r0;
                }
                if (seg) { seg->push_back(b); seg->push_back(r0); seg->push_back(r1 - r0); }
                if (body_bytes) *body_bytes += r1 - r0;
                inprev[b] = (uint16_t)(inprev[b] + np);
            }
        }
        if (budget && *budget != UMAX) *budget = (uint32_t)(*budget - counted);
        return true;
    }

    // A budget failure the simulation did not see (GrkSimWriter::swallowed): the packet, the
    // header bytes Grok's BitIO counted for it and its real header bytes.  When the final
    // simulation (pcrdBisectSimple :1352-1357) meets one, that count goes into the packet's PLT
    // entry and the tile part's precalculated length (SOT Psot / TLM, TileProcessor.cpp:243-259).
    struct Swallow { bool on = false; uint32_t c = 0, r = 0, pi = 0, l = 0; uint64_t hcnt = 0, hreal = 0; };
    Swallow final_sw;   // the final simulation's, once allocate() has run
    bool final_sw_pending = false;

    // T2Compress::compressPacketsSimulate (:59-112) walks every packet in the tile's own
    // progression whatever the progression order changes say: its THRESH_CALC PacketManager
    // sets each entry's progression to tcp->prg and its ranges to the whole tile
    // (updateCompressTcpProgressions, PacketManager.cpp:123-125, 565-589) and runs only the first
    // iterator (pocno = 1 outside Cinema 4K)
    bool simulate(uint32_t max_layers, uint64_t max_bytes, Swallow* swo = nullptr) {
        uint64_t budget = max_bytes;
        uint64_t* bp = max_bytes == 0xffffffffull ? nullptr : &budget;
        if (swo) *swo = Swallow();
        for (const PacketRef& pr : packet_order(P, P.tiles[t0], max_layers)) {   // rate control: one tile
            const ResG& R = P.tiles[t0].comps[pr.c].res[pr.r];
            uint64_t hc = 0;
            bool sw = false;
            if (!write_packet(R, pr.pi, pr.l, bp, nullptr, hdr, nullptr, &hc, &sw)) return false;
            if (sw && swo && !swo->on) *swo = Swallow{true, pr.c, pr.r, pr.pi, pr.l, hc, hdr.size()};
        }
        return true;
    }

    // ---- fast simulation for the bisection of layer l (single tile).  Layers < l are final,
    // so the T2 state after them is snapshotted once; every bisection step restores each
    // band of each packet (its tag trees and code-blocks) and codes only layer l.  A packet
    // header is the bit 1 followed by its bands' bits, and bands share no coding state, so
    // every (packet, band) is coded on its own into raw bits, in parallel, and the header
    // length is counted from the concatenation (stuffed_len).  compressPacketsSimulate's
    // bounded writes fail iff, with S the running size over packets in LRCP order, some
    // packet header reaches the remaining budget or some body exceeds it; sizes only grow,
    // so that is decided by the last packet:
    //   pass <=> S_(n-1) + hdr_n < budget  and  S_n <= budget.
    struct Chain { uint32_t c, r, pi; };
    struct Unit { uint32_t chain, band, nblk; };
    std::vector<Chain> chains;              // one layer's packets in LRCP order
    std::vector<Unit> units;                // (packet, band) pieces
    std::vector<uint32_t> uorder;           // units, largest first (dynamic schedule)
    std::vector<std::vector<uint32_t>> cunits;   // per packet: its units in band order
    std::vector<RawBits> ubits;
    std::vector<uint64_t> ubody;
    std::vector<TagTree> incl0, imsb0;      // snapshot after the final layers < l
    std::vector<uint16_t> inprev0;
    std::vector<uint8_t> nlb0;
    uint64_t prior = 0;                     // bytes of the final layers < l
    std::vector<uint64_t> csize, chdr;
    uint32_t last_chain = 0;                // chain of the layer's last packet in progression order
    void init_chains() {
        chains.clear(); units.clear();
        const TileG& T = P.tiles[t0];
        for (uint32_t r = 0; r < P.p.numres; ++r)
            for (uint32_t c = 0; c < P.nc; ++c)
                for (uint32_t pi = 0; pi < T.comps[c].res[r].pw * T.comps[c].res[r].ph; ++pi) chains.push_back({c, r, pi});
        // the packet the progression order writes last decides the budget test
        last_chain = chains.empty() ? 0 : (uint32_t)chains.size() - 1;
        {
            const std::vector<PacketRef> o1 = packet_order(P, T, 1);
            if (!o1.empty())
                for (uint32_t i = 0; i < (uint32_t)chains.size(); ++i)
                    if (chains[i].r == o1.back().r && chains[i].c == o1.back().c && chains[i].pi == o1.back().pi) last_chain = i;
        }
        cunits.assign(chains.size(), {});
        for (uint32_t i = 0; i < (uint32_t)chains.size(); ++i) {
            const ResG& R = T.comps[chains[i].c].res[chains[i].r];
            for (uint32_t bi = 0; bi < (uint32_t)R.bands.size(); ++bi) {
                const PrecG& PG = R.prc[bi][chains[i].pi];
                if (!PG.cw || !PG.ch) continue;
                cunits[i].push_back((uint32_t)units.size());
                units.push_back({i, bi, PG.cw * PG.ch});
            }
        }
        uorder.resize(units.size());
        for (uint32_t u = 0; u < (uint32_t)units.size(); ++u) uorder[u] = u;
        std::stable_sort(uorder.begin(), uorder.end(), [&](uint32_t x, uint32_t y) { return units[x].nblk > units[y].nblk; });
        ubits.assign(units.size(), RawBits());
        ubody.assign(units.size(), 0);
        csize.assign(chains.size(), 0); chdr.assign(chains.size(), 0);
        prior = 0;
        fsize.clear(); fhdr.clear(); ord_l = 0xffffffffu;
    }
    void restore_band(const PrecG& PG) {
        incl[PG.tree] = incl0[PG.tree]; imsb[PG.tree] = imsb0[PG.tree];
        for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
            const uint32_t b = PG.first_block + k;
            inprev[b] = inprev0[b]; nlb[b] = nlb0[b];
        }
    }
    // Bytes BitIO writes for the bit 1, the units' raw bits and a flush (BitIO.cpp): bytes
    // are 8-bit chunks of the raw bits, except that the chunk after an 0xFF byte carries 7
    // bits, and a final 0xFF byte is followed by one more.  Only chunk-grid positions where 8
    // ones start give 0xFF, so those positions are found word-wise and the rest is counted.
    uint64_t stuffed_len(const std::vector<uint32_t>& us, std::vector<uint64_t>& sb) const {
        sb.clear();
        uint64_t cur = 1ull << 63, N = 1;
        uint32_t cn = 1;
        auto app = [&](uint64_t x, uint32_t k) {   // the top k bits of x (bits below them zero)
            cur |= x >> cn;
            if (cn + k >= 64) { sb.push_back(cur); cur = cn ? x << (64 - cn) : 0; cn = cn + k - 64; }
            else cn += k;
        };
        for (uint32_t u : us) {
            const RawBits& rb = ubits[u];
            const size_t full = (size_t)(rb.n / 64);
            const uint32_t rem = (uint32_t)(rb.n % 64);
            for (size_t i = 0; i < full; ++i) app(rb.w[i], 64);
            if (rem) app(rb.w[full], rem);
            N += rb.n;
        }
        if (cn) sb.push_back(cur);
        sb.push_back(0);
        uint64_t pos = 0, bytes = 0;
        bool last_ff = false, end = false;
        for (size_t j = 0; j + 1 < sb.size() && !end; ++j) {
            const uint64_t x = sb[j], nx = sb[j + 1];
            uint64_t ones = x;
            for (int d = 1; d < 8; ++d) ones &= (x << d) | (nx >> (64 - d));
            while (ones && !end) {
                const int z = __builtin_clzll(ones);
                ones &= ~(1ull << (63 - z));
                const uint64_t p = (uint64_t)j * 64 + (uint64_t)z;   // bits p .. p+7 are ones
                if (p < pos || ((p - pos) & 7)) continue;
                bytes += (p - pos) / 8 + 1;                         // chunks up to the 0xFF one
                if (p + 8 >= N) { last_ff = true; pos = N; end = true; break; }
                bytes += 1;                                         // the 7-bit chunk after it
                pos = p + 15;
                if (pos >= N) { pos = N; end = true; }
            }
        }
        if (pos < N) bytes += (N - pos + 7) / 8;
        if (last_ff) ++bytes;
        return bytes;
    }
    const PrecG& unit_prec(const Unit& U, uint32_t* numbps = nullptr) const {
        const Chain& ch = chains[U.chain];
        const ResG& R = P.tiles[t0].comps[ch.c].res[ch.r];
        if (numbps) *numbps = R.bands[U.band].numbps;
        return R.prc[U.band][ch.pi];
    }
    void code_layer(uint32_t l) {   // every (packet, band) of layer l from the snapshot, in parallel
        const auto tc0 = std::chrono::steady_clock::now();
        // during a bounds_on bisection a unit none of whose counts changed since it was last
        // coded at this layer keeps its bits, body and coding state (they follow from the counts)
        const bool skip = skip_clean;
        if (skip) {
            cdirty.assign(chains.size(), 0);
            for (uint32_t u = 0; u < (uint32_t)units.size(); ++u) cdirty[units[u].chain] |= udirty[u];
        }
        prun(uorder.size(), [&](size_t j) {
            const uint32_t u = uorder[j];
            if (skip) { if (!udirty[u]) return; udirty[u] = 0; }
            const Unit& U = units[u];
            uint32_t numbps;
            const PrecG& PG = unit_prec(U, &numbps);
            if (l) restore_band(PG); else band_init(PG, numbps);
            // bits go to a thread-local writer and are swapped in at the end: units' writers
            // sit next to each other in ubits, and a bit-at-a-time writer shared a cache line
            // with its neighbours' (false sharing cost ~5x)
            thread_local RawBits rb;
            rb.clear();
            band_header(PG, l, rb);
            rb.finish();
            std::swap(rb, ubits[u]);
            ubody[u] = band_body(PG, l);
        });
        const auto tc2 = std::chrono::steady_clock::now();
        prun(chains.size(), [&](size_t i) {
            if (skip && !cdirty[i]) return;
            thread_local std::vector<uint64_t> sbuf;
            uint64_t body = 0;
            for (uint32_t u : cunits[i]) body += ubody[u];
            const uint64_t h = stuffed_len(cunits[i], sbuf);
            chdr[i] = h; csize[i] = h + body;
        });
        const auto tc3 = std::chrono::steady_clock::now();
        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count(); };
        prof_code += us(tc0, tc2); prof_stuff += us(tc2, tc3);
        static const bool check = getenv("GK_T2_CHECK_SIM") != nullptr;
        if (check) {   // debug: the packets' real sizes (write_packet) must match
            std::vector<uint8_t> hb;
            // and the coding state the simulation left must be the packets'
            const std::vector<TagTree> sim_incl = incl, sim_imsb = imsb;
            const std::vector<uint16_t> sim_inprev = inprev;
            const std::vector<uint8_t> sim_nlb = nlb;
            for (size_t i = 0; i < chains.size(); ++i) {
                const Chain& ch = chains[i];
                const ResG& R = P.tiles[t0].comps[ch.c].res[ch.r];
                if (l) for (uint32_t u : cunits[i]) restore_band(R.prc[units[u].band][ch.pi]);
                uint64_t body = 0;
                write_packet(R, ch.pi, l, nullptr, nullptr, hb, &body);
                if (hb.size() != chdr[i] || hb.size() + body != csize[i])
                    throw GkError("rate-control simulation: packet size mismatch");
            }
            auto same = [](const std::vector<TagTree>& a, const std::vector<TagTree>& b) {
                for (size_t t = 0; t < a.size(); ++t)
                    if (a[t].value != b[t].value || a[t].low != b[t].low || a[t].known != b[t].known) return false;
                return true;
            };
            if (!same(sim_incl, incl) || !same(sim_imsb, imsb) || sim_inprev != inprev || sim_nlb != nlb)
                throw GkError("rate-control simulation: coding state mismatch");
        }
    }
    uint64_t prof_code = 0, prof_stuff = 0;   // GK_PROFILE: code_layer phases (us)
    bool skip_clean = false;
    std::vector<uint8_t> cdirty;
    // The packets of layers <= l in progression order, as (chain, layer), and the final layers'
    // packet sizes: compressPacketsSimulate's outcome is a walk over them (packet_walk).
    std::vector<std::pair<uint32_t, uint32_t>> ord;
    uint32_t ord_l = 0xffffffffu;
    std::vector<std::vector<uint64_t>> fsize, fhdr;   // per final layer: each chain's packet bytes / header bytes
    void ensure_order(uint32_t l) {
        if (ord_l == l) return;
        const TileG& T = P.tiles[t0];
        std::vector<uint32_t> base((size_t)P.p.numres * P.nc, 0);   // first chain of (r, c)
        for (uint32_t i = (uint32_t)chains.size(); i-- > 0;) base[(size_t)chains[i].r * P.nc + chains[i].c] = i;
        ord.clear();
        for (const PacketRef& pr : packet_order(P, T, l + 1))
            ord.push_back({base[(size_t)pr.r * P.nc + pr.c] + pr.pi, pr.l});
        ord_l = l;
    }
    // compressPacketsSimulate (T2Compress.cpp:59-112) over packet sizes, in write_packet's
    // arithmetic: a body past the bytes left fails the layer, a packet met with no byte left
    // passes with all after it (its uint32 subtraction wraps), and a header reaching the bytes
    // left fails it unless that happens inside a number-of-passes or comma code, where Grok's
    // BitIO misses it and the count wraps as well (header_reaches).  Returns 1 (fits), 0 (fails)
    // or -1 when a final layer's packet header reaches the budget (its coding state is gone:
    // the caller runs the serial simulation).  *swo: a swallowed failure, if any.
    int packet_walk(uint32_t l, uint64_t max_bytes, Swallow* swo) {
        const bool sop = P.p.sop_eph & 2, eph = P.p.sop_eph & 4;
        constexpr uint32_t UMAX = 0xffffffffu;
        uint32_t rem = (uint32_t)max_bytes;
        *swo = Swallow();
        for (const auto& e : ord) {
            const uint64_t h = e.second < l ? fhdr[e.second][e.first] : chdr[e.first];
            const uint64_t sz = e.second < l ? fsize[e.second][e.first] : csize[e.first];
            uint32_t M = rem;
            if (sop && M != UMAX) M -= 6;
            uint64_t hc = h;
            if (M != 0 && h >= M) {
                if (e.second < l) return -1;
                if (!header_reaches(e.first, l, M, &hc)) return 0;
                if (!swo->on) {
                    const Chain& ch = chains[e.first];
                    *swo = Swallow{true, ch.c, ch.r, ch.pi, l, hc, h};
                }
            }
            if (M != UMAX) M -= (uint32_t)hc;
            if (eph && M != UMAX) M -= 2;
            const uint64_t body = sz - h;
            if (body > M) return 0;
            if (rem != UMAX) rem -= (uint32_t)(((sop ? 6 : 0) + hc + (eph ? 2 : 0) + body) & 0xffffffffu);
        }
        return 1;
    }
    // Layer l's packet of chain i, coded again from the snapshot through Grok's bounded BitIO
    // with M bytes left (GrkSimWriter): false if it fails, else true with the byte count it
    // reports (the failure swallowed).  The coding state ends as code_layer left it.
    bool header_reaches(uint32_t i, uint32_t l, uint32_t M, uint64_t* count) {
        GrkSimWriter sw(M);
        sw.putbit(1);
        for (uint32_t u : cunits[i]) {
            uint32_t numbps;
            const PrecG& PG = unit_prec(units[u], &numbps);
            if (l) restore_band(PG); else band_init(PG, numbps);
            band_header(PG, l, sw);
            band_body(PG, l);
        }
        sw.flush();
        *count = sw.offset;
        return !sw.failed;
    }
    // Could the walk above wrap before it fails?  That needs the bytes left in front of some
    // packet k to be 0 (0..5 with SOP) or, with EPH, 1 after its header: the running size
    // before k within [max_bytes - 8 - k's header bytes, max_bytes].  Bounds per chain (clo /
    // chi header bytes, cbody body bytes) for this layer, exact sizes for the final layers.
    bool may_hit(uint32_t l, uint64_t max_bytes) const {
        const uint64_t ovh = ((P.p.sop_eph & 2) ? 6 : 0) + ((P.p.sop_eph & 4) ? 2 : 0);
        uint64_t slo = 0, shi = 0;
        for (const auto& e : ord) {
            const uint64_t hmax = e.second < l ? fhdr[e.second][e.first] : chi[e.first];
            if (slo > max_bytes) return false;
            if (shi + hmax + 8 >= max_bytes) return true;
            if (e.second < l) { slo += fsize[e.second][e.first] + ovh; shi += fsize[e.second][e.first] + ovh; }
            else { slo += clo[e.first] + cbody[e.first] + ovh; shi += chi[e.first] + cbody[e.first] + ovh; }
        }
        return false;
    }
    bool simulate_layer(uint32_t l, uint64_t max_bytes, Swallow* swo) {
        *swo = Swallow();
        if (max_bytes == 0xffffffffull) return true;
        code_layer(l);
        ensure_order(l);
        const int r = packet_walk(l, max_bytes, swo);
        if (r >= 0) return r > 0;
        // the serial simulation, on a copy of the coding state the fast path keeps
        const std::vector<TagTree> si = incl, sm = imsb;
        const std::vector<uint16_t> sp = inprev;
        const std::vector<uint8_t> sn = nlb;
        const bool ok = simulate(l + 1, max_bytes, swo);
        incl = si; imsb = sm; inprev = sp; nlb = sn;
        return ok;
    }
    void finish_layer(uint32_t l) {   // layer l is final: advance the snapshot past it
        code_layer(l);
        for (uint64_t v : csize) prior += v;
        if (fsize.size() <= l) { fsize.resize(l + 1); fhdr.resize(l + 1); }
        fsize[l] = csize; fhdr[l] = chdr;
        incl0 = incl; imsb0 = imsb; inprev0 = inprev; nlb0 = nlb;
    }

    // ---- bisection steps decided without coding the packets.  A layer's header bits, all
    // but the stuffing, follow from its pass counts: per code-block the inclusion bit (blocks
    // already in packets), number of passes, comma code and length (make_layer caches them
    // with the count); the inclusion tag tree codes exactly one bit for every node with no
    // block included before l whose parent has one included by l (the root always: a node's
    // low is l when its parent lets it be coded, so it emits one 0 or one 1), and the
    // zero-bit-plane tree codes every node whose first block enters at l, from the parent's
    // value up to its own and a 1.  A header of R raw bits takes ceil(R/8) .. ceil(R/7)+2
    // bytes (a 7-bit chunk after each 0xFF, a final 0xFF doubled), so the layer's size is
    // known to a few parts in 10^4 and a step that range decides is not simulated.
    std::vector<uint32_t> bbits, blen;      // per code-block: header bits, body bytes at its count
    std::vector<uint32_t> ccount;           // per code-block: the count bbits/blen belong to
    std::vector<std::vector<uint8_t>> tA;   // per tree: a block of the subtree is in packets before l
    std::vector<std::vector<uint32_t>> tV;  // per tree: zero-bit-plane tag values (subtree minimum)
    std::vector<uint64_t> ubitn;            // per unit: raw header bits
    static uint32_t numpasses_bits(uint32_t n) { return n == 1 ? 1 : n == 2 ? 2 : n <= 5 ? 4 : n <= 36 ? 9 : 16; }
    // header bits (past the tag trees) and body bytes of block b taking passes [p0, inc)
    void block_cost(uint32_t b, uint32_t p0, uint32_t inc) {
        ccount[b] = inc;
        if (inc == p0) { bbits[b] = 0; blen[b] = 0; return; }
        const uint32_t np = inc - p0;
        const uint32_t len = rate(b, inc - 1) - (p0 ? rate(b, p0 - 1) : 0);
        const int nl = p0 ? (int)nlb0[b] : 3;
        const int c = std::max(0, floorlog2(len) + 1 - (nl + floorlog2(np)));
        bbits[b] = numpasses_bits(np) + (uint32_t)c + 1 + (uint32_t)(nl + c + floorlog2(np));
        blen[b] = len;
    }
    void bounds_prep(uint32_t l, const std::vector<uint16_t>& prev) {   // once per layer, after the snapshot
        const uint32_t nb = (uint32_t)P.blocks.size();
        if (bbits.size() != nb) { bbits.assign(nb, 0); blen.assign(nb, 0); ccount.assign(nb, 0xffffffffu); }
        tA.resize(P.ntrees); tV.resize(P.ntrees); tN.resize(P.ntrees); tC.resize(P.ntrees);
        ubitn.assign(units.size(), 0);
        ibits.assign(units.size(), 0); ibody.assign(units.size(), 0);
        udirty.assign(units.size(), 1);
        prun(uorder.size(), [&](size_t j) {   // units own disjoint trees and blocks
            const uint32_t u = uorder[j];
            uint32_t bnb;
            const PrecG& PG = unit_prec(units[u], &bnb);
            const std::vector<int32_t>& par = incl[PG.tree].parent;
            std::vector<uint8_t>& A = tA[PG.tree];
            A.assign(par.size(), 0);
            for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) A[k] = prev[PG.first_block + k] != 0;
            for (size_t n = 0; n < par.size(); ++n) if (A[n] && par[n] >= 0) A[par[n]] = 1;
            std::vector<uint32_t>& V = tV[PG.tree];
            if (V.size() != par.size()) {
                V.assign(par.size(), 0xffffffffu);
                for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) V[k] = bnb - info[4 * (size_t)(PG.first_block + k)];
                for (size_t n = 0; n < par.size(); ++n) if (par[n] >= 0) V[par[n]] = std::min(V[par[n]], V[n]);
            }
            // incremental state with no block included at l (see make_layer_inc)
            tN[PG.tree].assign(par.size(), 0);
            std::vector<uint32_t>& C = tC[PG.tree];
            C.assign(par.size(), 0);
            uint64_t bits = 0;
            for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                const uint32_t b = PG.first_block + k;
                bits += prev[b] != 0;
                lnp[(size_t)b * L + l] = 0;
                ccount[b] = prev[b]; bbits[b] = 0; blen[b] = 0;
            }
            for (size_t n = 0; n < par.size(); ++n) {
                if (A[n]) continue;
                if (par[n] < 0 || A[par[n]]) bits += 1;
                if (par[n] >= 0) C[par[n]] += 1;
            }
            ibits[u] = bits;
        });
        // work chunks: pieces of one unit's blocks, the unit's changes applied under its lock
        if (chunks.empty())
            for (uint32_t u = 0; u < (uint32_t)units.size(); ++u) {
                const uint32_t fb = unit_prec(units[u]).first_block;
                for (uint32_t k = 0; k < units[u].nblk; k += chunk_blocks())
                    chunks.push_back({u, fb + k, fb + std::min(units[u].nblk, k + chunk_blocks()), {}, {}, 0, HUGE_VAL, -HUGE_VAL});
            }
        nact = 0;
        for (ChunkI& C : chunks) {
            C.mslo = HUGE_VAL; C.mshi = -HUGE_VAL;
            C.act.resize(C.e - C.s);
            for (uint32_t b = C.s; b < C.e; ++b) C.act[b - C.s] = b;
            nact += C.act.size();
        }
        lay_hash = 0;
        jlog.clear();
        if (jstamp.size() != nb) { jstamp.assign(nb, 0); jgen = 0; }
    }
    // -1: the layer's packets overrun max_bytes, 1: they fit, 0: too close to call
    std::vector<uint64_t> clo, chi, cbody;   // per packet: header byte bounds, body bytes
    int decide(uint32_t l, uint64_t max_bytes, const std::vector<uint16_t>& prev) {
        if (max_bytes == 0xffffffffull) return 1;
        prun(uorder.size(), [&](size_t j) {
            const uint32_t u = uorder[j];
            const PrecG& PG = unit_prec(units[u]);
            const std::vector<int32_t>& par = incl[PG.tree].parent;
            const std::vector<uint8_t>& A = tA[PG.tree];
            const std::vector<uint32_t>& V = tV[PG.tree];
            thread_local std::vector<uint8_t> N;
            N.assign(par.size(), 0);
            uint64_t bits = 0, body = 0;
            for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                const uint32_t b = PG.first_block + k;
                const bool in = lnp[(size_t)b * L + l] != 0;
                if (prev[b]) bits += 1;
                else if (in) N[k] = 1;
                if (in) { bits += bbits[b]; body += blen[b]; }
            }
            for (size_t n = 0; n < par.size(); ++n) if (N[n] && par[n] >= 0) N[par[n]] = 1;
            for (size_t n = 0; n < par.size(); ++n) {
                if (A[n]) continue;
                const int32_t p = par[n];
                if (p < 0 || A[p] || N[p]) bits += 1;
                if (N[n]) bits += V[n] - (p < 0 ? 0u : V[p]) + 1;
            }
            ubitn[u] = bits; ubody[u] = body;
        });
        return bounds_decision(l, max_bytes, [&](uint32_t u) { return ubitn[u]; });
    }
    // The bounds test shared by decide / decide_inc.  With S the running size over the packets
    // of layers <= l in progression order (SOP / EPH bytes included) and the last packet's
    // header bytes h_n, the walk passes iff S_(n-1) + [6] + h_n < max_bytes and S_n <= max_bytes
    // (S_n - body_n - [2] = S_(n-1) + [6] + h_n), unless it wraps first (may_hit).
    template <class F> int bounds_decision(uint32_t l, uint64_t max_bytes, F bits_of) {
        ensure_order(l);
        const uint64_t ovh = ((P.p.sop_eph & 2) ? 6 : 0) + ((P.p.sop_eph & 4) ? 2 : 0);
        uint64_t lo = prior + ovh * ord.size(), hi = lo, last_tail = 0;
        clo.resize(chains.size()); chi.resize(chains.size()); cbody.resize(chains.size());
        for (size_t i = 0; i < chains.size(); ++i) {
            uint64_t R = 1, body = 0;
            for (uint32_t u : cunits[i]) { R += bits_of(u); body += ubody[u]; }
            clo[i] = (R + 7) / 8; chi[i] = (R + 6) / 7 + 2; cbody[i] = body;
            lo += clo[i] + body; hi += chi[i] + body;
            if (i == last_chain) last_tail = body + ((P.p.sop_eph & 4) ? 2 : 0);
        }
        if (hi <= max_bytes && hi - last_tail < max_bytes) return 1;
        if (lo > max_bytes || lo - last_tail >= max_bytes) return may_hit(l, max_bytes) ? 0 : -1;
        return 0;
    }
    // decide() from the per-unit sums make_layer_inc keeps (same arithmetic, no pass over blocks)
    int decide_inc(uint32_t l, uint64_t max_bytes) {
        if (max_bytes == 0xffffffffull) return 1;
        for (uint32_t u = 0; u < (uint32_t)units.size(); ++u) { ubitn[u] = ibits[u]; ubody[u] = ibody[u]; }
        return bounds_decision(l, max_bytes, [&](uint32_t u) { return ibits[u]; });
    }

    // ---- incremental bisection (bounds_on layers).  prev[] is fixed while layer l is
    // bisected and every later threshold lies between the interval's two ends, so a block
    // whose reuse test (count_at below) holds at both ends keeps its count to the end of
    // the bisection and leaves the active list.  The rest are recounted per step; a count
    // that changes updates the hash, the block's cached cost and its unit's header bits and
    // body bytes, and - when the block enters or leaves the layer with nothing in packets
    // before - the inclusion tree's per-node counts of such blocks.  A node's count turning
    // non-zero adds its zero-bit-plane bits (V[n] - V[parent] + 1) and one bit for each
    // child with no block in packets (decide()'s two tree terms), and the walk stops at the
    // first ancestor already counting one.  A step is one parallel pass over chunks of a
    // unit's blocks (recount in parallel; the changes applied by each chunk, the tree counts and
    // the unit's sums updated atomically).
    // act: blocks whose count may still change; log: this step's changes (block, old count)
    // mslo / mshi: the largest slo and smallest shi over the chunk's active blocks as the last
    // step that ran it left them (+inf / -inf when some block has no valid interval): a
    // threshold that passes the reuse test against both passes it for every active block
    // (t - s and the comparisons are monotone in s), so the chunk keeps its counts unread
    // (the early steps of a layer, thresholds far above every block's slopes)
    struct alignas(128) ChunkI { uint32_t u, s, e; std::vector<uint32_t> act, log; uint64_t hd; double mslo, mshi; };   // (a line pair each: chunks of one step are written by different threads)
    static uint32_t chunk_blocks() {   // GK_PCRD_CHUNK (tuning)
        static const uint32_t v = getenv("GK_PCRD_CHUNK") ? (uint32_t)atoi(getenv("GK_PCRD_CHUNK")) : 512u;
        return v ? v : 512u;
    }
    std::vector<ChunkI> chunks;
    size_t nact = 0;                             // active blocks over all chunks
    std::vector<std::vector<uint32_t>> tN, tC;   // per tree node: included new blocks below; children with A == 0
    std::vector<uint64_t> ibits, ibody;          // per unit: header bits (tag trees + blocks), body bytes
    std::vector<uint8_t> udirty;                 // per unit: counts changed since it was last coded
    uint64_t lay_hash = 0, prof_act = 0, prof_npar = 0;
    double prof_par_ms = 0, prof_ser_ms = 0;
    // (N[n] is updated atomically: chunks of one unit apply their changes concurrently; a
    // node's count and the bits of its 0 <-> non-zero transitions add up to the same totals in
    // any order)
    void tree_toggle(uint32_t tree, uint32_t k, bool enter, uint64_t& bits) {
        const std::vector<int32_t>& par = incl[tree].parent;
        const std::vector<uint8_t>& A = tA[tree];
        const std::vector<uint32_t>& V = tV[tree];
        const std::vector<uint32_t>& C = tC[tree];
        uint32_t* N = tN[tree].data();
        for (int32_t n = (int32_t)k; n >= 0 && !A[n]; n = par[n]) {
            const uint64_t w = (uint64_t)(V[n] - (par[n] < 0 ? 0u : V[par[n]]) + 1) + C[n];
            if (enter) { if (__atomic_fetch_add(&N[n], 1u, __ATOMIC_RELAXED)) break; bits += w; }
            else { if (__atomic_sub_fetch(&N[n], 1u, __ATOMIC_RELAXED)) break; bits -= w; }
        }
    }
    uint64_t make_layer_inc(uint32_t l, double thresh, double lo, double hi, const std::vector<uint16_t>& prev) {
#ifdef PCRD_TRACE
        fprintf(stderr, "l %u t %.6g [%.6g, %.6g] active %zu\n", l, thresh, lo, hi, nact);
#endif
        auto run_chunk = [&](size_t c) {
            ChunkI& C = chunks[c];
            C.hd = 0;
            if (C.act.empty()) return;
            if (thresh > 0 && thresh - C.mshi < kEps && !(thresh - C.mslo < kEps)) return;
            thread_local std::vector<uint32_t> chg;   // (block, new count) pairs
            chg.clear();
            size_t w = 0;
            const size_t n = C.act.size();
            double mslo = -HUGE_VAL, mshi = HUGE_VAL;
            for (size_t i = 0; i < n; ++i) {
                const uint32_t b = C.act[i];
                // the reuse test holds on an interval: at both ends, for every later threshold
                // (thresholds <= 0 take count_at's special cases)
                if (lo > 0 && reusable(b, lo) && reusable(b, hi)) continue;
                C.act[w++] = b;
                if (passes && i + PF < n) {
                    const uint32_t bp = C.act[i + PF];
                    __builtin_prefetch(passes + info[4 * (size_t)bp + 3] + prev[bp]);
                }
                const uint32_t cur = lnp[(size_t)b * L + l], inc = count_at(b, thresh, prev[b], cur);
                if (inc != prev[b] + cur) { chg.push_back(b); chg.push_back(inc); }
                if (vld[b]) { mslo = std::max(mslo, slo[b]); mshi = std::min(mshi, shi[b]); }
                else { mslo = HUGE_VAL; mshi = -HUGE_VAL; }
            }
            C.act.resize(w);
            if (mslo == HUGE_VAL) mshi = -HUGE_VAL;   // (a block without an interval keeps the chunk live)
            C.mslo = mslo; C.mshi = mshi;
            if (chg.empty()) return;
            const PrecG& PG = unit_prec(units[C.u]);
            // (the unit's sums take this chunk's deltas atomically; blocks, their costs and the
            // journal are the chunk's own)
            uint64_t hd = 0, bits = 0, body = 0;
            for (size_t j = 0; j < chg.size(); j += 2) {
                const uint32_t b = chg[j], inc = chg[j + 1];
                const uint16_t vo = lnp[(size_t)b * L + l], vn = (uint16_t)(inc - prev[b]);
                hd += mix64(((uint64_t)b << 16) | vn) - mix64(((uint64_t)b << 16) | vo);
                C.log.push_back(b); C.log.push_back(vo);
                if (vo) { bits -= bbits[b]; body -= blen[b]; }
                block_cost(b, prev[b], inc);
                if (vn) { bits += bbits[b]; body += blen[b]; }
                lnp[(size_t)b * L + l] = vn;
                if (!prev[b] && (vo == 0) != (vn == 0)) tree_toggle(PG.tree, b - PG.first_block, vn != 0, bits);
            }
            __atomic_fetch_add(&ibits[C.u], bits, __ATOMIC_RELAXED);
            __atomic_fetch_add(&ibody[C.u], body, __ATOMIC_RELAXED);
            __atomic_store_n(&udirty[C.u], (uint8_t)1, __ATOMIC_RELAXED);
            C.hd = hd;
        };
        const auto tp0 = std::chrono::steady_clock::now();
        size_t nwork = 0;   // active blocks of the chunks the reuse test does not skip
        for (const ChunkI& C : chunks)
            if (!(thresh > 0 && thresh - C.mshi < kEps && !(thresh - C.mslo < kEps))) nwork += C.act.size();
        const bool par = nwork >= 2048;
        prof_act += nwork;
        if (par) prun(chunks.size(), run_chunk);
        else for (size_t c = 0; c < chunks.size(); ++c) run_chunk(c);
        const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();
        (par ? prof_par_ms : prof_ser_ms) += dt;
        prof_npar += par;
        nact = 0;
        for (ChunkI& C : chunks) {
            lay_hash += C.hd; nact += C.act.size();
            jlog.insert(jlog.end(), C.log.begin(), C.log.end());
            C.log.clear();
        }
        return lay_hash;
    }
    // the change journal of this layer's bisection: the counts now equal those when the
    // journal held pos entries iff every block changed since has its count from then (the
    // old count of its first change after pos)
    std::vector<uint32_t> jlog, jstamp;
    uint32_t jgen = 0;
    bool same_counts_since(size_t pos, uint32_t l) {
        if (++jgen == 0) { std::fill(jstamp.begin(), jstamp.end(), 0); jgen = 1; }
        for (size_t i = pos; i < jlog.size(); i += 2) {
            const uint32_t b = jlog[i];
            if (jstamp[b] == jgen) continue;
            jstamp[b] = jgen;
            if (lnp[(size_t)b * L + l] != jlog[i + 1]) return false;
        }
        return true;
    }

    // makeLayerSimple (thresh >= 0) / makeLayerFinal (thresh < 0) (TileProcessor.cpp:1367-1515),
    // blocks in parallel.  During one layer's bisection prev[] is fixed, and a block's greedy
    // scan is a chain of comparisons thresh - slope < DBL_EPSILON; the scan (so the count)
    // repeats exactly for every threshold that takes each comparison the same way.  The
    // floating-point difference is monotone in both operands, so that set is
    //   thresh - shi < eps  and  !(thresh - slo < eps)
    // with shi the smallest slope that added passes and slo the largest that did not: the
    // block keeps (slo, shi) and reuses its count while both hold (vld: they are current).
    // Returns a hash of the layer's pass counts (equal counts => equal simulation outcome).
    std::vector<double> slo, shi;
    std::vector<uint8_t> vld;
    static constexpr double kEps = 2.220446049250313e-16;
    static uint64_t mix64(uint64_t x) {
        x += 0x9e3779b97f4a7c15ull;
        x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
        x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
        return x ^ (x >> 31);
    }
    inline bool reusable(uint32_t b, double t) const { return vld[b] && t - shi[b] < kEps && !(t - slo[b] < kEps); }
    // block b's pass count (cumulative) at threshold thresh, p0 passes in before this layer,
    // cur = its current count for the layer (kept while the comparisons repeat)
    inline uint32_t count_at(uint32_t b, double thresh, uint32_t p0, uint32_t cur) {
        const uint32_t np = npasses(b);
        if (thresh < 0) { vld[b] = 0; return std::max<uint32_t>(p0, np); }
        if (thresh == 0) { vld[b] = 0; return np; }
        if (reusable(b, thresh)) return p0 + cur;
        uint32_t inc = p0;
        double lo = -HUGE_VAL, hi = HUGE_VAL;
#ifdef PCRD_TRACE
        g_scans.fetch_add(1, std::memory_order_relaxed); g_scan_passes.fetch_add(np - p0, std::memory_order_relaxed);
#endif
        if (passes && np) {
            // the same arithmetic with the last included pass's rate and distortion in registers
            // (x - 0 == x exactly, so inc == 0 needs no case of its own)
            const GkPass* ps = passes + info[4 * (size_t)b + 3];
            uint32_t rb = p0 ? rate(b, p0 - 1) : 0;
            double db = p0 ? ps[p0 - 1].dist : 0.0;
            for (uint32_t q = p0; q < np; ++q) {
                const uint32_t r = q + 1 == np ? info[4 * (size_t)b + 2] : ps[q].rate;
                const double d = ps[q].dist;
                const uint32_t dr = r - rb;
                const double dd = d - db;
                if (!dr) { if (dd != 0) { inc = q + 1; rb = r; db = d; } continue; }
                const double slope = dd / dr;
                if (thresh - slope < kEps) { inc = q + 1; rb = r; db = d; hi = std::min(hi, slope); }
                else lo = std::max(lo, slope);
            }
            slo[b] = lo; shi[b] = hi; vld[b] = 1;
            return inc;
        }
        for (uint32_t q = p0; q < np; ++q) {
            uint32_t dr; double dd;
            if (inc == 0) { dr = rate(b, q); dd = dist(b, q); }
            else { dr = rate(b, q) - rate(b, inc - 1); dd = dist(b, q) - dist(b, inc - 1); }
            if (!dr) { if (dd != 0) inc = q + 1; continue; }
            const double slope = dd / dr;
            if (thresh - slope < kEps) { inc = q + 1; hi = std::min(hi, slope); }
            else lo = std::max(lo, slope);
        }
        slo[b] = lo; shi[b] = hi; vld[b] = 1;
        return inc;
    }
    void count_state(uint32_t nb) { if (vld.size() != nb) { slo.assign(nb, 0.0); shi.assign(nb, 0.0); vld.assign(nb, 0); } }
    bool bounds = false;      // bisection steps decided by header-size bounds (fast path)
    bool bounds_on = false;   // ... during this layer's bisection (make_layer caches block costs)
    uint64_t make_layer(uint32_t l, double thresh, bool final_attempt, std::vector<uint16_t>& prev) {
        const uint32_t nb = (uint32_t)P.blocks.size();
        const uint32_t chunk = 2048, nch = (b1 - b0 + chunk - 1) / chunk;
        count_state(nb);
        std::vector<uint64_t> hs(nch, 0);
        prun(nch, [&](size_t ci) {
        uint64_t hsum = 0;
        const uint32_t bend = std::min<uint32_t>(b1, b0 + (uint32_t)(ci + 1) * chunk);
        for (uint32_t b = b0 + (uint32_t)ci * chunk; b < bend; ++b) {
            if (passes && b + PF < bend) __builtin_prefetch(passes + info[4 * (size_t)(b + PF) + 3] + prev[b + PF]);
            if (l == 0) prev[b] = 0;
            const uint32_t inc = count_at(b, thresh, prev[b], lnp[(size_t)b * L + l]);
            const uint16_t v = (uint16_t)(inc - prev[b]);
            if (bounds_on && ccount[b] != inc) block_cost(b, prev[b], inc);
            lnp[(size_t)b * L + l] = v;
            hsum += mix64(((uint64_t)b << 16) | v);
            if (final_attempt) { prev[b] = (uint16_t)inc; vld[b] = 0; }
        }
        hs[ci] = hsum;
        });
        uint64_t h = 0;
        for (uint64_t v : hs) h += v;
        return h;
    }

    void allocate(size_t header_size) {
        const uint32_t nb = (uint32_t)P.blocks.size();
        std::vector<uint16_t> prev(nb, 0);
        if (!P.p.rate_control()) {
            for (uint32_t l = 0; l < L; ++l) make_layer(l, -1.0, true, prev);
            return;
        }
        // updateRates: compression ratio -> cumulative byte budget per layer
        double rates[GK_MAX_LAYERS];
        // per tile (CodeStreamCompress.cpp:965-1024): budgets from the tile's pixel count, the header
        // bytes before the first tile shared by area
        if (t1 != t0 + 1) throw GkError("rate control runs on one tile at a time");
        const TileG& TT = P.tiles[t0];
        const double size_pixel = (double)P.nc * P.prec, npix = (double)((uint64_t)(TT.x1 - TT.x0) * (TT.y1 - TT.y0));
        // tile-part generation: 14 bytes (SOT + SOD) per extra part, spread over the layers (the
        // parts of progression order changes do not count: `stride` needs m_enableTilePartGeneration)
        const double tp_offset = P.p.tp_div ? (double)((tile_part_split(P).n - 1) * 14) / (double)L : 0.0;
        for (uint32_t k = 0; k < L; ++k)
            // bits_empty = 8 x component 0's subsampling (updateRates, CodeStreamCompress.cpp:961)
            rates[k] = P.p.rates[k] > 0.0 ? (size_pixel * npix) / (P.p.rates[k] * 8.0 * P.sx(0) * P.sy(0)) - tp_offset : 0.0;
        const double sot_adjust = (npix * (double)header_size) / ((double)P.w * (double)P.h);
        if (rates[0] > 0.0) { rates[0] -= sot_adjust; if (rates[0] < 30.0f) rates[0] = 30.0f; }
        for (uint32_t k = 1; k + 1 < L; ++k)
            if (rates[k] > 0.0) { rates[k] -= sot_adjust; if (rates[k] < rates[k - 1] + 10.0) rates[k] = rates[k - 1] + 20.0; }
        if (L > 1 && rates[L - 1] > 0.0) {
            rates[L - 1] -= (sot_adjust + 2.0);
            if (rates[L - 1] < rates[L - 2] + 10.0) rates[L - 1] = rates[L - 2] + 20.0;
        }
        // slope range over every pass of the tile(s), blocks in parallel chunks
        const auto ta0 = std::chrono::steady_clock::now();
        const uint32_t schunk = 2048, nsch = (b1 - b0 + schunk - 1) / schunk;
        std::vector<double> smin(nsch, 1.7976931348623157e308), smax(nsch, -1);
        prun(nsch, [&](size_t ci) {
            double mn = 1.7976931348623157e308, mx = -1;
            const uint32_t bend = std::min<uint32_t>(b1, b0 + (uint32_t)(ci + 1) * schunk);
            for (uint32_t b = b0 + (uint32_t)ci * schunk; b < bend; ++b)
                for (uint32_t q = 0; q < npasses(b); ++q) {
                    int32_t dr; double dd;
                    if (q == 0) { dr = (int32_t)rate(b, 0); dd = dist(b, 0); }
                    else { dr = (int32_t)(rate(b, q) - rate(b, q - 1)); dd = dist(b, q) - dist(b, q - 1); }
                    if (dr == 0) continue;
                    double sl = dd / dr;
                    if (sl < mn) mn = sl;
                    if (sl > mx) mx = sl;
                }
            smin[ci] = mn; smax[ci] = mx;
        });
        double min_slope = 1.7976931348623157e308, max_slope = -1;
        for (uint32_t ci = 0; ci < nsch; ++ci) { min_slope = std::min(min_slope, smin[ci]); max_slope = std::max(max_slope, smax[ci]); }
        double upper = max_slope;
        // fixed quality (TileProcessor.cpp:1263-1267, 1299-1322): a layer's target is the tile's
        // distortion less maxSE / 10^(PSNR/10), maxSE = sum over components of (2^prec - 1)^2 x
        // the component's code-block area; tile->distortion is the blocks' total distortion
        // decrease summed in block order (T1CompressScheduler::compress, single-threaded order)
        double tile_dist = 0.0, maxSE = 0.0;
        std::vector<double> cum(L, 0.0);
        if (P.p.quality) {
            std::vector<uint64_t> npix(P.nc, 0);
            for (uint32_t b = b0; b < b1; ++b) {
                npix[P.blocks[b].comp] += (uint64_t)P.blocks[b].w * P.blocks[b].h;
                if (npasses(b)) tile_dist += dist(b, npasses(b) - 1);
            }
            const double m = (double)((1ull << P.prec) - 1);
            for (uint32_t c = 0; c < P.nc; ++c) maxSE += m * m * (double)npix[c];
        }
        // a layer's distortion decrease at the current counts, tile->layerDistoration (makeLayerSimple,
        // TileProcessor.cpp:1367-1458), summed in block order; p0 = passes in before the layer
        auto layer_dist = [&](uint32_t l, bool after_final) {
            double ld = 0.0;
            for (uint32_t b = b0; b < b1; ++b) {
                const uint32_t np = lnp[(size_t)b * L + l];
                if (!np) continue;
                const uint32_t p0 = after_final ? prev[b] - np : prev[b];
                ld += p0 ? dist(b, p0 + np - 1) - dist(b, p0 - 1) : dist(b, np - 1);
            }
            return ld;
        };
        const bool fast = t1 == t0 + 1 && !getenv("GK_T2_SERIAL_SIM") && !P.p.quality;
        static const bool prof = getenv("GK_PROFILE") != nullptr;
        using clk = std::chrono::steady_clock;
        auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        double t_make = 0, t_sim = 0, t_prep = 0, t_fin = 0;
        const double t_slopes = msd(ta0, clk::now());
        uint32_t n_it = 0, n_sim = 0;
        if (fast) init_chains();
        static const bool check = getenv("GK_T2_CHECK_SIM") != nullptr;
        // the header-size bounds assume one codeword segment per contribution
        bounds = fast && !getenv("GK_T2_NO_BOUNDS") && !(P.p.cblk_sty & (GK_STY_LAZY | GK_STY_TERMALL));
        uint32_t n_bound = 0;
        for (uint32_t l = 0; l < L; ++l) {
            uint64_t max_len = rates[l] > 0.0f ? (uint64_t)(uint32_t)ceil(rates[l]) : 0xffffffffull;
            bounds_on = bounds && rates[l] > 0.0;
            const double target = P.p.quality ? tile_dist - maxSE / pow(10.0, P.p.dist[l] / 10.0) : 0.0;
            if (bounds_on) {
                const auto tp = clk::now();
                count_state(nb);
                bounds_prep(l, prev);
                t_prep += msd(tp, clk::now());
            }
            if (P.p.layer_rc(l)) {
                double lower = min_slope, prevthresh = -1, thresh = 0;
                // pass counts equal to those at an end of the bisection interval give that end's
                // outcome (the simulation depends on nothing else): the simulation is skipped
                bool has_lo = false, has_hi = false;
                Swallow sw_hi;
                uint64_t h_lo = 0, h_hi = 0;
                size_t j_lo = 0, j_hi = 0;   // journal positions of the counts at lower / upper
                // the hash only nominates a match: the layer's pass counts are compared exactly
                std::vector<uint16_t> c_lo, c_hi, c_now;
                auto counts = [&](std::vector<uint16_t>& v) {
                    v.resize(b1 - b0);
                    for (uint32_t b = b0; b < b1; ++b) v[b - b0] = lnp[(size_t)b * L + l];
                };
                for (uint32_t it = 0; it < 128; ++it) {
                    thresh = (upper == -1) ? lower : (lower + upper) / 2;
                    const auto t0 = clk::now();
                    // every later threshold lies between lower and upper (just lower while upper is unset)
                    const double hu = upper == -1 ? lower : upper;
                    const uint64_t h = bounds_on ? make_layer_inc(l, thresh, std::min(lower, hu), std::max(lower, hu), prev)
                                                 : make_layer(l, thresh, false, prev);
                    const auto t1 = clk::now();
                    t_make += msd(t0, t1);
                    ++n_it;
                    if (prevthresh != -1 && fabs(prevthresh - thresh) < 0.001) break;
                    prevthresh = thresh;
                    bool ok;
                    Swallow sw_now;   // a fit through a swallowed failure (Swallow)
                    // (bounds_on: the exact compare from the change journal, no count copies)
                    auto same = [&](const std::vector<uint16_t>& c, size_t pos) {
                        if (bounds_on) return same_counts_since(pos, l);
                        counts(c_now);
                        return c_now == c;
                    };
                    if (has_hi && h == h_hi && same(c_hi, j_hi)) { ok = true; sw_now = sw_hi; }
                    else if (has_lo && h == h_lo && same(c_lo, j_lo)) ok = false;
                    else if (P.p.quality) {
                        // below the target: upperBound = thresh (TileProcessor.cpp:1311-1322)
                        const double ld = layer_dist(l, false);
                        ok = (l == 0 ? ld : cum[l - 1] + ld) < target;
                    } else {
                        int d = bounds_on ? decide_inc(l, max_len) : 0;
                        if (bounds_on && check) {   // debug: the incremental sums must equal a full pass
                            const std::vector<uint64_t> b0v = ubitn, b1v = ubody;
                            if (decide(l, max_len, prev) != d || ubitn != b0v || ubody != b1v)
                                throw GkError("rate-control bounds: incremental layer sums differ");
                        }
                        if (d && !check) { ok = d > 0; ++n_bound; }
                        else {
                            skip_clean = bounds_on;
                            ok = fast ? simulate_layer(l, max_len, &sw_now) : simulate(l + 1, max_len, &sw_now);
                            skip_clean = false;
                            ++n_sim;
                            if (bounds_on && check && max_len != 0xffffffffull) {
                                for (size_t i = 0; i < chains.size(); ++i)
                                    if (chdr[i] < clo[i] || chdr[i] > chi[i] || csize[i] - chdr[i] != cbody[i])
                                        throw GkError("rate-control bounds: packet size outside its bounds");
                                if (d && ok != (d > 0)) throw GkError("rate-control bounds: decision differs from the simulation");
                            }
                        }
                        t_sim += msd(t1, clk::now());
                    }
                    if (!ok) {
                        lower = thresh; h_lo = h; has_lo = true;
                        if (bounds_on) j_lo = jlog.size(); else counts(c_lo);
                        continue;
                    }
                    upper = thresh; h_hi = h; has_hi = true; sw_hi = sw_now;
                    if (bounds_on) j_hi = jlog.size(); else counts(c_hi);
                }
                // the final simulation (all layers, this layer's budget when it is the last)
                // replays the step that set upper; without one it runs here
                if (l + 1 == L) {
                    if (has_hi) final_sw = sw_hi;
                    else final_sw_pending = true;
                }
                const double fin = upper == -1 ? thresh : upper;
                if (bounds_on) {   // incrementally too (fin is an end of the interval), then final
                    const double hu = upper == -1 ? lower : upper;
                    const auto tm = clk::now();
                    make_layer_inc(l, fin, std::min(lower, hu), std::max(lower, hu), prev);
                    for (uint32_t b = b0; b < b1; ++b) { prev[b] = (uint16_t)(prev[b] + lnp[(size_t)b * L + l]); vld[b] = 0; }
                    t_make += msd(tm, clk::now());
                } else make_layer(l, fin, true, prev);
                if (P.p.quality) { const double ld = layer_dist(l, true); cum[l] = l == 0 ? ld : cum[l - 1] + ld; }
                upper = lower - 1;
            } else {
                make_layer(l, -1.0, true, prev);
            }
            if (fast && l + 1 < L) {
                const auto tf = clk::now();
                skip_clean = bounds_on;   // units coded at these counts keep their bits and state
                finish_layer(l);
                skip_clean = false;
                t_fin += msd(tf, clk::now());
            }
            bounds_on = false;
        }
        if (final_sw_pending) {   // (the coding state is not needed after allocate: packets restart it)
            const uint64_t last = rates[L - 1] > 0.0f ? (uint64_t)(uint32_t)ceil(rates[L - 1]) : 0xffffffffull;
            simulate(L, last, &final_sw);
        }
        if (prof)
            fprintf(stderr, "pcrd: %u bisection steps, %u simulated, %u decided by bounds; make_layer %.2f ms, simulation %.2f ms, bounds setup %.2f ms, "
                    "slope range %.2f ms, layer snapshots %.2f ms; %llu block recounts, %llu parallel steps %.2f ms, serial %.2f ms\n",
                    n_it, n_sim, n_bound, t_make, t_sim, t_prep, t_slopes, t_fin,
                    (unsigned long long)prof_act, (unsigned long long)prof_npar, prof_par_ms, prof_ser_ms);
        if (prof)
            fprintf(stderr, "pcrd code_layer: units %.2f ms, packet lengths %.2f ms (%zu units, %zu packets)\n",
                    prof_code / 1e3, prof_stuff / 1e3, units.size(), chains.size());
    }
};

static void put16(std::vector<uint8_t>& o, uint32_t v) { o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v); }
static void put32(std::vector<uint8_t>& o, uint32_t v) { put16(o, v >> 16); put16(o, v & 0xffff); }

// POC marker (A.6.6, CodeStreamCompress::writePoc :1278-1340): per entry RSpoc, CSpoc (1 or 2
// bytes), LYEpoc (2), REpoc, CEpoc (1 or 2), Ppoc.  clamp (a tile-part POC): layers /
// resolutions / components clamped to the tile's, as the main header's writePoc leaves them,
// and every progression replaced by *clamp (see build_tile_part) unless it is ~0u.
static void write_poc(std::vector<uint8_t>& o, const std::vector<Poc>& pocs, uint32_t nc, const Plan* clamp,
                      uint32_t prog = ~0u) {
    const uint32_t cw = nc <= 256 ? 1 : 2;
    put16(o, 0xff5f); put16(o, 2 + (uint32_t)pocs.size() * (5 + 2 * cw));
    for (Poc e : pocs) {
        if (clamp) {
            e.lye = std::min(e.lye, clamp->p.nlayers); e.re = std::min(e.re, clamp->p.numres); e.ce = std::min(e.ce, nc);
            if (prog != ~0u) e.prog = prog;
        }
        o.push_back((uint8_t)e.rs);
        if (cw == 1) o.push_back((uint8_t)e.cs); else put16(o, e.cs);
        put16(o, e.lye);
        o.push_back((uint8_t)e.re);
        if (cw == 1) o.push_back((uint8_t)e.ce); else put16(o, e.ce);
        o.push_back((uint8_t)e.prog);
    }
}

// Main header: SOC SIZ [CAP] COD QCD [TLM] [POC] [RGN] [COM]  (CodeStreamCompress::init_header_writing
// :822-860; marker writers :1054-1685)
static void write_main_header(std::vector<uint8_t>& o, const Plan& P, size_t* tlm_pos = nullptr) {
    put16(o, 0xff4f);
    put16(o, 0xff51); put16(o, 38 + 3 * P.nc);
    put16(o, P.p.ht() ? 0x4000 : 0);   // Rsiz: GRK_JPH_RSIZ_FLAG for HT (CodeStreamCompress.cpp:216-219)
    put32(o, P.x0 + P.w); put32(o, P.y0 + P.h); put32(o, P.x0); put32(o, P.y0);   // Xsiz Ysiz XOsiz YOsiz
    put32(o, P.p.tw ? P.p.tw : P.x0 + P.w - P.gx0); put32(o, P.p.th ? P.p.th : P.y0 + P.h - P.gy0);
    put32(o, P.gx0); put32(o, P.gy0);                                              // XTsiz YTsiz XTOsiz YTOsiz
    put16(o, P.nc);
    for (uint32_t i = 0; i < P.nc; ++i) {   // Ssiz, XRsiz, YRsiz
        o.push_back((uint8_t)((P.prec - 1) | (P.sgnd ? 0x80 : 0)));
        o.push_back((uint8_t)P.sx(i)); o.push_back((uint8_t)P.sy(i));
    }
    if (P.p.ht()) {   // CAP (CodeStreamCompress::write_cap :1064-1111): Pcap bit 15, Ccap = MAGBp code
        uint32_t B = 0;
        // param_qcd::get_MAGBp (HTParams.cpp:318-336): scalar expounded bands count from their
        // decomposition level (LL: num_decomps), in unsigned arithmetic as there
        for (uint32_t r = 0; r < P.p.numres; ++r)
            for (auto& Bd : P.tiles[0].comps[0].res[r].bands) {
                const uint32_t nb = P.p.irrev ? (P.p.numres - 1) - (r ? r - 1 : 0) : 1u;
                B = std::max(B, Bd.expn + P.p.numgbits - nb);
            }
        // an ROI upshift adds its bit-planes to the coded magnitudes (15444-15 A.2: MAGBp bounds
        // them; Grok's encoder never applies the shift to HT blocks)
        uint32_t rmax = 0;
        for (uint32_t c = 0; c < P.nc; ++c) rmax = std::max(rmax, P.p.roi(c));
        B += rmax;
        uint32_t Bp = B <= 8 ? 0 : B < 28 ? B - 8 : B < 48 ? 13 + (B >> 2) : 31;
        put16(o, 0xff50); put16(o, 8); put32(o, 0x00020000); put16(o, (P.p.irrev ? 0x20 : 0) | Bp);
    }
    put16(o, 0xff52); put16(o, 12 + (P.p.custom_prc ? P.p.numres : 0));
    o.push_back((uint8_t)((P.p.custom_prc ? 1 : 0) | P.p.sop_eph));   // Scod: precincts, SOP, EPH
    o.push_back((uint8_t)P.p.prog);   // progression order
    put16(o, P.p.nlayers);
    o.push_back((uint8_t)((P.p.mct && P.nc >= 3) ? 1 : 0));
    o.push_back((uint8_t)(P.p.numres - 1));
    o.push_back((uint8_t)(P.p.cbw - 2)); o.push_back((uint8_t)(P.p.cbh - 2));
    o.push_back((uint8_t)P.p.cblk_sty);
    o.push_back(P.p.irrev ? 0 : 1);
    if (P.p.custom_prc) for (uint32_t r = 0; r < P.p.numres; ++r) o.push_back((uint8_t)(P.p.prcw[r] | (P.p.prch[r] << 4)));
    uint32_t nbands = 3 * P.p.numres - 2;
    put16(o, 0xff5c);
    const CompG& C = P.tiles[0].comps[0];
    if (!P.p.irrev) {
        put16(o, 3 + nbands);
        o.push_back((uint8_t)(P.p.numgbits << 5));
        for (uint32_t r = 0; r < P.p.numres; ++r) for (auto& B : C.res[r].bands) o.push_back((uint8_t)(B.expn << 3));
    } else {
        put16(o, 3 + 2 * nbands);
        o.push_back((uint8_t)((P.p.numgbits << 5) | 2));
        for (uint32_t r = 0; r < P.p.numres; ++r) for (auto& B : C.res[r].bands) put16(o, (B.expn << 11) | B.mant);
    }
    if (P.p.tlm) {   // TLM placeholder (TileLengthMarkers::writeBegin, LengthCache.cpp:437-463): Stlm 0x60,
                     // 6 bytes (Ttlm u16, Ptlm u32) per tile part, filled in after the tiles are written
        const uint32_t nt = (uint32_t)P.tiles.size();
        if (4 + 6 * (size_t)nt > 65535) throw GkError("too many tiles for one TLM marker");
        const uint64_t ne = (uint64_t)nt * tile_part_split(P).n;   // one entry per tile part
        if (4 + 6 * ne > 65535) throw GkError("TLM marker overflow (too many tile parts)");
        put16(o, 0xff55); put16(o, (uint32_t)(4 + 6 * ne)); o.push_back(0); o.push_back(0x60);
        if (tlm_pos) *tlm_pos = o.size();
        o.insert(o.end(), (size_t)(6 * ne), 0);
    }
    // POC of tile 0 in the main header (init_header_writing :839-840), entries as given: writePoc
    // (:1278-1340) writes each before clamping it to the tile's layers / resolutions / components
    if (!P.p.pocs.empty()) write_poc(o, P.p.pocs, P.nc, nullptr);
    for (uint32_t c = 0; c < P.nc; ++c)   // RGN (CodeStreamCompress::write_regions / write_rgn :746-780, 1397-1410)
        if (P.p.roi(c)) {
            const uint32_t cw = P.nc <= 256 ? 1 : 2;
            put16(o, 0xff5e); put16(o, 4 + cw);
            if (cw == 1) o.push_back((uint8_t)c); else put16(o, c);
            o.push_back(0);   // Srgn: implicit (maxshift)
            o.push_back((uint8_t)P.p.roi(c));
        }
    if (!P.p.comments.empty()) {   // (CodeStreamCompress::write_com :1114-1145)
        for (const auto& c : P.p.comments) {
            put16(o, 0xff64); put16(o, 4 + (uint32_t)c.second.size()); put16(o, c.first);
            o.insert(o.end(), c.second.begin(), c.second.end());
        }
    } else if (P.p.write_com) {
        const char* txt = "Created by Grok     version 9.2.0";
        put16(o, 0xff64); put16(o, 4 + (uint32_t)strlen(txt)); put16(o, 1);
        o.insert(o.end(), txt, txt + strlen(txt));
    }
}

// ---------------------------------------------------------------------------
// JP2 file format (ISO 15444-1 Annex I): the boxes Grok writes around the codestream
// (FileFormatCompress.cpp:43-265, 619-665, 936-953) and the box walk that finds it
// (FileFormatDecompress.cpp:632-672).  No colour conversion is applied (sRGB / greyscale
// enumerated spaces, as grk_compress records for PNM input, PNMFormat.cpp:439-442).
// ---------------------------------------------------------------------------
static const uint32_t BOX_JP = 0x6a502020, BOX_FTYP = 0x66747970, BOX_JP2H = 0x6a703268, BOX_IHDR = 0x69686472,
                      BOX_COLR = 0x636f6c72, BOX_JP2C = 0x6a703263, BRAND_JP2 = 0x6a703220;
// FileFormatCompress::startCompress: the jp2c box carries an 8-byte XLBox when the raw image
// exceeds 2^30 bytes (the codestream may pass 4 GiB)
static bool jp2_needs_xl(const Plan& P) {
    return (uint64_t)P.nc * P.w * P.h * ((P.prec + 7) / 8) > (1ull << 30);
}
static size_t jp2_prefix_size(const Plan& P) { return 12 + 20 + 45 + (jp2_needs_xl(P) ? 16 : 8); }
// signature, file type, JP2 header (ihdr + colr) and the jp2c box header for a codestream of cs_len bytes
static void write_jp2_prefix(std::vector<uint8_t>& o, const Plan& P, uint64_t cs_len) {
    put32(o, 12); put32(o, BOX_JP); put32(o, 0x0d0a870a);
    put32(o, 20); put32(o, BOX_FTYP); put32(o, BRAND_JP2); put32(o, 0); put32(o, BRAND_JP2);
    put32(o, 8 + 22 + 15); put32(o, BOX_JP2H);
    put32(o, 22); put32(o, BOX_IHDR); put32(o, P.h); put32(o, P.w); put16(o, P.nc);
    o.push_back((uint8_t)((P.prec - 1) | (P.sgnd ? 0x80 : 0)));   // BPC (one precision for all components)
    o.push_back(7); o.push_back(0); o.push_back(0);                 // C = 7, UnkC = 0, IPR = 0
    put32(o, 15); put32(o, BOX_COLR); o.push_back(1); o.push_back(0); o.push_back(0);   // METH 1, PREC, APPROX
    put32(o, P.nc < 3 ? 17 : 16);                                   // EnumCS: greyscale / sRGB
    if (jp2_needs_xl(P)) {
        put32(o, 1); put32(o, BOX_JP2C); put32(o, (uint32_t)((cs_len + 16) >> 32)); put32(o, (uint32_t)(cs_len + 16));
    } else {
        const uint64_t L = cs_len + 8;
        put32(o, L < (1ull << 32) ? (uint32_t)L : 0); put32(o, BOX_JP2C);
    }
}
// JP2 file -> [off, off + len) of its contiguous codestream box; false for a raw codestream
static bool jp2_locate(ByteSrc& S, size_t& off, size_t& len) {
    if (S.len < 12 || S.be32(0) != 12 || S.be32(4) != BOX_JP) return false;
    if (S.be32(8) != 0x0d0a870a) throw GkError("corrupt JP2 signature box");
    size_t pos = 12;
    bool ftyp = false;
    while (pos + 8 <= S.len) {
        uint64_t L = S.be32(pos);
        const uint32_t T = S.be32(pos + 4);
        size_t hdr = 8;
        if (L == 1) {
            if (pos + 16 > S.len) throw GkError("corrupt JP2 box header");
            L = ((uint64_t)S.be32(pos + 8) << 32) | S.be32(pos + 12);
            hdr = 16;
        } else if (L == 0) {
            L = S.len - pos;   // last box
        }
        if (L < hdr || L > S.len - pos) throw GkError("corrupt JP2 box length");
        if (!ftyp && T != BOX_FTYP) throw GkError("malformed JP2: second box must be the file type box");
        ftyp = true;
        if (T == BOX_JP2C) { off = pos + hdr; len = (size_t)L - hdr; return true; }
        pos += (size_t)L;
    }
    throw GkError("JP2 file without a contiguous codestream box");
}

}  // namespace

// ---------------------------------------------------------------------------
// Context
// ---------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr; size_t cap = 0;
    void* get(size_t n) {
        if (n > cap) {
            if (p) (void)hipFree(p);
            p = nullptr; cap = 0;
            size_t c = std::max(n, (size_t)1 << 20);
            HIPCHK(hipMalloc(&p, c));
            cap = c;
        }
        return p;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};
struct HostBuf {
    void* p = nullptr; size_t cap = 0;
    void* get(size_t n) {
        if (n > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr; cap = 0;
            size_t c = std::max(n, (size_t)1 << 20);
            HIPCHK(hipHostMalloc(&p, c, 0));
            cap = c;
        }
        return p;
    }
    ~HostBuf() { if (p) (void)hipHostFree(p); }
};

struct gk_ctx {
    uint32_t dec_layers = 0;   // quality layers to decode (0 = all; grk_dparameters::cp_layer)
    // the decode in progress has a window: Grok then takes its partial-tile inverse
    // (CodeStreamDecompress.cpp:389, WaveletReverse.cpp:2237-2246), whose 5/3 single odd sample
    // across is H >> 1 (:1551-1554) where the whole-tile path has H / 2 (:583)
    bool dwt_partial = false;
    uint32_t dec_reduce = 0;   // highest resolutions discarded on decode (grk_dparameters::cp_reduce)
    bool win_whole_tile = false;   // gk_set_window_rule: windows keep the whole-tile inverse DWT rule
    int device = 0;
    bool registered = false;   // counted in g_dev_engines
    hipStream_t st = nullptr;
    hipStream_t aux[3] = {nullptr, nullptr, nullptr};   // encode T1: MQ chunks overlapping context modelling
    hipEvent_t xev[6];
    std::string err;
    gk_timings tm{};
    // cached plan
    std::string plan_key;
    Plan plan;
    // device buffers
    DevBuf arena;       // int32 work planes: nc * 2 * plane_elems
    DevBuf bytes;       // encode slots + header staging / decode staging
    DevBuf dblocks;     // GkBlock table
    DevBuf dpasses;     // GkPass per block
    DevBuf dinfo;       // 3 u32 per block
    DevBuf dseg;        // gather segments
    DevBuf dout;        // codestream (encode, when the caller wants host bytes) / input (decode from host)
    DevBuf dplanes;     // component planes staged from host
    DevBuf derr;
    DevBuf dsym, dsymoff, dpassend, dcminfo;
    DevBuf dmsstate, dseglen;      // mode-switch T1 state slabs, decode segment lengths
    DevBuf dscratch, dnmse, dord, dweight, dord_enc;
    HostBuf hinfo, hseg, hhdr, hpasses, hord, hweight, hord_enc;
    DevBuf dstage1, dstage2;   // decode: batched tile-part / packet header fetches (device input)
    HostBuf hstage1, hstage2;
    int16_t* nmse_tab = nullptr;   // device copy of the nmsedec tables (4 x 128)
    hipEvent_t ev[32];
    bool blocks_uploaded = false;
    uint32_t enc_b0 = 0, enc_b1 = 0;   // block range of the uploaded encode table
    std::vector<uint8_t> enc_dx, enc_dy;   // gk_set_subsampling: the next encodes' component subsampling
    std::vector<uint32_t> hdr_dx, hdr_dy, hdr_prec, hdr_sgnd;   // the last gk_decode_header's components
    bool enc_rc = false;                // its rate-control flag (GkBlock::flags bit 1)
    // band quantisation held by the cached plan's bands: the plan's own (encoder, native_qcd)
    // or that of the last decoded stream (band_qcd)
    std::vector<std::pair<uint32_t, uint32_t>> native_qcd, band_qcd;
    // results of the last gk_encode_blocks
    std::vector<gk_band_result> rb_bands;
    std::vector<gk_block_result> rb_blocks;
    std::vector<gk_pass_result> rb_passes;
    std::vector<uint8_t> rb_data;
};

static void set_params(Params& P, const gk_cparameters* cp, uint32_t nc) {
    for (int i = 0; i < GK_MAXRLVLS; ++i) { P.prcw[i] = 15; P.prch[i] = 15; }
    if (!cp) return;
    // CodeStreamCompress.cpp:159: 1..33 resolutions; res_spec indexes the 33-entry precinct arrays
    if (cp->numresolution > GK_MAXRLVLS) throw GkError("numresolution must be at most 33");
    if (cp->res_spec > GK_MAXRLVLS) throw GkError("res_spec must be at most 33");
    P.numres = cp->numresolution ? cp->numresolution : 6;
    P.cbw = (uint32_t)floorlog2(cp->cblockw_init ? cp->cblockw_init : 64);
    P.cbh = (uint32_t)floorlog2(cp->cblockh_init ? cp->cblockh_init : 64);
    P.irrev = cp->irreversible ? 1 : 0;
    P.mct = cp->mct;
    P.numgbits = cp->numgbits ? cp->numgbits : 2;
    P.nlayers = cp->numlayers ? cp->numlayers : 1;
    if (P.nlayers > GK_MAX_LAYERS) P.nlayers = GK_MAX_LAYERS;
    // a tile takes the PSNR targets under allocationByQuality, the compression ratios otherwise
    // (CodeStreamCompress.cpp:387-393)
    P.quality = cp->allocationByQuality != 0;
    for (uint32_t l = 0; l < GK_MAX_LAYERS; ++l) {
        P.rates[l] = (l < P.nlayers && !P.quality && cp->layer_rate[l] > 0.0) ? cp->layer_rate[l] : 0.0;
        P.dist[l] = (l < P.nlayers && P.quality && cp->layer_distortion[l] > 0.0) ? cp->layer_distortion[l] : 0.0;
    }
    if (cp->csty & ~7u) throw GkError("unknown coding style bits (csty)");
    P.sop_eph = cp->csty & 6u;
    P.write_com = cp->write_comment;
    // caller comments (CodeStreamCompress.cpp:303-330): entry i is kept when non-empty and not longer
    // than GRK_MAX_COMMENT_LENGTH; write_com then writes entries 0 .. kept - 1 that are valid (an
    // entry skipped early shifts the count, as there).  Lengths that overflow Lcom are refused.
    P.comments.clear();
    if (cp->num_comments > GK_NUM_COMMENTS) throw GkError("at most 256 comments");
    uint32_t kept = 0;
    for (uint32_t i = 0; i < cp->num_comments; ++i)
        if (cp->comment_len[i] && cp->comment[i]) ++kept;
    for (uint32_t i = 0; i < kept; ++i) {
        if (!cp->comment_len[i] || !cp->comment[i]) continue;
        if (cp->comment_len[i] > 65531) throw GkError("comment longer than a COM marker holds (65531 bytes)");
        P.comments.push_back({cp->is_binary_comment[i] ? 0u : 1u, std::string(cp->comment[i], cp->comment_len[i])});
    }
    P.cblk_sty = cp->cblk_sty;
    if (cp->prog_order < 0 || cp->prog_order > 4) throw GkError("unknown progression order");
    P.prog = (uint32_t)cp->prog_order;
    P.roishift.clear();
    // CodeStreamCompress.cpp:538-541: roishift on the component whose index equals roi_compno;
    // an index past the last component matches none (no ROI), as in Grok
    if (cp->roi_compno >= 0 && (uint32_t)cp->roi_compno < nc && cp->roi_shift) {
        if (cp->roi_shift >= 32) throw GkError("ROI shift must be below 32");
        P.roishift.assign(nc, 0);
        P.roishift[(size_t)cp->roi_compno] = (uint8_t)cp->roi_shift;
    }
    if (cp->numpocs > 32) throw GkError("at most 32 progression order changes");
    P.pocs.clear();
    for (uint32_t i = 0; i < cp->numpocs; ++i) {
        const gk_poc& g = cp->pocs[i];
        if (g.prog < 0 || g.prog > 4 || g.resE > GK_MAXRLVLS || g.resS >= g.resE || g.compS >= g.compE || !g.layE ||
            g.layE > 65535 || g.compE > 16384)
            throw GkError("bad progression order change");
        Poc e; e.rs = g.resS; e.cs = g.compS; e.lye = g.layE; e.re = g.resE; e.ce = g.compE; e.prog = (uint32_t)g.prog;
        P.pocs.push_back(e);
    }
    P.tp_div = cp->enableTilePartGeneration ? cp->newTilePartProgressionDivider : 0;
    if (P.tp_div && P.tp_div != 'L' && P.tp_div != 'R' && P.tp_div != 'C')
        throw GkError("tile-part divider must be L, R or C");
    if (cp->tile_size_on) {
        if (!cp->t_width || !cp->t_height) throw GkError("tile size must be non-zero when tiling is on");
        P.tw = cp->t_width; P.th = cp->t_height;
    }
    P.tlm = cp->writeTLM != 0; P.plt = cp->writePLT != 0;
    if (cp->cod_format != 0 && cp->cod_format != 2) throw GkError("cod_format must be GRK_CODEC_J2K (0) or GRK_CODEC_JP2 (2)");
    P.jp2 = cp->cod_format == 2;
    if ((cp->csty & 1) && cp->res_spec) {   // CodeStreamCompress.cpp:542-590
        P.custom_prc = true;
        uint32_t p = 0;
        for (int r = (int)P.numres - 1; r >= 0; --r, ++p) {
            uint32_t pw, ph;
            if (p < cp->res_spec) { pw = cp->prcw_init[p]; ph = cp->prch_init[p]; }
            else {
                pw = cp->prcw_init[cp->res_spec - 1] >> (p - (cp->res_spec - 1));
                ph = cp->prch_init[cp->res_spec - 1] >> (p - (cp->res_spec - 1));
            }
            P.prcw[r] = pw < 1 ? 1 : (uint32_t)floorlog2(pw);
            P.prch[r] = ph < 1 ? 1 : (uint32_t)floorlog2(ph);
            // a size of exactly 1 gives exponent 0: legal at resolution 0 (1 x 1 code-blocks),
            // without a band partition (B.6: PPx - 1) above it
            if (r > 0 && (!P.prcw[r] || !P.prch[r]))
                throw GkError("precinct size 1 above resolution 0 (exponent 0 has no band partition)");
        }
    }
}

// CodeStreamCompress::validateProgressionOrders (CodeStreamCompress.cpp:1685-1747): the POC
// entries, clamped to the stream's layers / resolutions / components, must cover every
// (layer, resolution, component); a list that leaves a packet out is refused ("POC: missing
// packets") rather than dropping its code-blocks from the codestream.
static void check_poc_coverage(const Params& P, uint32_t nc) {
    if (P.pocs.empty()) return;
    const uint32_t L = P.nlayers, R = P.numres;
    std::vector<uint8_t> seen((size_t)L * R * nc, 0);
    for (const Poc& q : P.pocs)
        for (uint32_t r = q.rs; r < std::min(q.re, R); ++r)
            for (uint32_t c = q.cs; c < std::min(q.ce, nc); ++c)
                for (uint32_t l = 0; l < std::min(q.lye, L); ++l) seen[((size_t)l * R + r) * nc + c] = 1;
    for (uint8_t v : seen)
        if (!v) throw GkError("POC: missing packets (the progression order changes do not cover every packet)");
}

static std::string plan_key(const Plan& P) {
    char buf[256];
    snprintf(buf, sizeof buf, "%u %u %u %u %u %u %u %u %u %u %u %u", P.w, P.h, P.nc, P.prec, P.sgnd, P.p.numres, P.p.cbw,
             P.p.cbh, P.p.irrev, P.p.mct, P.p.numgbits, P.p.custom_prc ? 1 : 0);
    std::string k(buf);
    if (P.subsampled())
        for (uint32_t c = 0; c < P.nc; ++c) k += " s" + std::to_string(P.sx(c)) + "x" + std::to_string(P.sy(c));
    for (size_t c = 0; c < P.cprec.size(); ++c) k += " p" + std::to_string(P.cprec[c]) + (P.csgnd[c] ? "s" : "u");
    k += " sty" + std::to_string(P.p.cblk_sty) + " t" + std::to_string(P.p.tw) + "x" + std::to_string(P.p.th);
    k += " o" + std::to_string(P.x0) + "," + std::to_string(P.y0) + "," + std::to_string(P.gx0) + "," + std::to_string(P.gy0);
    for (size_t c = 0; c < P.p.roishift.size(); ++c)   // non-zero (component, shift) pairs only
        if (P.p.roishift[c]) k += " roi" + std::to_string(c) + ":" + std::to_string(P.p.roishift[c]);
    for (uint32_t r = 0; r < P.p.numres; ++r) k += " " + std::to_string(P.p.prcw[r]) + "," + std::to_string(P.p.prch[r]);
    for (const Params::CompCod& q : P.p.cc) {   // COC: every component's coding
        k += " coc" + std::to_string(q.numres) + "," + std::to_string(q.cbw) + "," + std::to_string(q.cbh) + "," +
             std::to_string(q.cblk_sty) + "," + std::to_string(q.irrev);
        for (uint32_t r = 0; r < q.numres; ++r) k += ":" + std::to_string(q.prcw[r]) + "," + std::to_string(q.prch[r]);
    }
    return k;
}

static void ensure_plan(gk_ctx* ctx, const Plan& want) {
    std::string k = plan_key(want);
    if (k == ctx->plan_key) {
        // same geometry: refresh the parameters that do not shape the plan (layers, rates,
        // TLM/PLT, COM), which the cached plan would otherwise carry over from the last call
        ctx->plan.p = want.p;
        return;
    }
    ctx->plan = want;
    build_plan(ctx->plan);
    ctx->plan_key = k;
    ctx->blocks_uploaded = false;
    ctx->native_qcd.clear();
    for (const CompG& C : ctx->plan.tiles[0].comps) {
        ctx->native_qcd.push_back({ctx->plan.p.numgbits, ~0u});
        for (const ResG& R : C.res)
            for (const BandG& B : R.bands) ctx->native_qcd.push_back({B.expn, B.mant});
    }
    ctx->band_qcd = ctx->native_qcd;
}
// Encode uses the plan's own quantisation: undo a decoded stream's QCD if one was applied.
static void restore_native_qcd(gk_ctx* ctx) {
    if (ctx->band_qcd == ctx->native_qcd) return;
    for (TileG& T : ctx->plan.tiles) assign_steps_tile(ctx->plan, T);
    ctx->band_qcd = ctx->native_qcd;
}

// Level 1 fused with the sample stage: the caller's planes (sample type stype) are read by the
// first forward level through the DC shift (+ RCT / ICT for the first three components when
// mct3) and written by the last inverse level through the inverse MCT, DC shift and clamp, only
// inside the window (region coordinates; planes[c] addresses the window origin).
struct L1Io {
    int stype = GK_S32;
    bool mct3 = false;
    std::vector<const void*> planes;     // component c's plane at its output rectangle's origin
    std::vector<uint32_t> strides;
    std::vector<int32_t> shift, mn, mx;  // per component: DC shift, clamp range (its precision)
    uint32_t cx0 = 0, cy0 = 0, cx1 = 0, cy1 = 0;   // inverse: the output rectangle on the canvas
};

// Forward/inverse DWT over all components with the ping-pong placement of gk_common.h; every
// level is one launch per tile shape with the components in grid.z.
// lstop (inverse only): the last level undone (1 = full resolution; reduced-resolution decode
// stops at reduce + 1, leaving resolution numres - 1 - reduce at the tiles' corners)
static void run_dwt(gk_ctx* ctx, const Region& RG, bool forward, uint32_t jb = 0, uint32_t je = 0xffffffffu,
                    uint32_t ib = 0, uint32_t ie = 0xffffffffu, const L1Io* io = nullptr, uint32_t lstop = 1) {
    Plan& P = ctx->plan;
    int32_t* arena = (int32_t*)ctx->arena.p;
    const uint64_t cst = 2 * (uint64_t)RG.plane;   // component plane pairs
    ctx->tm.dwt_launches = 0; ctx->tm.dwt_bytes = 0;
    // per group (sampling grid, levels and transform; one group without subsampling or COC), level
    // by level, one launch per run of its components and tile class
    for (const SGroup& G : P.groups) {
    const uint32_t L = G.numres - 1;
    const uint32_t irrev = G.irrev;
    const Region RGg = group_region(P, RG, G);
    const uint32_t nlev = forward ? L : (L + 1 > lstop ? L + 1 - lstop : 0);
    for (uint32_t i = 0; i < nlev; ++i) {
        uint32_t l = forward ? i + 1 : L - i;     // level being (un)done
        for (const auto& run : G.runs)
        for (const ShapeG& S0 : G.shapes) {       // one launch per tile class, grid.z = its tiles
            const uint32_t c0 = run.first, ncr = run.second - run.first;
            int32_t* const base = arena + (size_t)c0 * cst;   // component c0's plane pair
            ShapeG S = S0;                        // restricted to tile rows [jb, je), columns [ib, ie)
            // members k of the class: tile column ci + k si; those in [ib, ie) are k in [k0, k1)
            auto krange = [](uint64_t c, uint64_t st, uint32_t n, uint64_t b, uint64_t e, uint32_t& k0, uint32_t& k1) {
                k0 = (uint32_t)std::min<uint64_t>(n, b > c ? (b - c + st - 1) / st : 0);
                k1 = (uint32_t)(e > c ? std::min<uint64_t>(n, (e - c + st - 1) / st) : 0);
            };
            uint32_t ki0, ki1, kj0, kj1;
            krange(S.ci, S.si, S.tb.nx, ib, ie, ki0, ki1);
            krange(S.cj, S.sj, S.tb.ny, jb, je, kj0, kj1);
            if (ki0 >= ki1 || kj0 >= kj1) continue;
            S.tb.i0 = ki0; S.tb.nx = ki1 - ki0;
            S.tb.j0 = kj0; S.tb.ny = kj1 - kj0;
            // member k's region position: px0 + k dx - RG.x0 = k dx - ox (modulo 2^32; the true value >= 0)
            // (the region on the group's grid)
            S.tb.ox = RGg.x0 - S.px0; S.tb.oy = RGg.y0 - S.py0;
            const uint32_t w = S.resw[l - 1], h = S.resh[l - 1];
            // a level whose input resolution starts on an odd coordinate (either axis), or every
            // level under GK_DWT_ANY: the parity-general kernels (gk_dwt_any.hip)
            static const bool force_any = getenv("GK_DWT_ANY") != nullptr;
            if ((S.parx[l - 1] || S.pary[l - 1] || force_any) && !(l == 1 && io)) {
                int32_t* A = base;
                int32_t* B = A + RG.plane;
                int32_t* src_l = (l & 1) ? A : B;
                int32_t* dst_l = (l & 1) ? B : A;
                const uint64_t area = (uint64_t)w * h * S.tb.count();
                gk_launch_dwt_any(ctx->st, irrev, forward, forward ? src_l : dst_l, forward ? dst_l : src_l, RG.stride,
                                  w, h, S.parx[l - 1], S.pary[l - 1], S.tb, GkComps{cst, ncr}, !forward && ctx->dwt_partial);
                ctx->tm.dwt_launches += 3;
                ctx->tm.dwt_bytes += area * 8 * ncr;
                continue;
            }
            const uint64_t area = (uint64_t)w * h * S.tb.count();
            int32_t* A = base;
            int32_t* B = A + RG.plane;
            int32_t* src_l = (l & 1) ? A : B;     // D_{l-1}: level l input plane (l-1 odd -> B)
            int32_t* dst_l = (l & 1) ? B : A;     // D_l
            if (l == 1 && io) {
                // fused level 1: three components through the MCT, the others one by one
                const uint64_t es = gk_sample_size(io->stype);
                // the output rectangle on this group's grid, relative to its region
                GkWin win;
                if (!forward) {
                    win.x0 = (int32_t)(ceildiv(io->cx0, G.dx) - G.ox - RGg.x0); win.y0 = (int32_t)(ceildiv(io->cy0, G.dy) - G.oy - RGg.y0);
                    win.x1 = (int32_t)(ceildiv(io->cx1, G.dx) - G.ox - RGg.x0); win.y1 = (int32_t)(ceildiv(io->cy1, G.dy) - G.oy - RGg.y0);
                }
                for (uint32_t c = c0; c < run.second;) {
                    const int nc = (io->mct3 && c == 0 && run.second >= 3) ? 3 : 1;
                    int32_t* dl = dst_l + (size_t)(c - c0) * cst;
                    GkPtr3 pp;
                    for (int k = 0; k < nc; ++k) pp.p[k] = io->planes[c + k];
                    if (forward) {
                        if (irrev)
                            gk_launch_dwt97_fwd_l1(ctx->st, io->stype, nc, pp, io->strides[c],
                                                   reinterpret_cast<float*>(dl), cst, RG.stride, w, h, S.tb,
                                                   io->shift[c]);
                        else
                            gk_launch_dwt53_fwd_l1(ctx->st, io->stype, nc, pp, io->strides[c], dl, cst,
                                                   RG.stride, w, h, S.tb, io->shift[c]);
                    } else {
                        if (irrev)
                            gk_launch_dwt97_inv_l1(ctx->st, io->stype, nc, reinterpret_cast<const float*>(dl),
                                                   cst, RG.stride, pp, io->strides[c], win, w, h, S.tb, io->shift[c],
                                                   io->mn[c], io->mx[c]);
                        else
                            gk_launch_dwt53_inv_l1(ctx->st, io->stype, nc, dl, cst, RG.stride, pp,
                                                   io->strides[c], win, w, h, S.tb, io->shift[c], io->mn[c], io->mx[c]);
                    }
                    ctx->tm.dwt_launches++;
                    ctx->tm.dwt_bytes += area * (4 + es) * nc;
                    c += nc;
                }
                continue;
            }
            const GkComps cs{cst, ncr};
            if (irrev) {
                float* fs = reinterpret_cast<float*>(src_l);
                float* fd = reinterpret_cast<float*>(dst_l);
                if (forward) gk_launch_dwt97_fwd(ctx->st, fs, RG.stride, fd, RG.stride, w, h, S.tb, cs);
                else gk_launch_dwt97_inv(ctx->st, fd, RG.stride, fs, RG.stride, w, h, S.tb, cs);
            } else {
                if (forward) gk_launch_dwt53_fwd(ctx->st, src_l, RG.stride, dst_l, RG.stride, w, h, S.tb, cs);
                else gk_launch_dwt53_inv(ctx->st, dst_l, RG.stride, src_l, RG.stride, w, h, S.tb, cs);
            }
            ctx->tm.dwt_launches++;
            ctx->tm.dwt_bytes += area * 8 * ncr;
        }
    }
    }
}

static float ev_ms(gk_ctx* ctx, int a, int b) {
    float ms = 0; (void)hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]); return ms;
}

// ---------------------------------------------------------------------------
// Encode
// ---------------------------------------------------------------------------
// Encode tiles [tb, te) (te = 0: all).  with_header: SOC..main header + tile parts + EOC
// (a complete codestream); otherwise only the tile parts, back to back, with their
// lengths in part_lens (tile sharding across devices).
static void setup_plan(gk_ctx* ctx, const gk_image_info* info, const gk_cparameters* cp) {
    Plan want;
    want.w = info->w; want.h = info->h; want.nc = info->numcomps; want.prec = info->prec; want.sgnd = info->sgnd;
    set_params(want.p, cp, want.nc);
    // canvas offsets: image origin (grk_image::x0 / y0) and tile grid origin (grk_cparameters::tx0 / ty0);
    // grk_compress.cpp:1554-1576 / B.3: the grid starts at or above-left of the image, its first
    // tile reaches into the image area
    want.x0 = info->x0; want.y0 = info->y0;
    want.gx0 = cp ? cp->tx0 : 0; want.gy0 = cp ? cp->ty0 : 0;
    if (!ctx->enc_dx.empty()) {   // gk_set_subsampling
        if (ctx->enc_dx.size() != want.nc) throw GkError("gk_set_subsampling was given a different component count");
        want.cdx = ctx->enc_dx; want.cdy = ctx->enc_dy;
        if (!want.subsampled()) { want.cdx.clear(); want.cdy.clear(); }
    }
    if (want.gx0 > want.x0 || want.gy0 > want.y0) throw GkError("tile grid origin must lie at or above-left of the image origin");
    if ((uint64_t)want.x0 + want.w > 0xffffffffull || (uint64_t)want.y0 + want.h > 0xffffffffull)
        throw GkError("image area past the 32-bit canvas");
    if (want.p.tw && ((uint64_t)want.gx0 + want.p.tw <= want.x0 || (uint64_t)want.gy0 + want.p.th <= want.y0))
        throw GkError("the first tile must overlap the image area");
    if (want.nc < 3) want.p.mct = 0;
    // CodeStreamCompress.cpp:501-512: no MCT unless the first three components share a grid
    if (want.p.mct && !want.mct3()) want.p.mct = 0;
    check_poc_coverage(want.p, want.nc);
    if ((want.p.cblk_sty & GK_STY_HT) && want.p.cblk_sty != GK_STY_HT)
        throw GkError("HTJ2K cannot be combined with Part-1 mode switches");   // CodeStreamDecompress.cpp:1781
    if (want.p.cblk_sty > 0x7f) throw GkError("unknown code-block style bits");
    if (want.nc > 255 || want.nc == 0) throw GkError("bad component count");
    if (want.prec == 0 || want.prec > 31) throw GkError("component precision must be 1..31 bits");
    if (want.w == 0 || want.h == 0) throw GkError("empty image");
    // grk_compress.cpp:981-988 (and A.6.1's xcb, ycb): 4 <= side <= 1024, at most 4096 samples
    if (want.p.cbw < 2 || want.p.cbh < 2 || want.p.cbw > 10 || want.p.cbh > 10 || want.p.cbw + want.p.cbh > 12)
        throw GkError("code-block size must be 4..1024 per side with at most 4096 samples");
    ensure_plan(ctx, want);
    restore_native_qcd(ctx);
    // encode: ROI-scaled indices keep 6 fractional bits below them in a 31-bit magnitude
    // (the decoders take up to 30 band bit-planes, checked where a stream's QCD is applied)
    if (!ctx->plan.p.roishift.empty())
    for (const TileG& T : ctx->plan.tiles)
        for (uint32_t ci = 0; ci < (uint32_t)T.comps.size(); ++ci)
            for (const ResG& R : T.comps[ci].res)
                for (const auto& B : R.bands)
                    if (ctx->plan.p.roi(ci) && B.numbps > 25) throw GkError("ROI shift too large for this precision");
}

// gk_encode_blocks: the T1 results of the (single) tile in canonical order, the block bytes
// compacted on the device (the HT pieces joined: MagSgn head, then MEL + VLC tail) and copied out.
static void dump_blocks(gk_ctx* ctx, const uint32_t* hinfo, const GkPass* dps, uint32_t npass_total,
                        uint8_t* dbytes, uint64_t slot0) {
    const Plan& P = ctx->plan;
    hipStream_t st = ctx->st;
    const bool ht = P.p.ht();
    std::vector<GkPass> hp(std::max(npass_total, 1u));
    if (!ht && npass_total)
        HIPCHK(hipMemcpyAsync(hp.data(), dps, sizeof(GkPass) * npass_total, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->rb_bands.clear(); ctx->rb_blocks.clear(); ctx->rb_passes.clear();
    std::vector<uint64_t> seg;
    uint64_t pos = 0;
    const TileG& T = P.tiles[0];
    for (uint32_t c = 0; c < P.nc; ++c)
        for (uint32_t r = 0; r < P.p.numres; ++r) {
            const ResG& R = T.comps[c].res[r];
            for (uint32_t bi = 0; bi < R.bands.size(); ++bi) {
                const BandG& B = R.bands[bi];
                ctx->rb_bands.push_back({c, r, bi, B.orient, R.pw * R.ph, B.step_enc});
                for (uint32_t pi = 0; pi < R.pw * R.ph; ++pi) {
                    const PrecG& PG = R.prc[bi][pi];
                    for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                        const uint32_t b = PG.first_block + k;
                        const GkBlock& G = P.blocks[b];
                        gk_block_result o{};
                        o.comp = c; o.res = r; o.band = bi; o.precinct = pi; o.cblk = k;
                        o.x0 = P.bxy[2 * (size_t)b]; o.y0 = P.bxy[2 * (size_t)b + 1];
                        o.x1 = o.x0 + G.w; o.y1 = o.y0 + G.h;
                        o.numbps = hinfo[4 * (size_t)b]; o.npasses = hinfo[4 * (size_t)b + 1];
                        o.len = hinfo[4 * (size_t)b + 2];
                        o.pass_off = (uint32_t)ctx->rb_passes.size();
                        o.data_off = pos;
                        const uint64_t so = G.data_off - slot0;
                        if (ht && o.npasses) {
                            const uint32_t ms = hinfo[4 * (size_t)b + 3], tl = o.len - ms;
                            if (ms) { seg.push_back(so); seg.push_back(pos); seg.push_back(ms); }
                            seg.push_back(so + G.data_cap - tl); seg.push_back(pos + ms); seg.push_back(tl);
                            ctx->rb_passes.push_back({o.len, o.len, 0.0});
                        } else if (o.npasses) {
                            seg.push_back(so); seg.push_back(pos); seg.push_back(o.len);
                            const GkPass* ps = hp.data() + hinfo[4 * (size_t)b + 3];
                            for (uint32_t q = 0; q < o.npasses; ++q)
                                ctx->rb_passes.push_back({q + 1 == o.npasses ? o.len : ps[q].rate, ps[q].len, ps[q].dist});
                        }
                        pos += o.len;
                        ctx->rb_blocks.push_back(o);
                    }
                }
            }
        }
    ctx->rb_data.resize(pos);
    if (pos) {
        uint64_t* hs = (uint64_t*)ctx->hseg.get(seg.size() * 8);
        memcpy(hs, seg.data(), seg.size() * 8);
        uint64_t* ds = (uint64_t*)ctx->dseg.get(seg.size() * 8);
        HIPCHK(hipMemcpyAsync(ds, hs, seg.size() * 8, hipMemcpyHostToDevice, st));
        uint8_t* dst = (uint8_t*)ctx->dout.get(pos);
        gk_launch_gather(st, dbytes, dst, ds, (uint32_t)(seg.size() / 3));
        HIPCHK(hipMemcpyAsync(ctx->rb_data.data(), dst, pos, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
}

static size_t encode_impl(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
                          int comps_on_device, const gk_cparameters* cp, uint8_t* out, size_t cap, int out_on_device,
                          int* rc, uint32_t tb = 0, uint32_t te = 0, bool with_header = true,
                          uint32_t* part_lens = nullptr, bool blocks_only = false) {
    setup_plan(ctx, info, cp);
    Plan& P = ctx->plan;
    const uint32_t ntiles = (uint32_t)P.tiles.size();
    if (te == 0) { tb = 0; te = ntiles; }
    if (tb >= te || te > ntiles) throw GkError("bad tile range");
    const bool sub = P.subsampled();
    const uint32_t nb = (uint32_t)P.blocks.size();
    const uint32_t b0 = P.tiles[tb].b0, b1 = P.tiles[te - 1].b1, nbr = b1 - b0;   // block range of the tiles
    const uint32_t jb = tb / P.ntx, je = (te - 1) / P.ntx + 1;                     // tile rows touched
    const uint32_t ry0 = P.tiles[jb * P.ntx].y0 - P.y0, ry1 = P.tiles[(je - 1) * P.ntx].y1 - P.y0;  // image rows touched
    hipStream_t st = ctx->st;

    launch_check(__LINE__);

    HIPCHK(hipEventRecord(ctx->ev[0], st));
    // work planes for the sample rows of the selected tiles only
    const Region RG = make_region(0, ry0, P.w, ry1);
    int32_t* arena = (int32_t*)ctx->arena.get(RG.plane * P.nc * 2 * sizeof(int32_t));
    const uint32_t nrows = ry1 - ry0;
    // the caller's planes (int32 or 8/16-bit samples); host planes are staged (those rows only)
    const int stype = sample_type(info->sample_bytes, P.prec, P.sgnd != 0);
    const size_t es = gk_sample_size(stype);
    std::vector<const void*> src(P.nc);
    std::vector<uint32_t> sstr(P.nc);
    // component c reads the rows of the selected tiles on its grid (the region on its sampling
    // group's grid: every row of the image width); host planes are staged back to back
    std::vector<Region> RGg;
    for (const SGroup& G : P.groups) RGg.push_back(group_region(P, RG, G));
    {
        size_t tot = 0;
        for (uint32_t c = 0; c < P.nc; ++c) tot += (size_t)RGg[P.group_of[c]].w * RGg[P.group_of[c]].h;
        uint8_t* dp = comps_on_device ? nullptr : (uint8_t*)ctx->dplanes.get(tot * es + 16);
        size_t o = 0;
        for (uint32_t c = 0; c < P.nc; ++c) {
            const Region& R = RGg[P.group_of[c]];
            const uint8_t* first = (const uint8_t*)comps[c] + (size_t)R.y0 * strides[c] * es;
            if (comps_on_device) { src[c] = first; sstr[c] = strides[c]; continue; }
            HIPCHK(hipMemcpy2DAsync(dp + o * es, (size_t)R.w * es, first, (size_t)strides[c] * es, (size_t)R.w * es, R.h,
                                    hipMemcpyHostToDevice, st));
            src[c] = dp + o * es; sstr[c] = R.w;
            o += (size_t)R.w * R.h;
        }
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    int32_t shift = P.sgnd ? 0 : (1 << (P.prec - 1));
    auto planeA = [&](uint32_t c) { return arena + (size_t)c * 2 * RG.plane; };
    auto planeAf = [&](uint32_t c) { return reinterpret_cast<float*>(planeA(c)); };
    const bool mct3 = P.mct3();
    if (mct3 && (sstr[1] != sstr[0] || sstr[2] != sstr[0])) throw GkError("the first three components must share a stride");
    L1Io io;
    // DC shift + MCT run inside the first DWT level (unless a tile starts on an odd coordinate:
    // then they run first and level 1 takes the parity-general kernels)
    const bool fused = P.p.numres > 1 && P.l1_fusable;
    if (fused) {
        io.stype = stype; io.mct3 = mct3; io.shift.assign(P.nc, shift);
        io.planes.assign(src.begin(), src.end());
        io.strides = sstr;
    } else {
        // no decomposition (or a tile on an odd origin): DC shift + MCT into plane A of each
        // component (each component's plane at its own size)
        auto cw = [&](uint32_t c) { return RGg[P.group_of[c]].w; };
        auto ch = [&](uint32_t c) { return RGg[P.group_of[c]].h; };
        if (!P.p.irrev) {
            if (mct3) gk_launch_dc_rct_fwd(st, stype, src[0], src[1], src[2], sstr[0], planeA(0), planeA(1), planeA(2), RG.stride, cw(0), ch(0), shift);
            for (uint32_t c = mct3 ? 3 : 0; c < P.nc; ++c) gk_launch_dc_fwd(st, stype, src[c], sstr[c], planeA(c), RG.stride, cw(c), ch(c), shift);
        } else {
            if (mct3) gk_launch_dc_ict_fwd(st, stype, src[0], src[1], src[2], sstr[0], planeAf(0), planeAf(1), planeAf(2), RG.stride, cw(0), ch(0), shift);
            for (uint32_t c = mct3 ? 3 : 0; c < P.nc; ++c) gk_launch_dc_fwd_f(st, stype, src[c], sstr[c], planeAf(c), RG.stride, cw(c), ch(c), shift);
        }
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[2], st));
    run_dwt(ctx, RG, true, jb, je, 0, 0xffffffffu, fused ? &io : nullptr);
    if (const char* dp = getenv("GK_DUMP_DWT")) {   // debug: the work planes after the forward DWT
        std::vector<int32_t> hv((size_t)P.nc * 2 * RG.plane);
        HIPCHK(hipMemcpyAsync(hv.data(), arena, hv.size() * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (FILE* f = fopen(dp, "wb")) {
            const uint32_t hd[4] = {P.nc, RG.stride, RG.h, RG.w};
            fwrite(hd, 4, 4, f);
            fwrite(hv.data(), 4, hv.size(), f);
            fclose(f);
        }
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[3], st));
    // T1 over the block range [b0, b1): every per-block device array is range-local
    const bool do_rc = P.p.rate_control();
    const uint64_t slot0 = P.blocks[b0].data_off;
    const uint64_t slot1 = b1 < nb ? P.blocks[b1].data_off : P.slot_bytes;
    const uint64_t slot_span = slot1 - slot0;    // the range's slots; host bytes are staged after them
    uint8_t* dbytes = (uint8_t*)ctx->bytes.get(slot_span + (64u << 20));
    const uint32_t nbx = std::max(nbr, 1u);
    GkBlock* dblk = (GkBlock*)ctx->dblocks.get(sizeof(GkBlock) * nbx);
    GkPass* dps = (GkPass*)ctx->dpasses.get(sizeof(GkPass) * GK_MAX_PASSES * (size_t)nbx);
    uint32_t* dinfo = (uint32_t*)ctx->dinfo.get(16 * (size_t)nbx + 16);
    int* derr = (int*)ctx->derr.get(64);
    uint32_t* dpcount = (uint32_t*)(derr + 4);
    uint8_t* dsym = P.p.ht() ? nullptr : (uint8_t*)ctx->dsym.get(P.sym_off[b1] - P.sym_off[b0] + 256);
    uint64_t* dsymoff = (uint64_t*)ctx->dsymoff.get(8 * ((size_t)nbr + 1));
    uint32_t* dpe = (uint32_t*)ctx->dpassend.get(4 * GK_MAX_PASSES * (size_t)nbx);
    uint32_t* dcm = (uint32_t*)ctx->dcminfo.get(8 * (size_t)nbx);
    int32_t* dnmse = do_rc ? (int32_t*)ctx->dnmse.get(4 * GK_MAX_PASSES * (size_t)nbx) : nullptr;
    if (!ctx->blocks_uploaded || ctx->enc_b0 != b0 || ctx->enc_b1 != b1 || ctx->enc_rc != do_rc) {
        // the range's blocks with offsets into this call's planes and slots
        GkBlock* hb = (GkBlock*)ctx->hpasses.get(sizeof(GkBlock) * nbx + 8 * ((size_t)nbr + 1));
        uint64_t* hso = (uint64_t*)(hb + nbx);
        for (uint32_t i = 0; i < nbr; ++i) {
            hb[i] = P.blocks[b0 + i];
            hb[i].band_off = relocate(P, group_region(P, RG, P.groups[P.group_of[hb[i].comp]]), hb[i].band_off);
            hb[i].stride = RG.stride;
            hb[i].data_off -= slot0;
            hb[i].flags = (uint8_t)((hb[i].flags & ~2u) | (do_rc ? 2u : 0u));
        }
        for (uint32_t i = 0; i <= nbr; ++i) hso[i] = P.sym_off[b0 + i] - P.sym_off[b0];
        HIPCHK(hipMemcpyAsync(dblk, hb, sizeof(GkBlock) * nbr, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(dsymoff, hso, 8 * ((size_t)nbr + 1), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));   // the staging buffer is reused below
        ctx->blocks_uploaded = true; ctx->enc_b0 = b0; ctx->enc_b1 = b1; ctx->enc_rc = do_rc;
    }
    HIPCHK(hipMemsetAsync(derr, 0, 64, st));
    // solo MQ waves (gk_t1enc.hip mq_solo_block): GK_T1ENC_SOLO = how many of the heaviest blocks
    // of the first chunk they code (without chunks: the first blocks in index order; tests)
    const uint32_t nsolo_env = []() { const char* v = getenv("GK_T1ENC_SOLO"); return v ? (uint32_t)atoi(v) : 0u; }();
    if (P.p.ht()) {
        // HT cleanup pass (T1HT::compress, T1HT.cpp:109-133); MEL bytes staged in the symbol buffer
        uint8_t* mel = (uint8_t*)ctx->dsym.get((size_t)nbx * GK_HT_MEL_CAP + 256);
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[8], st));
        gk_launch_ht_enc(st, arena, dblk, dbytes, mel, GK_HT_MEL_CAP, dinfo, nbr, derr, P.p.wide());
    } else if (P.p.t1_generic()) {
        // mode switches: lane-per-block coder with per-pass termination rules (gk_t1ms.hip)
        uint8_t* mst = (uint8_t*)ctx->dmsstate.get(gk_t1ms_state_bytes(nbx));
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[8], st));
        gk_launch_t1_enc_ms(st, arena, dblk, dbytes, dps, dinfo, nbr, derr, ctx->nmse_tab, dpcount, mst, P.p.cblk_sty & 0x3f);
    } else if (nbr < 8192 || getenv("GK_T1ENC_SERIAL")) {
        gk_launch_t1_cm(st, arena, dblk, dsymoff, dsym, dpe, dcm, nbr, derr, ctx->nmse_tab, dnmse);
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[8], st));
        gk_launch_t1_mq(st, dsym, dsymoff, dpe, dcm, dblk, dbytes, dps, dinfo, nbr, derr, dnmse, dpcount, nullptr, 0,
                        0xffffffffu, std::min(nsolo_env, nbr));
    } else {
        // Context modelling and MQ coding overlap.  Blocks go heaviest first (most coded
        // bit-planes, k_t1_weight) in three chunks; chunk i's MQ kernel starts on its own stream
        // once chunk i is modelled, so the longest MQ chains run while the lighter blocks are
        // still being modelled.  An MQ workgroup fills its CU's LDS, so the modelling waves never
        // share a SIMD with an MQ chain (sharing one slowed the chains more than the overlap
        // gained).  Each block is coded exactly as in one pass; only the launch order changes.
        uint32_t* dw = (uint32_t*)ctx->dweight.get(4 * (size_t)nbr);
        gk_launch_t1_weight(st, arena, dblk, dw, nbr);
        uint32_t* hw = (uint32_t*)ctx->hweight.get(4 * (size_t)nbr);
        HIPCHK(hipMemcpyAsync(hw, dw, 4 * (size_t)nbr, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        // counting sort, descending, on the estimate quantised to 4096 buckets of the range
        uint32_t wmax = 1;
        for (uint32_t i = 0; i < nbr; ++i) wmax = std::max(wmax, hw[i]);
        const uint32_t kB = 4096;
        auto key = [&](uint32_t i) { return kB - 1 - (uint32_t)(((uint64_t)hw[i] * (kB - 1)) / wmax); };
        std::vector<uint32_t> start(kB + 1, 0);
        for (uint32_t i = 0; i < nbr; ++i) start[key(i)]++;
        for (uint32_t k = 0, acc = 0; k <= kB; ++k) { const uint32_t c = start[k]; start[k] = acc; acc += c; }
        uint32_t* ho = (uint32_t*)ctx->hord_enc.get(4 * (size_t)nbr);
        for (uint32_t i = 0; i < nbr; ++i) ho[start[key(i)]++] = i;
        uint32_t* dord = (uint32_t*)ctx->dord_enc.get(4 * (size_t)nbr);
        HIPCHK(hipMemcpyAsync(dord, ho, 4 * (size_t)nbr, hipMemcpyHostToDevice, st));
        // chunk ends as fractions of the blocks (GK_T1ENC_CUTS, up to three), rounded to whole MQ
        // workgroups (4 x 64 blocks); the last chunk's MQ runs on the main stream.  Defaults
        // measured per workload (bench enc_t1): without rate control 0.125, 0.375 (C2 9.18 ms;
        // 0.08, 0.25: 9.3), with it, where the modelling also sums distortions, 0.08, 0.25 (C3
        // 14.96-15.22 ms against 15.6-15.8)
        static std::vector<double> frs[2];
        std::vector<double>& fr = frs[do_rc ? 1 : 0];
        if (fr.empty()) {
            const char* cv = getenv("GK_T1ENC_CUTS");
            std::string cs = cv ? cv : (do_rc ? "0.08,0.25" : "0.125,0.375");
            for (size_t q = 0; q < cs.size();) {
                size_t e = cs.find(',', q);
                if (e == std::string::npos) e = cs.size();
                const double f = atof(cs.substr(q, e - q).c_str());
                if (f > 0 && f < 1 && fr.size() < 3) fr.push_back(f);
                q = e + 1;
            }
        }
        std::vector<uint32_t> cut(1, 0);
        for (double f : fr) {
            const uint32_t c = (uint32_t)(nbr * f) / 256 * 256;
            if (c > cut.back() && c < nbr) cut.push_back(c);
        }
        cut.push_back(nbr);
        const int nch = (int)cut.size() - 1;
        for (int k = 0; k < nch; ++k) {
            const uint32_t base = cut[k], cnt = cut[k + 1] - cut[k];
            gk_launch_t1_cm(st, arena, dblk, dsymoff, dsym, dpe, dcm, nbr, derr, ctx->nmse_tab, dnmse, dord, base, cnt);
            if (k + 1 < nch) {
                HIPCHK(hipEventRecord(ctx->xev[k], st));
                HIPCHK(hipStreamWaitEvent(ctx->aux[k], ctx->xev[k], 0));
                gk_launch_t1_mq(ctx->aux[k], dsym, dsymoff, dpe, dcm, dblk, dbytes, dps, dinfo, nbr, derr, dnmse, dpcount,
                                dord, base, cnt, k == 0 ? std::min(nsolo_env, cnt) : 0u);
                HIPCHK(hipEventRecord(ctx->xev[3 + k], ctx->aux[k]));
            } else {
                launch_check(__LINE__);
                HIPCHK(hipEventRecord(ctx->ev[8], st));
                gk_launch_t1_mq(st, dsym, dsymoff, dpe, dcm, dblk, dbytes, dps, dinfo, nbr, derr, dnmse, dpcount, dord,
                                base, cnt);
            }
        }
        for (int k = 0; k + 1 < nch; ++k) HIPCHK(hipStreamWaitEvent(st, ctx->xev[3 + k], 0));
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[4], st));
    // GK_PROFILE=1: host phase times of the encode's T2 (stderr)
    static const bool eprof = getenv("GK_PROFILE") != nullptr;
    using eclk = std::chrono::steady_clock;
    auto ems = [](eclk::time_point a, eclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto te0 = eclk::now();
    uint32_t* hinfo = (uint32_t*)ctx->hinfo.get(16 * (size_t)nb + 64);
    HIPCHK(hipMemcpyAsync(hinfo + 4 * (size_t)b0, dinfo, 16 * (size_t)nbr, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(hinfo + 4 * (size_t)nb, derr, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t t1err = hinfo[4 * (size_t)nb], npass_total = hinfo[4 * (size_t)nb + 4];
    if (t1err) throw GkError(t1err & 2 ? "T1 symbol buffer overflow" : "T1 code-block slot overflow");
    const bool ht = P.p.ht();
    const GkPass* hpasses = nullptr;
    // pass records: rate control, and BYPASS / TERMALL (a length per codeword segment)
    if ((do_rc || (P.p.cblk_sty & (GK_STY_LAZY | GK_STY_TERMALL))) && !ht) {
        GkPass* hp = (GkPass*)ctx->hpasses.get(sizeof(GkPass) * (size_t)std::max(npass_total, 1u));
        HIPCHK(hipMemcpyAsync(hp, dps, sizeof(GkPass) * (size_t)npass_total, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        hpasses = hp;
    }
    if (blocks_only) {   // gk_encode_blocks: T1 results only (the host of a T1 plugin runs T2)
        dump_blocks(ctx, hinfo, dps, npass_total, dbytes, slot0);
        *rc = 0;
        return 0;
    }

    // ---- host T2 (T2Compress.cpp:113-240) with layer formation / rate allocation
    std::vector<uint8_t> H;
    H.reserve(1 << 12);
    size_t tlm_pos = 0;
    write_main_header(H, P, &tlm_pos);
    // updateRates' header bytes: the stream position after the main header (JP2 boxes and the
    // jp2c box header come first in a .jp2), CodeStreamCompress.cpp:963
    const size_t rc_header_size = H.size() + (P.p.jp2 ? jp2_prefix_size(P) : 0);
    if (!with_header) H.clear();
    const auto te1 = eclk::now();
    if (const char* ds = getenv("GK_DUMP_SYMS"); ds && dsym && !P.p.t1_generic()) {
        // debug: per-block MQ symbol counts (decisions) and coded bit-planes, u32 pairs
        std::vector<uint32_t> pe((size_t)GK_MAX_PASSES * nbr), cm(2 * (size_t)nbr), out(2 * (size_t)nbr);
        HIPCHK(hipMemcpy(pe.data(), dpe, 4 * pe.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(cm.data(), dcm, 4 * cm.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < nbr; ++i) {
            out[2 * i] = cm[2 * i + 1] ? pe[(size_t)GK_MAX_PASSES * i + cm[2 * i + 1] - 1] : 0;
            out[2 * i + 1] = cm[2 * i];
        }
        if (FILE* f = fopen(ds, "wb")) { fwrite(out.data(), 4, out.size(), f); fclose(f); }
    }
    if (const char* dp = getenv("GK_DUMP_PASSES")) {   // debug: pass records for tools/pcrd_bench
        if (FILE* f = fopen(dp, "wb")) {
            const uint32_t hdr[2] = {nb, npass_total};
            fwrite(hdr, 4, 2, f);
            fwrite(hinfo, 16, nb, f);
            if (hpasses) fwrite(hpasses, sizeof(GkPass), npass_total, f);
            fclose(f);
        }
    }
    T2Enc T2(P, hinfo, hpasses, tb, te);
    std::vector<T2Enc::Swallow> tsw(te - tb);   // per tile: the final simulation's swallowed failure
    if (te - tb == 1 || !P.p.rate_control()) {
        T2.allocate(rc_header_size);
        tsw[0] = T2.final_sw;
    } else {
        // rate control per tile (TileProcessor::pcrdBisectSimple runs per tile): many tiles run
        // side by side on one thread each, a few run one after the other on the whole pool
        const bool par = te - tb >= host_pool().size();
        auto one = [&](size_t q) {
            const uint32_t t = tb + (uint32_t)q;
            T2Enc Tt(P, hinfo, hpasses, t, t + 1);
            Tt.serial = par;
            Tt.allocate(rc_header_size);
            tsw[q] = Tt.final_sw;
            const TileG& TG = P.tiles[t];
            std::copy(Tt.lnp.begin() + (size_t)TG.b0 * T2.L, Tt.lnp.begin() + (size_t)TG.b1 * T2.L,
                      T2.lnp.begin() + (size_t)TG.b0 * T2.L);
        };
        if (par) host_pool().run(te - tb, one);
        else for (uint32_t q = 0; q < te - tb; ++q) one(q);
    }
    const auto te2 = eclk::now();
    // segments: (src_off in dbytes, dst_off in codestream, len); host bytes staged after the slots
    std::vector<uint64_t> seg;
    seg.reserve(3 * ((size_t)nb * (ht ? 2 : 1) + 64));
    std::vector<uint8_t> hdrs;   // all host bytes, in order, copied to staging
    uint64_t pos = 0;            // codestream position
    auto add_host = [&](const uint8_t* p, size_t n) {
        if (!n) return;
        seg.push_back(slot_span + hdrs.size()); seg.push_back(pos); seg.push_back(n);
        hdrs.insert(hdrs.end(), p, p + n);
        pos += n;
    };
    // JP2 boxes before the codestream; the jp2c length is written once the size is known
    std::vector<uint8_t> J;
    const bool jp2 = P.p.jp2 && with_header;
    if (jp2) write_jp2_prefix(J, P, 0);
    add_host(J.data(), J.size());
    const size_t main_at = J.size();   // the main header's position in hdrs
    add_host(H.data(), H.size());
    // per tile: packets (T2Compress::compressPackets) and the tile-part header; tiles are
    // independent, so they are built in parallel host threads and appended in tile order
    struct Pk { uint32_t hoff, hlen, s0, s1, len; };
    struct TileOut {
        std::vector<uint8_t> tp;     // SOT [PLT] SOD (every tile part's, concatenated)
        std::vector<uint8_t> phdr;   // packet headers
        std::vector<Pk> pk;
        std::vector<uint32_t> bsegs; // (block, first byte, length) of every packet body
        uint64_t psot = 0;
        std::vector<uint32_t> pkey;  // tile part of each packet
        std::vector<uint32_t> tp_off, pk_first;   // per tile part: header offset in tp, first packet
        std::vector<uint64_t> psots;
    };
    const TilePartSplit TPS = tile_part_split(P);
    if (part_lens && TPS.n > 1) throw GkError("tile-part generation is not supported with tile sharding");
    std::vector<TileOut> tout(te - tb);
    const bool par_chains = te - tb == 1;   // one tile: its precinct chains run in parallel instead
    auto build_tile_part = [&](uint32_t t, TileOut& O) {
        const TileG& T = P.tiles[t];
        const T2Enc::Swallow& sw = tsw[t - tb];
        // A (resolution, component, precinct) chain owns its code-blocks and tag trees, so chains
        // are independent; within a chain the layers are sequential (T2 state carries over).
        struct Chain { uint32_t r, c, pi; };
        std::vector<Chain> chains;
        for (uint32_t r = 0; r < P.p.numres; ++r)
            for (uint32_t c = 0; c < P.nc; ++c)
                for (uint32_t pi = 0; pi < T.comps[c].res[r].pw * T.comps[c].res[r].ph; ++pi) chains.push_back({r, c, pi});
        const uint32_t L = P.p.nlayers;
        std::vector<TileOut> co(chains.size());   // per chain: headers, body segments, one Pk per layer
        auto run_chain = [&](size_t q) {
            const Chain& ch = chains[q];
            const ResG& R = T.comps[ch.c].res[ch.r];
            TileOut& C = co[q];
            std::vector<uint32_t> body;
            std::vector<uint8_t> hb;
            for (uint32_t l = 0; l < L; ++l) {
                body.clear();
                T2.write_packet(R, ch.pi, l, nullptr, &body, hb);
                Pk k{(uint32_t)C.phdr.size(), (uint32_t)hb.size(), (uint32_t)C.bsegs.size(), 0, (uint32_t)hb.size()};
                C.phdr.insert(C.phdr.end(), hb.begin(), hb.end());
                for (size_t i = 0; i < body.size(); i += 3) {
                    if (!body[i + 2]) continue;
                    C.bsegs.push_back(body[i]); C.bsegs.push_back(body[i + 1]); C.bsegs.push_back(body[i + 2]);
                    k.len += body[i + 2];
                }
                k.s1 = (uint32_t)C.bsegs.size();
                C.pk.push_back(k);
            }
        };
        if (par_chains && chains.size() > 1) {
            // One tile: (chain, band) units in parallel - a band's tag trees and code-blocks are
            // its own, so each codes its part of every layer's header as raw bits and its body
            // segments; per (chain, layer) the header is then the bit 1, the bands' bits in band
            // order and a flush through the stuffing writer (the same bit sequence write_packet
            // writes), the body the bands' segments in band order.  The top resolution's three
            // bands (C2: 4,096 blocks each) no longer run as one chain.
            struct BandU { uint32_t q, bi; };
            std::vector<BandU> bu;
            std::vector<uint32_t> bu0(chains.size() + 1, 0);
            for (size_t q = 0; q < chains.size(); ++q) {
                const ResG& R = T.comps[chains[q].c].res[chains[q].r];
                for (uint32_t bi = 0; bi < R.bands.size(); ++bi)
                    if (R.prc[bi][chains[q].pi].cw && R.prc[bi][chains[q].pi].ch) bu.push_back({(uint32_t)q, bi});
                bu0[q + 1] = (uint32_t)bu.size();
            }
            std::vector<std::vector<RawBits>> ubit(bu.size(), std::vector<RawBits>(L));
            std::vector<std::vector<uint32_t>> useg(bu.size());     // (block, first byte, length)
            std::vector<std::vector<uint32_t>> uend(bu.size(), std::vector<uint32_t>(L));   // useg end per layer
            std::vector<size_t> bord(bu.size());
            for (size_t i = 0; i < bord.size(); ++i) bord[i] = bord.size() - 1 - i;   // largest first
            host_pool().run(bord.size(), [&](size_t j) {
                const size_t u = bord[j];
                const Chain& ch = chains[bu[u].q];
                const ResG& R = T.comps[ch.c].res[ch.r];
                const PrecG& PG = R.prc[bu[u].bi][ch.pi];
                T2.band_init(PG, R.bands[bu[u].bi].numbps);
                std::vector<uint32_t>& sg = useg[u];
                for (uint32_t l = 0; l < L; ++l) {
                    RawBits& rb = ubit[u][l];
                    T2.band_header(PG, l, rb);
                    rb.finish();
                    for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                        const uint32_t b = PG.first_block + k;
                        const uint32_t np = T2.lnp[(size_t)b * L + l];
                        if (!np) continue;
                        const uint32_t r0 = T2.inprev[b] ? T2.rate(b, T2.inprev[b] - 1) : 0, r1 = T2.rate(b, T2.inprev[b] + np - 1);
                        if (r1 > r0) { sg.push_back(b); sg.push_back(r0); sg.push_back(r1 - r0); }
                        T2.inprev[b] = (uint16_t)(T2.inprev[b] + np);
                    }
                    uend[u][l] = (uint32_t)sg.size();
                }
            });
            host_pool().run(chains.size(), [&](size_t q) {
                TileOut& C = co[q];
                for (uint32_t l = 0; l < L; ++l) {
                    const uint32_t h0 = (uint32_t)C.phdr.size();
                    PktBitWriter bw(C.phdr);
                    bw.putbit(1);
                    for (uint32_t u = bu0[q]; u < bu0[q + 1]; ++u) {
                        const RawBits& rb = ubit[u][l];
                        const size_t full = (size_t)(rb.n / 64);
                        const uint32_t rem = (uint32_t)(rb.n % 64);
                        for (size_t i = 0; i < full; ++i) { bw.put((uint32_t)(rb.w[i] >> 32), 32); bw.put((uint32_t)rb.w[i], 32); }
                        if (rem) {
                            const uint64_t x = rb.w[full] >> (64 - rem);
                            if (rem > 32) { bw.put((uint32_t)(x >> 32), rem - 32); bw.put((uint32_t)x, 32); }
                            else bw.put((uint32_t)x, rem);
                        }
                    }
                    bw.flush();
                    const uint32_t hlen = (uint32_t)C.phdr.size() - h0;
                    Pk k{h0, hlen, (uint32_t)C.bsegs.size(), 0, hlen};
                    for (uint32_t u = bu0[q]; u < bu0[q + 1]; ++u) {
                        const uint32_t s0 = l ? uend[u][l - 1] : 0, s1 = uend[u][l];
                        for (uint32_t i = s0; i < s1; i += 3) k.len += useg[u][i + 2];
                        C.bsegs.insert(C.bsegs.end(), useg[u].begin() + s0, useg[u].begin() + s1);
                    }
                    k.s1 = (uint32_t)C.bsegs.size();
                    C.pk.push_back(k);
                }
            });
        } else {
            for (size_t q = 0; q < chains.size(); ++q) run_chain(q);
        }
        // packets in the progression order (chains are numbered in (resolution, component,
        // precinct) order)
        std::vector<uint32_t> chain_at(P.p.numres * P.nc + 1, 0);
        for (uint32_t r = 0, q = 0; r < P.p.numres; ++r)
            for (uint32_t c = 0; c < P.nc; ++c) { chain_at[r * P.nc + c] = q; q += T.comps[c].res[r].pw * T.comps[c].res[r].ph; }
        std::vector<uint32_t> entry;
        const std::vector<PacketRef> order = packet_order(P, T, L, &P.p.pocs, TPS.poc ? &entry : nullptr);
        for (size_t oi = 0; oi < order.size(); ++oi) {
                const PacketRef& pr = order[oi];
                O.pkey.push_back(TPS.poc ? entry[2 * oi] : TPS.key(pr));
                const size_t q = chain_at[pr.r * P.nc + pr.c] + pr.pi;
                const uint32_t l = pr.l;
                const TileOut& C = co[q];
                Pk k = C.pk[l];
                const uint32_t h0 = (uint32_t)O.phdr.size(), s0 = (uint32_t)O.bsegs.size();
                if (P.p.sop_eph & 2) {   // SOP: FF91, Lsop 4, Nsop = the packet's index in the tile (T2Compress.cpp:286-303)
                    const uint32_t nsop = (TPS.poc ? entry[2 * oi + 1] : (uint32_t)O.pk.size()) & 0xffff;
                    const uint8_t sop[6] = {0xff, 0x91, 0, 4, (uint8_t)(nsop >> 8), (uint8_t)nsop};
                    O.phdr.insert(O.phdr.end(), sop, sop + 6);
                }
                O.phdr.insert(O.phdr.end(), C.phdr.begin() + k.hoff, C.phdr.begin() + k.hoff + k.hlen);
                if (P.p.sop_eph & 4) { O.phdr.push_back(0xff); O.phdr.push_back(0x92); }   // EPH (:312-319)
                const uint32_t ovh = ((P.p.sop_eph & 2) ? 6 : 0) + ((P.p.sop_eph & 4) ? 2 : 0);
                k.hlen += ovh; k.len += ovh;
                O.bsegs.insert(O.bsegs.end(), C.bsegs.begin() + k.s0, C.bsegs.begin() + k.s1);
                k.hoff = h0; k.s1 = s0 + (k.s1 - k.s0); k.s0 = s0;
                O.pk.push_back(k);
            }
        // tile parts: SOT [PLT] SOD (CodeStreamCompress::writeTilePart :858-900); the PLT of every
        // packet of the tile goes into the first part's header (TileProcessor::writeTilePartT2)
        std::vector<uint8_t>& tp = O.tp;
        size_t pk0 = 0;
        for (uint32_t part = 0; part < TPS.n; ++part) {
            size_t pk1 = pk0;
            while (pk1 < O.pk.size() && O.pkey[pk1] == part) ++pk1;
            const size_t h0 = tp.size();
            O.tp_off.push_back((uint32_t)h0); O.pk_first.push_back((uint32_t)pk0);
            put16(tp, 0xff90); put16(tp, 10); put16(tp, t); put32(tp, 0); tp.push_back((uint8_t)part);
            tp.push_back((uint8_t)TPS.n);
            // POC in the tile's first tile part (writeTilePart :870-875): writePoc writes tile 0's
            // list (tcp = m_cp.tcps) as the main header's writePoc clamped it, each entry's
            // progression being what tile 0's last PacketManager left: for tile 0 its own
            // rate-control simulation (THRESH_CALC: tcp->prg), for later tiles tile 0's final pass
            // (the given progressions)
            if (part == 0 && !P.p.pocs.empty()) write_poc(tp, P.p.pocs, P.nc, &P, t == 0 ? P.p.prog : ~0u);
            if (P.p.plt && part == 0) {   // PacketLengthMarkers::write (PacketLengthMarkers.cpp:107-175): Zplt 0, 7-bit groups MSB first
                // the lengths come from the final simulation (compressPacketSimulate :427-428):
                // with progression order changes they are listed in the tile's own progression,
                // and a swallowed failure there counted its packet's header as Grok's BitIO did
                std::vector<uint32_t> lens;
                const uint32_t ovh = ((P.p.sop_eph & 2) ? 6 : 0) + ((P.p.sop_eph & 4) ? 2 : 0);
                for (const PacketRef& pr : packet_order(P, T, L)) {
                    uint32_t len = co[chain_at[pr.r * P.nc + pr.c] + pr.pi].pk[pr.l].len + ovh;
                    if (sw.on && pr.c == sw.c && pr.r == sw.r && pr.pi == sw.pi && pr.l == sw.l)
                        len = (uint32_t)(len + sw.hcnt - sw.hreal);
                    lens.push_back(len);
                }
                std::vector<uint8_t> v;
                for (const uint32_t len : lens) {
                    const int nbits = floorlog2(len) + 1, nbytes = (nbits + 6) / 7;
                    for (int q = nbytes - 1; q >= 0; --q) v.push_back((uint8_t)(((len >> (7 * q)) & 0x7F) | (q ? 0x80 : 0)));
                }
                if (3 + v.size() > 65535) throw GkError("PLT marker overflow (too many packets in one tile)");
                put16(tp, 0xff58); put16(tp, (uint32_t)(3 + v.size())); tp.push_back(0);
                tp.insert(tp.end(), v.begin(), v.end());
            }
            put16(tp, 0xff93);
            uint64_t psot = tp.size() - h0;
            for (size_t q = pk0; q < pk1; ++q) psot += O.pk[q].len;
            // a tile in one part with one progression writes the length TileProcessor precalculated
            // from the final simulation (canPreCalculateTileLen, TileProcessor.cpp:54-57, 243-259)
            if (TPS.n == 1 && sw.on) psot = psot + sw.hcnt - sw.hreal;
            if (psot > 0xffffffffull) throw GkError("tile part exceeds 4 GiB");
            tp[h0 + 6] = (uint8_t)(psot >> 24); tp[h0 + 7] = (uint8_t)(psot >> 16); tp[h0 + 8] = (uint8_t)(psot >> 8);
            tp[h0 + 9] = (uint8_t)psot;
            O.psots.push_back(psot);
            pk0 = pk1;
        }
        if (pk0 != O.pk.size()) throw GkError("tile-part split out of packet order");
        O.tp_off.push_back((uint32_t)tp.size()); O.pk_first.push_back((uint32_t)pk0);
        O.psot = O.psots[0];
    };
    if (par_chains) build_tile_part(tb, tout[0]);   // (its chains use the pool: no nested pool call)
    else host_pool().run(te - tb, [&](size_t q) { build_tile_part(tb + (uint32_t)q, tout[q]); });
    const auto te3 = eclk::now();
    for (uint32_t t = tb; t < te; ++t) {
        TileOut& O = tout[t - tb];
        if (part_lens) part_lens[t - tb] = (uint32_t)O.psot;
        for (uint32_t part = 0; part < TPS.n; ++part) {
        const uint64_t psot = O.psots[part];
        if (P.p.tlm && with_header) {   // one TLM entry per tile part, in stream order
            uint8_t* e = hdrs.data() + main_at + tlm_pos + 6 * ((size_t)t * TPS.n + part);   // the main header is hdrs[main_at ..)
            e[0] = (uint8_t)(t >> 8); e[1] = (uint8_t)t;
            e[2] = (uint8_t)(psot >> 24); e[3] = (uint8_t)(psot >> 16); e[4] = (uint8_t)(psot >> 8); e[5] = (uint8_t)psot;
        }
        add_host(O.tp.data() + O.tp_off[part], O.tp_off[part + 1] - O.tp_off[part]);
        const uint32_t pa = O.pk_first[part], pe = O.pk_first[part + 1];
        if (!ht && te - tb == 1 && (size_t)O.bsegs.size() >= 3 * 8192) {
            // one tile's many body segments (C2 / C3: 49 k per layer) in parallel per packet: a
            // packet's triples, header bytes and stream position follow from the ones before it
            const uint32_t np = pe - pa;
            std::vector<size_t> sb(np + 1), hb(np + 1);
            std::vector<uint64_t> pb(np + 1);
            sb[0] = seg.size(); hb[0] = hdrs.size(); pb[0] = pos;
            for (uint32_t i = 0; i < np; ++i) {
                const Pk& k = O.pk[pa + i];
                sb[i + 1] = sb[i] + (k.hlen ? 3 : 0) + (k.s1 - k.s0);
                hb[i + 1] = hb[i] + k.hlen;
                pb[i + 1] = pb[i] + k.len;
            }
            seg.resize(sb[np]);
            hdrs.resize(hb[np]);
            host_pool().run(np, [&](size_t i) {
                const Pk& k = O.pk[pa + i];
                uint64_t* w = seg.data() + sb[i];
                uint64_t p = pb[i];
                if (k.hlen) {
                    w[0] = slot_span + hb[i]; w[1] = p; w[2] = k.hlen; w += 3;
                    memcpy(hdrs.data() + hb[i], O.phdr.data() + k.hoff, k.hlen);
                    p += k.hlen;
                }
                for (uint32_t q = k.s0; q < k.s1; q += 3) {
                    const uint32_t b = O.bsegs[q], off = O.bsegs[q + 1], n = O.bsegs[q + 2];
                    w[0] = P.blocks[b].data_off - slot0 + off; w[1] = p; w[2] = n; w += 3;
                    p += n;
                }
            });
            pos = pb[np];
            continue;
        }
        for (uint32_t pq = pa; pq < pe; ++pq) {
            const Pk& k = O.pk[pq];
            add_host(O.phdr.data() + k.hoff, k.hlen);
            for (uint32_t q = k.s0; q < k.s1; q += 3) {
                const uint32_t b = O.bsegs[q], off = O.bsegs[q + 1], n = O.bsegs[q + 2];
                const GkBlock& G = P.blocks[b];
                const uint64_t so = G.data_off - slot0;   // the block's slot in this call's byte arena
                if (ht) {   // MagSgn head at the slot start, MEL+VLC tail at the slot end
                    const uint32_t ms = hinfo[4 * (size_t)b + 3], tl = n - ms;
                    if (ms) { seg.push_back(so); seg.push_back(pos); seg.push_back(ms); pos += ms; }
                    seg.push_back(so + G.data_cap - tl); seg.push_back(pos); seg.push_back(tl);
                    pos += tl;
                    continue;
                }
                seg.push_back(so + off); seg.push_back(pos); seg.push_back(n);
                pos += n;
            }
        }
        }
    }
    uint8_t eoc[2] = {0xff, 0xd9};
    if (with_header) add_host(eoc, 2);
    const size_t total = pos;
    if (jp2) {
        J.clear();
        write_jp2_prefix(J, P, total - jp2_prefix_size(P));
        memcpy(hdrs.data(), J.data(), J.size());
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[5], st));
    if (eprof)
        fprintf(stderr, "encode t2: fetch %.2f ms, allocate %.2f ms, packets %.2f ms, segments %.2f ms\n", ems(te0, te1),
                ems(te1, te2), ems(te2, te3), ems(te3, eclk::now()));
    if (total > cap) { *rc = -2; return total; }
    // ---- device assembly
    if (hdrs.size() > (64u << 20)) throw GkError("packet headers exceed staging");
    uint8_t* hh = (uint8_t*)ctx->hhdr.get(hdrs.size());
    memcpy(hh, hdrs.data(), hdrs.size());
    HIPCHK(hipMemcpyAsync(dbytes + slot_span, hh, hdrs.size(), hipMemcpyHostToDevice, st));
    uint64_t* hs = (uint64_t*)ctx->hseg.get(seg.size() * 8);
    memcpy(hs, seg.data(), seg.size() * 8);
    uint64_t* ds = (uint64_t*)ctx->dseg.get(seg.size() * 8);
    HIPCHK(hipMemcpyAsync(ds, hs, seg.size() * 8, hipMemcpyHostToDevice, st));
    uint8_t* dst = out_on_device ? out : (uint8_t*)ctx->dout.get(total);
    gk_launch_gather(st, dbytes, dst, ds, (uint32_t)(seg.size() / 3));
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[6], st));
    if (!out_on_device) HIPCHK(hipMemcpyAsync(out, dst, total, hipMemcpyDeviceToHost, st));
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[7], st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->tm.mct_ms = ev_ms(ctx, 1, 2);
    ctx->tm.dwt_ms = ev_ms(ctx, 2, 3);
    ctx->tm.t1_ms = ev_ms(ctx, 3, 4);
    ctx->tm.t1_cm_ms = ev_ms(ctx, 3, 8);
    ctx->tm.t1_coder_ms = ev_ms(ctx, 8, 4);
    ctx->tm.cs_bytes = total;
    {
        uint64_t tbytes = 0;
        for (uint32_t b = b0; b < b1; ++b) tbytes += hinfo[4 * (size_t)b + 2];
        ctx->tm.t1_bytes = tbytes;
    }
    ctx->tm.t2_ms = ev_ms(ctx, 4, 5);
    ctx->tm.assemble_ms = ev_ms(ctx, 5, 7);
    ctx->tm.total_ms = ev_ms(ctx, 0, 7);
    ctx->tm.t1_blocks = nbr;
    *rc = 0;
    return total;
}

// ---------------------------------------------------------------------------
// Decode
// ---------------------------------------------------------------------------
struct TilePart {                  // packet bytes [data, end) of one tile part
    uint32_t tile; size_t sot, data, end;
    std::vector<uint32_t> plt;      // packet lengths from PLT markers (empty without PLT)
    // a tile's later tile parts (TPsot 1, 2, ...), merged behind its first: their packet
    // ranges continue the tile's packet sequence (B.10.4 / T2Decompress over the tile's
    // parts in order); their PLT lengths are appended to plt
    std::vector<std::pair<size_t, size_t>> more;
    uint32_t tpsot = 0;
    std::vector<Poc> pocs;          // after merge_tile_parts: the tile's progression order changes (empty: the main header's)
    // packed packet headers (A.7.4 / A.7.5): this part's PPT markers (Zppt, Ippt); after
    // merge_tile_parts the tile's headers (its PPT data in Zppt order, or its PPM run) in hdrs
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> ppt;
    std::vector<uint8_t> hdrs;
    bool packed = false;
    // the part's COD / COC / QCD / QCC (marker, body), in stream order: the tile's own coding and
    // quantisation (merge_tile_parts appends the later parts')
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> cmark;
};
// POC marker body (A.6.6): per entry RSpoc, CSpoc (1 or 2 bytes), LYEpoc (2), REpoc, CEpoc
// (1 or 2; 0 = 256 with one byte), Ppoc.  Appended to out: CodeStreamDecompress::read_poc
// (:1148-1231) appends to the tcp's list (:1171-1172), so a tile-part POC extends the main
// header's list the tile's tcp was copied from (merge_tile_parts).
template <class Src>
static void parse_poc(Src& S, size_t s, uint32_t L, uint32_t nc, std::vector<Poc>& out) {
    const uint32_t cw = nc <= 256 ? 1 : 2, esz = 5 + 2 * cw;
    if (L < 2 + esz || (L - 2) % esz) throw GkError("corrupt POC marker");
    for (size_t q = s; q + esz <= s + L - 2; q += esz) {
        Poc e;
        e.rs = S.at(q);
        e.cs = cw == 1 ? S.at(q + 1) : S.be16(q + 1);
        e.lye = S.be16(q + 1 + cw);
        e.re = S.at(q + 3 + cw);
        e.ce = cw == 1 ? S.at(q + 4 + cw) : S.be16(q + 4 + cw);
        if (cw == 1 && e.ce == 0) e.ce = 256;
        e.prog = S.at(q + 4 + 2 * cw);
        if (e.prog > 4 || e.re > 33) throw GkError("corrupt POC marker");
        out.push_back(e);
    }
}
// The main header as read, with the tile parts' positions and their tile-part header markers
// (CodeStreamDecompress's tile-part handlers: COD :1725, COC, QCD, QCC; a tile-part RGN,
// read_rgn :1480-1520, is refused rather than skipped)
struct Header {
    Plan want;
    QuantList qcd;                                    // per component (apply_qcd)
    std::vector<std::vector<uint8_t>> qbody;          // per component: its main QCC body, else the QCD's
    size_t first_sot = 0;
    std::vector<TilePart> parts;
    std::vector<std::pair<uint32_t, uint32_t>> tlm;   // (tile, tile-part length) from TLM markers
    std::vector<uint8_t> cod, qcd_body;               // main COD / QCD marker bodies (after Lxxx)
    std::vector<std::vector<uint8_t>> ccod;           // per component: its coding as a COC body states it
                                                      // (Scoc, SPcoc): its main COC, else the COD's
    std::map<uint32_t, std::vector<uint8_t>> ppm;     // PPM bodies by Zppm (PPMMarker::read)
};
// The COD's coding in COC form: Scod's precinct flag, then SPcod from the decomposition levels on
static std::vector<uint8_t> cod_as_coc(const std::vector<uint8_t>& cod) {
    std::vector<uint8_t> v{(uint8_t)(cod[0] & 1)};
    v.insert(v.end(), cod.begin() + 5, cod.end());
    return v;
}
// A component's coding from its COC-form body (read_SPCod_SPCoc): levels, code-block size and
// style, transform, precinct sizes (default 2^15 without the precinct flag)
static void comp_coding(const std::vector<uint8_t>& v, Params::CompCod& k) {
    if (v.size() < 6) throw GkError("corrupt COC marker");
    k.numres = v[1] + 1u; k.cbw = v[2] + 2u; k.cbh = v[3] + 2u; k.cblk_sty = v[4]; k.irrev = v[5] == 0 ? 1 : 0;
    if (k.numres > GK_MAXRLVLS) throw GkError("corrupt COC marker (more than 32 decomposition levels)");
    if (k.cbw > 10 || k.cbh > 10 || k.cbw + k.cbh > 12) throw GkError("corrupt COC marker (code-block size)");
    if ((k.cblk_sty & 0x40) && k.cblk_sty != 0x40) throw GkError("HTJ2K combined with Part-1 mode switches");
    if (k.cblk_sty > 0x7f) throw GkError("unknown code-block style bits");
    for (uint32_t r = 0; r < GK_MAXRLVLS; ++r) { k.prcw[r] = 15; k.prch[r] = 15; }
    if (v[0] & 1) {
        if (v.size() < 6 + k.numres) throw GkError("corrupt COC marker (precinct sizes)");
        for (uint32_t r = 0; r < k.numres; ++r) {
            k.prcw[r] = v[6 + r] & 15; k.prch[r] = v[6 + r] >> 4;
            if (r > 0 && (!k.prcw[r] || !k.prch[r])) throw GkError("COC: precinct exponent 0 above resolution 0");
        }
    }
}

static std::vector<uint8_t> marker_body(ByteSrc& S, size_t s, uint32_t L) {
    std::vector<uint8_t> v(L - 2);
    for (uint32_t k = 0; k + 2 < L; ++k) v[k] = S.at(s + k);
    return v;
}

// Tile-part COD / COC / QCD / QCC set one tile's coding or quantisation (the tile's tcp, a copy of
// the main header's: CodeStreamDecompress read_cod / read_coc / read_qcd / read_qcc); collected per
// tile part here, applied by tile_coding.  COC: Ccoc (1 byte below 257 components, else 2), Scoc
// (precinct flag), then SPcoc laid out as COD's SPcod; QCC: Cqcc, then Sqcc / SPqcc as QCD's body.
// Tile-part RGN: the tile's ROI shift of one component (read_rgn :1476-1520).
static void collect_coding_marker(ByteSrc& S, size_t s, uint32_t m, uint32_t L, const Header& Hd,
                                  std::vector<std::pair<uint32_t, std::vector<uint8_t>>>& out) {
    if (m != 0xff52 && m != 0xff53 && m != 0xff5c && m != 0xff5d && m != 0xff5e) return;
    if (L < 3) throw GkError("corrupt COD/COC/QCD/QCC marker");
    std::vector<uint8_t> b = marker_body(S, s, L);
    const uint32_t nc = Hd.want.nc, cw = nc <= 256 ? 1 : 2;
    if (m == 0xff53 || m == 0xff5d) {
        if (b.size() <= cw) throw GkError("corrupt COC/QCC marker");
        const uint32_t c = cw == 1 ? b[0] : (uint32_t)b[0] << 8 | b[1];
        if (c >= nc) throw GkError("bad component number in COC/QCC");
        if (m == 0xff53 && b.size() < cw + 6) throw GkError("corrupt COC marker");
    }
    if (m == 0xff52 && b.size() < 10) throw GkError("corrupt COD marker");
    if (m == 0xff5e) {   // Crgn, Srgn, SPrgn
        if (b.size() != cw + 2) throw GkError("corrupt RGN marker");
        const uint32_t c = cw == 1 ? b[0] : (uint32_t)b[0] << 8 | b[1];
        if (c >= nc) throw GkError("bad component number in RGN");
        if (b[cw] != 0) throw GkError("only the implicit (maxshift) ROI style is defined");
        if (b[cw + 1] >= 32) throw GkError("unsupported ROI shift");
    }
    out.push_back({m, std::move(b)});
}
// A tile's coding and quantisation: the main header's (cod, ccod, qbody) changed by its tile-part
// markers.  read_cod (CodeStreamDecompress.cpp:2521-2623) sets the tile's stream fields and copies
// its SPcod to every component, read_coc (:2631-2670) one component's, in marker order;
// quantisation follows read_SQcd_SQcc's scoping (Quantizer.cpp:208-235): a tile QCC wins over a
// tile QCD, which wins over the main header's QCC / QCD, in any marker order.  True when the tile
// is coded differently from the main header.
struct TileCoding { std::vector<uint8_t> cod; std::vector<std::vector<uint8_t>> ccod, qbody; std::vector<uint8_t> roi; };
static bool tile_coding(const Header& Hd, const TilePart& H, TileCoding& tc) {
    tc.cod = Hd.cod; tc.ccod = Hd.ccod; tc.qbody = Hd.qbody;
    const uint32_t nc = Hd.want.nc, cw = nc <= 256 ? 1 : 2;
    std::vector<uint8_t> main_roi(nc, 0);
    for (uint32_t c = 0; c < nc && c < Hd.want.p.roishift.size(); ++c) main_roi[c] = Hd.want.p.roishift[c];
    tc.roi = main_roi;
    std::vector<uint8_t> tqcc(nc, 0);
    for (const auto& mk : H.cmark) {
        const std::vector<uint8_t>& v = mk.second;
        if (mk.first == 0xff52) {
            tc.cod = v;
            for (auto& q : tc.ccod) q = cod_as_coc(v);
        } else if (mk.first == 0xff5c) {
            for (uint32_t c = 0; c < nc; ++c) if (!tqcc[c]) tc.qbody[c] = v;
        } else if (mk.first == 0xff5e) {
            tc.roi[cw == 1 ? v[0] : (uint32_t)v[0] << 8 | v[1]] = v[cw + 1];
        } else {
            const uint32_t c = cw == 1 ? v[0] : (uint32_t)v[0] << 8 | v[1];
            std::vector<uint8_t> b(v.begin() + cw, v.end());
            if (mk.first == 0xff5d) { tc.qbody[c] = std::move(b); tqcc[c] = 1; }
            else tc.ccod[c] = std::move(b);
        }
    }
    return tc.cod != Hd.cod || tc.ccod != Hd.ccod || tc.qbody != Hd.qbody || tc.roi != main_roi;
}
// The tiles of the canvas tile grid (B.3)
static uint32_t grid_tiles(const Plan& W) {
    const uint64_t tw = W.p.tw ? W.p.tw : 1, th = W.p.th ? W.p.th : 1;
    return (uint32_t)(((uint64_t)W.x0 + W.w - W.gx0 + tw - 1) / tw * (((uint64_t)W.y0 + W.h - W.gy0 + th - 1) / th));
}
// A tile part's end from its Psot, checked: the next SOT (Lsot 10, a tile index of the grid) or
// EOC must start there, or the stream end.  Grok writes Psot (and TLM) from its rate-control
// simulation's count when its BitIO swallowed a budget failure, a few bytes
// off the part's real length; the nearest such marker within 8 bytes is taken instead.
static size_t resync_part_end(ByteSrc& S, size_t pos, size_t end, uint32_t nt) {
    auto ok = [&](size_t q) {
        if (q == S.len || (q + 2 == S.len && S.be16(q) == 0xffd9)) return true;
        return q + 12 <= S.len && S.be16(q) == 0xff90 && S.be16(q + 2) == 10 && S.be16(q + 4) < nt;
    };
    if (end <= S.len && ok(end)) return end;
    for (size_t d = 1; d <= 8; ++d) {
        if (end >= pos + 14 + d && end - d <= S.len && ok(end - d)) return end - d;
        if (end + d <= S.len && ok(end + d)) return end + d;
    }
    return end;
}
// PPT marker (A.7.5; CodeStreamDecompress::read_ppt): Zppt, then Ippt (packed packet headers of
// the tile); not in a stream with PPM (read_ppt's error)
template <class Hdr> static std::pair<uint32_t, std::vector<uint8_t>> read_ppt(ByteSrc& S, size_t s, uint32_t L, const Hdr& Hd) {
    if (L < 3) throw GkError("corrupt PPT marker");
    if (!Hd.ppm.empty()) throw GkError("PPT marker in a stream with PPM markers");
    std::vector<uint8_t> v(L - 3);
    for (uint32_t k = 0; k + 3 < L; ++k) v[k] = S.at(s + 1 + k);
    return {S.at(s), std::move(v)};
}
// The tile parts by the SOT chain (Psot of each), their tile-part header markers read
template <class Hdr> static void walk_sot_chain(ByteSrc& S, Hdr& Hd) {
    Plan& W = Hd.want;
    const uint32_t nt = grid_tiles(W);
    size_t pos = Hd.first_sot;
    while (pos + 12 <= S.len && S.be16(pos) == 0xff90) {
        const uint32_t isot = S.be16(pos + 4), psot = S.be32(pos + 6);
        size_t end = psot ? pos + psot : (S.len >= 2 ? S.len - 2 : S.len);
        if (end > S.len + 8 || end < pos + 14) throw GkError("corrupt SOT (Psot)");
        end = resync_part_end(S, pos, end, nt);
        if (end > S.len) throw GkError("corrupt SOT (Psot)");
        size_t j = pos + 12;
        std::vector<Poc> tpoc;
        std::vector<std::pair<uint32_t, std::vector<uint8_t>>> tppt, tmark;
        while (j + 4 <= end && S.be16(j) != 0xff93) {
            if (S.be16(j) == 0xff5f) parse_poc(S, j + 4, S.be16(j + 2), W.nc, tpoc);   // tile-part POC
            if (S.be16(j) == 0xff61) tppt.push_back(read_ppt(S, j + 4, S.be16(j + 2), Hd));
            collect_coding_marker(S, j + 4, S.be16(j), S.be16(j + 2), Hd, tmark);
            j += 2 + S.be16(j + 2);
        }
        if (j + 2 > end || S.be16(j) != 0xff93) throw GkError("missing SOD");
        Hd.parts.push_back({isot, pos, j + 2, end, {}, {}, S.at(pos + 10), std::move(tpoc)});
        Hd.parts.back().ppt = std::move(tppt);
        Hd.parts.back().cmark = std::move(tmark);
        pos = end;
    }
}
// A TLM whose lengths do not lead from SOT to SOT (read_tile_part_headers)
struct TlmMismatch : GkError { TlmMismatch() : GkError("TLM does not match the SOT markers") {} };

// COD body (Scod, SGcod, SPcod; read_cod :2521-2623) into the stream-level fields (progression,
// SOP / EPH, layers, MCT) and the default coding of p
static void read_cod_fields(const std::vector<uint8_t>& b, Params& p) {
    if (b.size() < 10) throw GkError("corrupt COD marker");
    const uint32_t scod = b[0];
    if (b[1] > 4) throw GkError("corrupt COD marker (progression order)");
    p.prog = b[1];
    p.sop_eph = scod & 6;
    p.nlayers = (uint32_t)b[2] << 8 | b[3];
    if (!p.nlayers) throw GkError("corrupt COD marker (no layers)");
    p.mct = b[4];
    // SGcod MCT: 0 none, 1 RCT / ICT; 2 = a Part-2 array transform (MCT / MCC / MCO markers,
    // Grok's decompress_custom), not on this path
    if (p.mct > 1) throw GkError("Part-2 array multiple-component transforms are not supported on this path");
    p.numres = b[5] + 1;
    // at most 32 decomposition levels (CodeStreamDecompress.cpp:1733)
    if (p.numres > GK_MAXRLVLS) throw GkError("corrupt COD marker (more than 32 decomposition levels)");
    p.cbw = b[6] + 2; p.cbh = b[7] + 2;
    if (p.cbw > 10 || p.cbh > 10 || p.cbw + p.cbh > 12) throw GkError("corrupt COD marker (code-block size)");
    p.cblk_sty = b[8];
    if ((p.cblk_sty & GK_STY_HT) && p.cblk_sty != GK_STY_HT)
        throw GkError("HTJ2K combined with Part-1 mode switches");   // CodeStreamDecompress.cpp:1781-1788
    if (p.cblk_sty > 0x7f) throw GkError("unknown code-block style bits");
    p.irrev = b[9] == 0 ? 1 : 0;
    p.custom_prc = false;
    for (int k = 0; k < GK_MAXRLVLS; ++k) { p.prcw[k] = 15; p.prch[k] = 15; }
    if (scod & 1) {
        if (b.size() < 10 + p.numres) throw GkError("corrupt COD marker (precinct sizes)");
        p.custom_prc = true;
        for (uint32_t r = 0; r < p.numres; ++r) {
            const uint32_t v = b[10 + r]; p.prcw[r] = v & 15; p.prch[r] = v >> 4;
            if (r > 0 && (!p.prcw[r] || !p.prch[r])) throw GkError("COD: precinct exponent 0 above resolution 0");
        }
    }
}
// The coding of every component (Params::cc when they differ) and the quantisation (Hd.qcd) from
// the COD, the per-component COC-form bodies and the quantisation bodies; MCT restrictions checked
static void apply_coding(Header& Hd) {
    Plan& W = Hd.want;
    W.p.cc.clear();
    bool differ = false;
    for (uint32_t c = 0; c < W.nc; ++c) differ = differ || Hd.ccod[c] != Hd.ccod[0] || Hd.ccod[c] != cod_as_coc(Hd.cod);
    if (differ) {
        W.p.cc.resize(W.nc);
        for (uint32_t c = 0; c < W.nc; ++c) comp_coding(Hd.ccod[c], W.p.cc[c]);
        // the inverse MCT picks RCT / ICT by component 0's transform (TileProcessor::mctDecompress)
        if (W.p.mct && W.nc >= 3 && (W.p.cc[1].irrev != W.p.cc[0].irrev || W.p.cc[2].irrev != W.p.cc[0].irrev))
            throw GkError("MCT over components with different transforms is not supported");
    }
    if (W.p.mct && W.nc >= 3 && (W.c_prec(1) != W.c_prec(0) || W.c_prec(2) != W.c_prec(0) ||
                                 W.c_sgnd(1) != W.c_sgnd(0) || W.c_sgnd(2) != W.c_sgnd(0)))
        throw GkError("MCT over components of different precisions or signs is not supported on this path");
    Hd.qcd.clear();
    for (uint32_t c = 0; c < W.nc; ++c) parse_quant(Hd.qbody[c], W.p.c_numres(c), Hd.qcd);
}

static void parse_header(ByteSrc& S, Header& Hd) {
    size_t i = 0;
    if (S.len < 4 || S.be16(0) != 0xff4f) throw GkError("not a J2K codestream (no SOC)");
    i = 2;
    Plan& W = Hd.want;
    for (int k = 0; k < GK_MAXRLVLS; ++k) { W.p.prcw[k] = 15; W.p.prch[k] = 15; }
    bool have_siz = false, have_cod = false;
    std::vector<size_t> coc_qcc;   // COC: checked against COD once the main header is read
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> qcc;   // main-header QCC: (component, Sqcc + SPqcc)
    while (i + 4 <= S.len) {
        uint32_t m = S.be16(i);
        if (m == 0xff90) { Hd.first_sot = i; break; }
        uint32_t L = S.be16(i + 2);
        size_t s = i + 4;
        if (L < 2 || i + 2 + L > S.len) throw GkError("corrupt main header (marker length)");
        if (m == 0xff51) {
            if (L < 41) throw GkError("corrupt SIZ marker");
            const uint32_t X1 = S.be32(s + 2), Y1 = S.be32(s + 6);
            W.x0 = S.be32(s + 10); W.y0 = S.be32(s + 14); W.gx0 = S.be32(s + 26); W.gy0 = S.be32(s + 30);
            if (X1 <= W.x0 || Y1 <= W.y0) throw GkError("corrupt SIZ marker (empty image)");
            W.w = X1 - W.x0; W.h = Y1 - W.y0;
            W.p.tw = S.be32(s + 18); W.p.th = S.be32(s + 22);
            if (!W.p.tw || !W.p.th) throw GkError("bad tile size");
            // B.3 (CodeStreamDecompress::read_siz): grid origin at or above-left of the image, the
            // first tile overlapping it
            if (W.gx0 > W.x0 || W.gy0 > W.y0 || (uint64_t)W.gx0 + W.p.tw <= W.x0 || (uint64_t)W.gy0 + W.p.th <= W.y0)
                throw GkError("corrupt SIZ marker (tile grid offset)");
            if ((uint64_t)W.gx0 + W.p.tw >= X1 && (uint64_t)W.gy0 + W.p.th >= Y1) W.p.tw = W.p.th = 0;   // one tile
            W.nc = S.be16(s + 34);
            if (W.nc == 0 || W.nc > 255 || L < 38 + 3 * W.nc) throw GkError("corrupt SIZ marker (component count)");
            if (!W.w || !W.h) throw GkError("corrupt SIZ marker (empty image)");
            uint32_t sz = S.at(s + 36);
            W.prec = (sz & 0x7f) + 1; W.sgnd = (sz & 0x80) ? 1 : 0;
            if (W.prec > 31) throw GkError("component precision > 31 bits not supported");
            W.cdx.assign(W.nc, 1); W.cdy.assign(W.nc, 1);
            for (uint32_t c = 0; c < W.nc; ++c) {
                // XRsiz / YRsiz: 1..255 (read_siz)
                W.cdx[c] = S.at(s + 37 + 3 * c); W.cdy[c] = S.at(s + 38 + 3 * c);
                if (!W.cdx[c] || !W.cdy[c]) throw GkError("corrupt SIZ marker (component subsampling 0)");
            }
            if (!W.subsampled()) { W.cdx.clear(); W.cdy.clear(); }
            // Ssiz per component: precisions / signs may differ (each component DC-shifted and
            // clamped by its own, Quantizer steps from its own); prec becomes the largest
            W.cprec.assign(W.nc, 0); W.csgnd.assign(W.nc, 0);
            bool mixed = false;
            for (uint32_t c = 0; c < W.nc; ++c) {
                const uint32_t v = S.at(s + 36 + 3 * c);
                W.cprec[c] = (uint8_t)((v & 0x7f) + 1); W.csgnd[c] = (uint8_t)(v >> 7);
                if (W.cprec[c] > 31) throw GkError("component precision > 31 bits not supported");
                mixed = mixed || W.cprec[c] != W.prec || W.csgnd[c] != W.sgnd;
                W.prec = std::max<uint32_t>(W.prec, W.cprec[c]);
            }
            if (!mixed) { W.cprec.clear(); W.csgnd.clear(); }
            have_siz = true;
        } else if (m == 0xff52) {
            if (L < 12) throw GkError("corrupt COD marker");
            Hd.cod = marker_body(S, s, L);
            read_cod_fields(Hd.cod, W.p);
            have_cod = true;
        } else if (m == 0xff5c) {
            if (L < 4) throw GkError("corrupt QCD marker");
            W.p.numgbits = S.at(s) >> 5;
            if ((S.at(s) & 0x1f) > 2) throw GkError("corrupt QCD marker (quantisation style)");
            Hd.qcd_body = marker_body(S, s, L);
        } else if (m == 0xff55) {   // TLM (TileLengthMarkers::read, cache/LengthCache.cpp)
            const uint32_t stlm = S.at(s + 1), st = (stlm >> 4) & 3, sp = (stlm >> 6) & 1;
            const uint32_t esz = st + (sp ? 4 : 2);
            size_t e = s + 2;
            uint32_t tnext = Hd.tlm.empty() ? 0 : Hd.tlm.back().first + 1;
            while (e + esz <= s + L - 2) {
                uint32_t t = st == 0 ? tnext : (st == 1 ? S.at(e) : S.be16(e));
                uint32_t len = sp ? S.be32(e + st) : S.be16(e + st);
                Hd.tlm.push_back({t, len});
                tnext = t + 1;
                e += esz;
            }
        } else if (m == 0xff5f) {   // POC in the main header: every tile's packet order
            parse_poc(S, s, L, W.nc, W.p.pocs);
        } else if (m == 0xff5e) {   // RGN (CodeStreamDecompress::read_rgn :1480-1520)
            const uint32_t cw = W.nc <= 256 ? 1 : 2;
            if (L != 4 + cw) throw GkError("corrupt RGN marker");
            const uint32_t c = cw == 1 ? S.at(s) : S.be16(s);
            if (c >= W.nc) throw GkError("bad component number in RGN");
            if (S.at(s + cw) != 0) throw GkError("only the implicit (maxshift) ROI style is defined");
            const uint32_t shift = S.at(s + cw + 1);
            if (shift >= 32) throw GkError("unsupported ROI shift");
            if (W.p.roishift.size() < W.nc) W.p.roishift.resize(W.nc, 0);
            W.p.roishift[c] = (uint8_t)shift;
        } else if (m == 0xff5d) {   // QCC (A.6.5): one component's quantisation replaces the QCD's
            if (!have_siz) throw GkError("QCC before SIZ");
            const uint32_t cw = W.nc <= 256 ? 1 : 2;
            if (L < 4 + cw) throw GkError("corrupt QCC marker");
            const uint32_t c = cw == 1 ? S.at(s) : S.be16(s);
            if (c >= W.nc) throw GkError("bad component number in QCC");
            std::vector<uint8_t> b = marker_body(S, s, L);
            qcc.push_back({c, std::vector<uint8_t>(b.begin() + cw, b.end())});
        } else if (m == 0xff53) {
            coc_qcc.push_back(i);
        } else if (m == 0xff72 || m == 0xff73 || (m >= 0xff74 && m <= 0xff79)) {
            // Part-2 extensions (DFS, ADS, MCT, MCC, NLT, MCO, CBD, ATK: ISO 15444-2 A.2) change
            // how the stream decodes; refused rather than ignored
            throw GkError("Part-2 (ISO 15444-2) extension markers are not supported on this path");
        } else if (m == 0xff60) {   // PPM (A.7.4): Zppm, then (Nppm, Ippm) runs
            if (L < 3) throw GkError("corrupt PPM marker");
            if (!Hd.ppm.emplace(S.at(s), marker_body(S, s + 1, L - 1)).second) throw GkError("PPM: Zppm read twice");
        }
        i += 2 + L;
    }
    if (!have_siz || !have_cod || Hd.qcd_body.empty() || !Hd.first_sot) throw GkError("incomplete main header");
    // per component: the QCD's quantisation, replaced by its main-header QCC (a main QCC takes
    // precedence over the main QCD in any marker order, Quantizer.cpp:215-235)
    Hd.qbody.assign(W.nc, Hd.qcd_body);
    for (auto& q : qcc) Hd.qbody[q.first] = q.second;
    // per component: the COD's coding, replaced by its main-header COC (A.6.2; read_coc fills the
    // component's tccp, a main COC winning over the main COD in either order)
    Hd.ccod.assign(W.nc, cod_as_coc(Hd.cod));
    for (size_t k : coc_qcc) {
        const uint32_t L = S.be16(k + 2), cw = W.nc <= 256 ? 1 : 2;
        const std::vector<uint8_t> b = marker_body(S, k + 4, L);
        if (b.size() < cw + 6) throw GkError("corrupt COC marker");
        const uint32_t c = cw == 1 ? b[0] : (uint32_t)b[0] << 8 | b[1];
        if (c >= W.nc) throw GkError("bad component number in COC/QCC");
        Hd.ccod[c].assign(b.begin() + cw, b.end());
    }
    apply_coding(Hd);
    // tile parts: SOT (Isot, Psot, TPsot, TNsot), tile-part header markers (PLT, ...), SOD, packets
    // (CodeStreamDecompress SOT/SOD handlers; TLM and PLT are only needed for random access)
    size_t pos = Hd.first_sot;
    bool tlm_ok = !Hd.tlm.empty() && S.dev;
    if (tlm_ok) {
        // device-resident stream with TLM: tile-part positions without walking the SOT chain;
        // the tile-part headers are fetched in one batch by the decoder (data = 0 until then).
        // A TLM that does not fit the stream (e.g. a full-image TLM in front of a subset of
        // the tile parts) is ignored and the SOT chain is walked instead.
        for (auto& tl : Hd.tlm) {
            const size_t end = pos + tl.second;
            if (tl.second < 14 || end > S.len) { tlm_ok = false; break; }
            Hd.parts.push_back({tl.first, pos, 0, end, {}});
            pos = end;
        }
        if (!tlm_ok) { Hd.parts.clear(); pos = Hd.first_sot; }
    }
    if (!tlm_ok) walk_sot_chain(S, Hd);
    if (Hd.parts.empty()) throw GkError("no tile parts");
}

// Device-resident codestream: copy scattered ranges (tile-part headers, packet headers) to
// the host with one gather launch and one D2H copy, and register them with the byte source.
static void fetch_ranges(gk_ctx* ctx, ByteSrc& S, const std::vector<std::pair<size_t, size_t>>& rg, HostBuf& hb,
                         DevBuf& db) {
    if (rg.empty()) return;
    size_t tot = 0;
    for (auto& r : rg) tot += r.second;
    uint8_t* dst = (uint8_t*)db.get(tot + 64);
    uint64_t* hs = (uint64_t*)ctx->hseg.get(rg.size() * 24 + 8);
    size_t o = 0;
    for (size_t i = 0; i < rg.size(); ++i) { hs[3 * i] = rg[i].first; hs[3 * i + 1] = o; hs[3 * i + 2] = rg[i].second; o += rg[i].second; }
    uint64_t* ds = (uint64_t*)ctx->dseg.get(rg.size() * 24 + 8);
    HIPCHK(hipMemcpyAsync(ds, hs, rg.size() * 24, hipMemcpyHostToDevice, ctx->st));
    gk_launch_gather(ctx->st, S.dev, dst, ds, (uint32_t)rg.size());
    uint8_t* h = (uint8_t*)hb.get(tot + 64);
    HIPCHK(hipMemcpyAsync(h, dst, tot, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    std::vector<ByteSrc::Region> regs;
    o = 0;
    for (auto& r : rg) { regs.push_back({r.first, r.second, h + o}); o += r.second; }
    S.add_regions(regs);
}

// Tile-part headers of parts located through TLM: SOD position and PLT packet lengths
// (PacketLengthMarkers::readPLT: Zplt, then 7-bit groups MSB first, bit 7 = continuation).
static void read_tile_part_headers(gk_ctx* ctx, ByteSrc& S, Header& Hd) {
    const uint32_t nc = Hd.want.nc;
    std::vector<std::pair<size_t, size_t>> rg;
    for (auto& TP : Hd.parts)
        if (!TP.data) rg.push_back({TP.sot, std::min<size_t>(TP.end - TP.sot, 4096)});
    fetch_ranges(ctx, S, rg, ctx->hstage1, ctx->dstage1);
    for (auto& TP : Hd.parts) {
        if (TP.data) continue;
        if (S.be16(TP.sot) != 0xff90 || S.be16(TP.sot + 4) != TP.tile || S.be32(TP.sot + 6) != TP.end - TP.sot)
            throw TlmMismatch();
        TP.tpsot = S.at(TP.sot + 10);
        size_t j = TP.sot + 12;
        while (j + 4 <= TP.end && S.be16(j) != 0xff93) {
            const uint32_t m = S.be16(j), L = S.be16(j + 2);
            if (m == 0xff5f) parse_poc(S, j + 4, L, nc, TP.pocs);   // tile-part POC
            if (m == 0xff61) TP.ppt.push_back(read_ppt(S, j + 4, L, Hd));
            collect_coding_marker(S, j + 4, m, L, Hd, TP.cmark);
            if (m == 0xff58) {
                uint32_t v = 0;
                for (size_t q = j + 5; q < j + 2 + L; ++q) {
                    const uint32_t b = S.at(q);
                    v = (v << 7) | (b & 0x7f);
                    if (!(b & 0x80)) { TP.plt.push_back(v); v = 0; }
                }
            }
            j += 2 + L;
        }
        if (j + 2 > TP.end || S.be16(j) != 0xff93) throw GkError("missing SOD");
        TP.data = j + 2;
    }
}

// With PLT, every packet's start is known: fetch the first bytes of each packet (its header;
// bound from the packet's code-block count) in one batch before T2 parses them.
static void prefetch_packet_headers(gk_ctx* ctx, ByteSrc& S, const Plan& P, const Header& Hd) {
    std::vector<std::pair<size_t, size_t>> rg;
    for (const auto& TP : Hd.parts) {
        if (TP.plt.empty() || TP.tile >= P.tiles.size()) continue;
        const TileG& T = P.tiles[TP.tile];
        size_t pos = TP.data, end = TP.end, k = 0, nextp = 0;
        for (const PacketRef& pr : packet_order(P, T, P.p.nlayers, TP.pocs.empty() ? &P.p.pocs : &TP.pocs)) {
            if (k >= TP.plt.size()) break;
            const ResG& R = T.comps[pr.c].res[pr.r];
            while (pos >= end && nextp < TP.more.size()) { pos = TP.more[nextp].first; end = TP.more[nextp].second; ++nextp; }
            size_t nblk = 0;
            for (uint32_t bi = 0; bi < R.bands.size(); ++bi) nblk += (size_t)R.prc[bi][pr.pi].cw * R.prc[bi][pr.pi].ch;
            const size_t len = TP.plt[k++];
            if (pos + len > end) return;   // inconsistent PLT: fall back to page fetches
            rg.push_back({pos, std::min(len, 72 + 16 * nblk)});   // (SOP / EPH included)
            pos += len;
        }
    }
    fetch_ranges(ctx, S, rg, ctx->hstage2, ctx->dstage2);
}

// win (optional): x0, y0, x1, y1 — decode only the tiles intersecting the window and write
// the window into comps (whose element 0 is the window's top-left sample).
// A tile's tile parts in TPsot order become one entry: the first part's range, the others
// in `more`, PLT lengths concatenated (packets never straddle tile parts, A.4.2).  The tile's
// progression order changes are the main header's list extended by each part's POC in turn
// (read_poc appends to the tile's copy of the main tcp, CodeStreamDecompress.cpp:1171-1172;
// OpenJPEG's opj_j2k_read_poc does the same).  PLT is not used for such a tile: Grok lists its
// lengths in the tile's own progression, not in the order the packets are written
// (TileProcessor::pcrdBisectSimple's final simulation, T2Compress.cpp:427-428).
static void merge_tile_parts(Header& Hd) {
    std::unordered_map<uint32_t, size_t> first;
    std::vector<TilePart> out;
    for (TilePart& TP : Hd.parts) {
        auto it = first.find(TP.tile);
        if (it == first.end()) {
            if (TP.tpsot != 0) throw GkError("tile parts out of order (first TPsot is not 0)");
            first.emplace(TP.tile, out.size());
            out.push_back(std::move(TP));
            continue;
        }
        TilePart& H = out[it->second];
        if (TP.tpsot != H.more.size() + 1) throw GkError("tile parts out of order (TPsot)");
        H.more.push_back({TP.data, TP.end});
        for (auto& e : TP.ppt) H.ppt.push_back(std::move(e));
        for (auto& e : TP.cmark) H.cmark.push_back(std::move(e));
        H.plt.insert(H.plt.end(), TP.plt.begin(), TP.plt.end());
        H.pocs.insert(H.pocs.end(), TP.pocs.begin(), TP.pocs.end());
    }
    // packed packet headers: PPM's Nppm runs (PPMMarker::merge), the k-th taken by tile k (T2Decompress
    // indexes m_tile_packet_headers by tile, :257-266: kept to one tile part per tile), or the tile's
    // PPT data in Zppt order (merge_ppt, one index space per tile)
    std::vector<std::vector<uint8_t>> runs;
    if (!Hd.ppm.empty()) {
        std::vector<uint8_t> v;
        for (auto& kv : Hd.ppm) v.insert(v.end(), kv.second.begin(), kv.second.end());
        for (size_t at = 0; at < v.size();) {
            if (v.size() - at < 4) throw GkError("PPM: not enough bytes for Nppm");
            const uint32_t n = (uint32_t)v[at] << 24 | (uint32_t)v[at + 1] << 16 | (uint32_t)v[at + 2] << 8 | v[at + 3];
            at += 4;
            if (v.size() - at < n) throw GkError("PPM: packed headers shorter than Nppm");
            runs.emplace_back(v.begin() + at, v.begin() + at + n);
            at += n;
        }
    }
    for (TilePart& H : out) {
        if (!Hd.ppm.empty()) {
            if (!H.more.empty()) throw GkError("PPM with several tile parts per tile is not supported on this path");
            if (H.tile >= runs.size()) throw GkError("PPM has no packed packet headers for a tile");
            H.hdrs = runs[H.tile]; H.packed = true;
        } else if (!H.ppt.empty()) {
            std::map<uint32_t, std::vector<uint8_t>> z;
            for (auto& e : H.ppt)
                if (!z.emplace(e.first, std::move(e.second)).second) throw GkError("PPT: Zppt read twice");
            for (auto& kv : z) H.hdrs.insert(H.hdrs.end(), kv.second.begin(), kv.second.end());
            H.packed = true;
        }
        if (H.packed) H.plt.clear();   // (packet lengths are not used with packed headers)
    }
    const std::vector<Poc>& main_pocs = Hd.want.p.pocs;
    for (TilePart& H : out) {
        // PLT lengths that do not add up to the tile's data are not used (R-BUG-8 streams)
        uint64_t plt_sum = 0, data = H.end - H.data;
        for (uint32_t v : H.plt) plt_sum += v;
        for (auto& m : H.more) data += m.second - m.first;
        if (!H.plt.empty() && plt_sum != data) H.plt.clear();
        if (!H.pocs.empty()) H.pocs.insert(H.pocs.begin(), main_pocs.begin(), main_pocs.end());
        if (H.pocs.size() > GK_MAXRLVLS) throw GkError("too many progression order changes (read_poc: at most 33)");
        if (!H.pocs.empty() || !main_pocs.empty()) H.plt.clear();
    }
    Hd.parts.swap(out);
}

// A pass over some of the stream's tiles (tiles coded with their own parameters): the tiles it
// decodes, their coding (else the main header's), the output frame's origin (image-relative; the
// caller's window origin) and the inverse rule of the whole call
struct TilePass {
    std::vector<uint8_t> tiles;   // by tile index: decoded in this pass
    const TileCoding* coding = nullptr;
    uint32_t fx = 0, fy = 0;
    bool partial = false;
};
static void decode_impl(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, void* const* comps,
                        const uint32_t* strides, uint32_t sample_bytes, int out_on_device, const uint32_t* win = nullptr,
                        const TilePass* pass = nullptr) {
    hipStream_t st = ctx->st;
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[0], st));
    const uint8_t* const cs_in = cs;
    const size_t len_in = len;
    // Grok's partial-tile inverse (its single odd 5/3 sample shifted, not halved) follows a window
    // set with setDecompressWindow; decompressTile without one keeps the whole-tile rule
    ctx->dwt_partial = pass ? pass->partial : win != nullptr && !ctx->win_whole_tile;
    // GK_PROFILE=1: host phase times of the decode (stderr)
    static const bool prof = getenv("GK_PROFILE") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto h0 = now();
    ByteSrc S;
    S.len = len; S.st = st;
    if (cs_on_device) S.dev = cs; else S.host = cs;
    {
        size_t joff = 0, jlen = 0;
        if (jp2_locate(S, joff, jlen)) {   // JP2 file: decode its codestream box
            cs += joff; len = jlen;
            S = ByteSrc(); S.len = len; S.st = st;
            if (cs_on_device) S.dev = cs; else S.host = cs;
        }
    }
    Header Hd;
    parse_header(S, Hd);
    if (pass && pass->coding) {   // the pass's tiles: their own coding and quantisation
        Hd.cod = pass->coding->cod; Hd.ccod = pass->coding->ccod; Hd.qbody = pass->coding->qbody;
        read_cod_fields(Hd.cod, Hd.want.p);
        Hd.want.p.roishift.assign(pass->coding->roi.begin(), pass->coding->roi.end());
        bool any_roi = false;
        for (uint8_t r : pass->coding->roi) any_roi = any_roi || r;
        if (!any_roi) Hd.want.p.roishift.clear();
        apply_coding(Hd);
    }
    if (Hd.want.nc < 3) Hd.want.p.mct = 0;
    ensure_plan(ctx, Hd.want);
    Plan& P = ctx->plan;
    if (Hd.qcd != ctx->band_qcd) { apply_qcd(P, Hd.qcd); ctx->band_qcd = Hd.qcd; }
    // the Part-1 decoders hold twice the magnitude plus the half-bit, (2M+1) << q, in an int32:
    // a band (ROI shift included) of more than 30 bit-planes cannot be held (every tile has the
    // same bands as tile 0)
    for (uint32_t c = 0; c < P.nc; ++c)
        if (!P.p.c_ht(c))
            for (const ResG& R : P.tiles[0].comps[c].res)
                for (const BandG& B : R.bands)
                    if (B.numbps > 30) throw GkError("more than 30 band bit-planes (ROI shift included) not supported");
    const uint32_t red = ctx->dec_reduce;
    if (red >= P.min_numres()) throw GkError("reduce must be less than the number of resolutions");
    // subsampled components: every component plane at its own size, rectangles on its grid
    auto keep_window = [&]() {   // keep only the tile parts of tiles intersecting the window
        if (!win) return;
        if (win[0] >= win[2] || win[1] >= win[3] || win[2] > P.w || win[3] > P.h) throw GkError("bad decode window");
        std::vector<TilePart> keep;
        for (auto& TP : Hd.parts) {
            if (TP.tile >= P.tiles.size()) throw GkError("corrupt SOT (tile index)");
            const TileG& T = P.tiles[TP.tile];   // (canvas tile against the image-relative window)
            if (T.x0 - P.x0 < win[2] && win[0] < T.x1 - P.x0 && T.y0 - P.y0 < win[3] && win[1] < T.y1 - P.y0)
                keep.push_back(std::move(TP));
        }
        Hd.parts.swap(keep);
        if (Hd.parts.empty()) throw GkError("no tile part intersects the window");
    };
    keep_window();
    if (S.dev) {
        try {
            read_tile_part_headers(ctx, S, Hd);
        } catch (const TlmMismatch&) {   // (R-BUG-8 streams) the SOT chain instead
            Hd.parts.clear();
            walk_sot_chain(S, Hd);
            keep_window();
        }
    }
    merge_tile_parts(Hd);
    if (pass) {
        std::vector<TilePart> keep;
        for (auto& TP : Hd.parts)
            if (TP.tile < pass->tiles.size() && pass->tiles[TP.tile]) keep.push_back(std::move(TP));
        Hd.parts.swap(keep);
        if (Hd.parts.empty()) throw GkError("internal: a tile pass without tiles");
    } else {
        // tiles coded with their own parameters (tile-part COD / COC / QCD / QCC): the tiles with
        // the main header's coding in one pass, then each other tile in a pass of its own, through
        // its rectangle (clipped to the window) into the same output frame.  Passes write disjoint
        // tile rectangles in stream order on one HIP stream; a tile absent from a pass's tile
        // rectangle is written as zero by that pass before its own pass writes it.
        std::vector<TileCoding> own(Hd.parts.size());
        std::vector<uint8_t> differs(Hd.parts.size(), 0);
        bool any = false;
        for (size_t q = 0; q < Hd.parts.size(); ++q) {
            if (Hd.parts[q].cmark.empty()) continue;
            differs[q] = tile_coding(Hd, Hd.parts[q], own[q]);
            any = any || differs[q];
        }
        if (any) {
            const size_t ntl = P.tiles.size();
            const uint32_t full[4] = {0, 0, P.w, P.h};
            const uint32_t* wv = win ? win : full;
            TilePass base;
            base.tiles.assign(ntl, 0);
            base.fx = win ? win[0] : 0; base.fy = win ? win[1] : 0;
            base.partial = ctx->dwt_partial;
            bool main_tiles = false;
            for (size_t q = 0; q < Hd.parts.size(); ++q)
                if (!differs[q] && Hd.parts[q].tile < ntl) { base.tiles[Hd.parts[q].tile] = 1; main_tiles = true; }
            if (main_tiles) decode_impl(ctx, cs_in, len_in, cs_on_device, comps, strides, sample_bytes, out_on_device, win, &base);
            for (size_t q = 0; q < Hd.parts.size(); ++q) {
                if (!differs[q]) continue;
                const uint32_t t = Hd.parts[q].tile;
                if (t >= ntl) throw GkError("corrupt SOT (tile index)");
                const TileG& T = P.tiles[t];
                const uint32_t tw[4] = {std::max(T.x0 - P.x0, wv[0]), std::max(T.y0 - P.y0, wv[1]),
                                        std::min(T.x1 - P.x0, wv[2]), std::min(T.y1 - P.y0, wv[3])};
                if (tw[0] >= tw[2] || tw[1] >= tw[3]) continue;
                TilePass tp = base;
                tp.tiles.assign(ntl, 0);
                tp.tiles[t] = 1;
                tp.coding = &own[q];
                decode_impl(ctx, cs_in, len_in, cs_on_device, comps, strides, sample_bytes, out_on_device, tw, &tp);
            }
            return;
        }
    }
    if (S.dev) prefetch_packet_headers(ctx, S, P, Hd);
    // ---- tiles present, their rectangle, and the code-blocks that reach the output
    std::vector<int32_t> part_of(P.tiles.size(), -1);
    for (size_t q = 0; q < Hd.parts.size(); ++q) {
        const TilePart& TPt = Hd.parts[q];
        if (TPt.tile >= P.tiles.size()) throw GkError("corrupt SOT (tile index)");
        if (part_of[TPt.tile] >= 0) throw GkError("corrupt stream (tile parts of one tile merged twice)");
        part_of[TPt.tile] = (int32_t)q;
    }
    uint32_t ib = P.ntx, ie = 0, jb = P.nty, je = 0;
    for (const TilePart& TPt : Hd.parts) {
        const uint32_t t = TPt.tile;
        ib = std::min(ib, t % P.ntx); ie = std::max(ie, t % P.ntx + 1);
        jb = std::min(jb, t / P.ntx); je = std::max(je, t / P.ntx + 1);
    }
    // work planes cover the tile rectangle only (tiles of the rectangle without a tile part
    // decode as zero); the output region is the rectangle, clipped to the window
    const TileG& Tfirst = P.tiles[(size_t)jb * P.ntx + ib];
    const TileG& Tlast = P.tiles[(size_t)(je - 1) * P.ntx + ie - 1];
    const Region RG = make_region(Tfirst.x0 - P.x0, Tfirst.y0 - P.y0, Tlast.x1 - P.x0, Tlast.y1 - P.y0);   // image-relative
    uint32_t rx0 = RG.x0, ry0 = RG.y0, rx1 = RG.x0 + RG.w, ry1 = RG.y0 + RG.h, ox = 0, oy = 0;
    if (win) {
        rx0 = std::max(rx0, win[0]); ry0 = std::max(ry0, win[1]); rx1 = std::min(rx1, win[2]); ry1 = std::min(ry1, win[3]);
        ox = win[0]; oy = win[1];
    }
    if (pass) { ox = pass->fx; oy = pass->fy; }
    const uint32_t ncols = rx1 - rx0, nrows = ry1 - ry0;
    // the region on each sampling group's grid (RG itself without subsampling)
    std::vector<Region> RGg;
    for (const SGroup& G : P.groups) RGg.push_back(group_region(P, RG, G));
    // Per tile: which code-blocks reach [rx0, rx1) x [ry0, ry1).  Inverse lifting reconstructs
    // sample n of a level from low/high coefficients within a few positions of n/2 (5/3: the
    // update/predict steps reach one neighbour each; 9/7: four steps), so the coefficients a
    // window needs at each level are its projection padded by that reach, clamped to the band
    // (the padded band window of TileComponentWindowBuffer / T2Decompress.cpp:55-116).  Blocks
    // outside are not decoded (their samples only feed outputs outside the window), and with
    // PLT a packet none of whose blocks is needed is skipped unparsed.
    // (on the canvas: the output rectangle moved by the image origin)
    const uint32_t cx0 = rx0 + P.x0, cy0 = ry0 + P.y0, cx1 = rx1 + P.x0, cy1 = ry1 + P.y0;
    auto block_needed = [&](const TileG& T, std::vector<uint8_t>& need) {
        need.assign(T.b1 - T.b0, 1);
        if (!win || (cx0 <= T.x0 && T.x1 <= cx1 && cy0 <= T.y0 && T.y1 <= cy1)) return;
        // per sampling group (its grid, levels and transform; the components of a group share
        // their geometry): lo[a][l], hi[a][l] = needed [begin, end) in level-l low / high band
        // coordinates, axis a
        const size_t ng = P.groups.size();
        std::vector<std::array<std::array<std::array<uint32_t, 2>, GK_MAXRLVLS + 1>, 2>> LO(ng), HI(ng);
        std::vector<uint8_t> done(ng, 0);
        for (uint32_t c = 0; c < P.nc; ++c) {
        const uint32_t g = P.group_of[c];
        if (done[g]) continue;
        done[g] = 1;
        const SGroup& SG = P.groups[g];
        const uint32_t Lv = SG.numres - 1, pad = SG.irrev ? 4 : 2;
        auto& lo = LO[g];
        auto& hi = HI[g];
        const CompG& C0 = T.comps[c];
        for (int ax = 0; ax < 2; ++ax) {
            // the window and the tile on the group's grid
            const uint32_t d = ax ? SG.dy : SG.dx;
            uint32_t s0 = ceildiv(ax ? std::max(cy0, T.y0) : std::max(cx0, T.x0), d);
            uint32_t s1 = ceildiv(ax ? std::min(cy1, T.y1) : std::min(cx1, T.x1), d);
            lo[ax][0][0] = s0; lo[ax][0][1] = s1;
            for (uint32_t l = 1; l <= Lv; ++l) {
                const ResG& Rl = C0.res[SG.numres - l];       // resolution holding level-l bands
                const ResG& Rlow = C0.res[SG.numres - 1 - l]; // its low-pass image
                const uint32_t c0 = s0 / 2 > pad ? s0 / 2 - pad : 0, c1 = (s1 + 1) / 2 + pad;
                const uint32_t lx0 = ax ? Rlow.y0 : Rlow.x0, lx1 = lx0 + (ax ? Rlow.h : Rlow.w);
                const BandG& Bh = Rl.bands[ax ? 1 : 0];       // HL (high in x) / LH (high in y)
                const uint32_t hx0 = ax ? Bh.y0 : Bh.x0, hx1 = ax ? Bh.y1 : Bh.x1;
                lo[ax][l][0] = std::max(c0, lx0); lo[ax][l][1] = std::min(c1, lx1);
                hi[ax][l][0] = std::max(c0, hx0); hi[ax][l][1] = std::min(c1, hx1);
                s0 = lo[ax][l][0]; s1 = std::max(lo[ax][l][0], lo[ax][l][1]);
            }
        }
        }
        for (uint32_t c = 0; c < P.nc; ++c) {
            const uint32_t g = P.group_of[c], nres = P.groups[g].numres;
            const auto& lo = LO[g];
            const auto& hi = HI[g];
            for (uint32_t r = 0; r < nres; ++r) {
                const ResG& R = T.comps[c].res[r];
                const uint32_t lev = r ? nres - r : nres - 1;
                for (uint32_t bi = 0; bi < R.bands.size(); ++bi) {
                    const uint32_t o = R.bands[bi].orient;
                    const uint32_t* nx = (o & 1) ? hi[0][lev].data() : lo[0][lev].data();
                    const uint32_t* ny = (o & 2) ? hi[1][lev].data() : lo[1][lev].data();
                    for (uint32_t pi = 0; pi < R.pw * R.ph; ++pi) {
                        const PrecG& PG = R.prc[bi][pi];
                        for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                            const uint32_t bb = PG.first_block + k;
                            const GkBlock& G = P.blocks[bb];
                            const uint32_t x = P.bxy[2 * (size_t)bb], y = P.bxy[2 * (size_t)bb + 1];
                            need[bb - T.b0] = x < nx[1] && nx[0] < x + G.w && y < ny[1] && ny[0] < y + G.h;
                        }
                    }
                }
            }
        }
    };
    std::vector<std::vector<uint8_t>> part_need(Hd.parts.size());
    host_pool().run(Hd.parts.size(), [&](size_t q) { block_needed(P.tiles[Hd.parts[q].tile], part_need[q]); });
    // ---- T2 (T2Decompress.cpp:216-570), LRCP, per tile part.  Tile parts are independent
    // (own precincts, tag trees and code-blocks), so they are parsed in parallel host threads
    // into tile-local state (index = block - tile's first block).
    struct Chunk { uint64_t pos; uint32_t b, len, boff; };   // boff: the block's bytes before this chunk
    struct PartState {
        std::vector<Chunk> chunks;
        std::vector<uint8_t> included, numbps;
        std::vector<uint16_t> npasses;
        std::vector<uint32_t> numlenbits, len;
        // BYPASS / TERMALL: per block the byte length of each codeword segment and the passes
        // of its last segment (T2Decompress::initSegment, T2Decompress.cpp:28-54)
        std::vector<std::vector<uint32_t>> seglens;
        std::vector<uint16_t> segp;
    };
    // BYPASS / TERMALL components: several codeword segments per block (per component with COC)
    auto comp_multiseg = [&](uint32_t c) { return (P.p.c_sty(c) & (GK_STY_LAZY | GK_STY_TERMALL)) != 0; };
    bool multiseg = false;
    for (uint32_t c = 0; c < P.nc; ++c) multiseg = multiseg || comp_multiseg(c);
    auto seg_max = [&](uint32_t c, uint32_t sg) -> uint32_t {
        if (P.p.c_sty(c) & GK_STY_TERMALL) return 1;
        return sg == 0 ? 10 : ((sg & 1) ? 2 : 1);
    };
    std::vector<PartState> ps(Hd.parts.size());
    auto t2_part = [&](size_t q, ByteSrc& BS) {
        const TilePart& TPt = Hd.parts[q];
        PartState& st2 = ps[q];
        const std::vector<uint8_t>& need = part_need[q];
        struct Trees { DecTree incl, imsb; };
        std::vector<Trees> trees;
        std::unordered_map<uint32_t, size_t> tidx;   // trees by first_block of each precinct-band
        const TileG& TG = P.tiles[TPt.tile];
        const uint32_t tb0 = TG.b0, ntb = TG.b1 - TG.b0;
        st2.included.assign(ntb, 0); st2.numbps.assign(ntb, 0); st2.npasses.assign(ntb, 0);
        st2.numlenbits.assign(ntb, 0); st2.len.assign(ntb, 0);
        if (multiseg) { st2.seglens.assign(ntb, {}); st2.segp.assign(ntb, 0); }
        st2.chunks.reserve(ntb);
        size_t tile_end = TPt.end;
        size_t pos = TPt.data, pk = 0, nextp = 0;
        ByteSrc HS;   // the tile's packed packet headers (PPM / PPT)
        HS.host = TPt.hdrs.data(); HS.len = TPt.hdrs.size();
        size_t hpos = 0;
        const std::vector<PacketRef> order = packet_order(P, TG, P.p.nlayers, TPt.pocs.empty() ? &P.p.pocs : &TPt.pocs);
        // layer limit (tcp->numLayersToDecompress): packets of later layers are skipped through
        // PLT or parsed without their data (T2Decompress::processPacket, T2Decompress.cpp:55-116)
        const uint32_t maxl = ctx->dec_layers ? std::min(ctx->dec_layers, P.p.nlayers) : P.p.nlayers;
        for (size_t oi = 0; oi < order.size(); ++oi, ++pk) {
                        const uint32_t l = order[oi].l, r = order[oi].r, c = order[oi].c, pi = order[oi].pi;
                        const ResG& R = TG.comps[c].res[r];
                        const uint32_t rmax = P.p.c_numres(c) - ctx->dec_reduce;   // resolutions decoded
                        const bool mseg = comp_multiseg(c);
                        while (pos >= tile_end && nextp < TPt.more.size()) {   // the tile's next tile part
                            pos = TPt.more[nextp].first; tile_end = TPt.more[nextp].second; ++nextp;
                        }
                        if (pos >= tile_end) return;
                        const bool skip_l = l >= maxl || r >= rmax;
                        if (skip_l && pk < TPt.plt.size()) { pos += TPt.plt[pk]; continue; }
                        if (pk < TPt.plt.size()) {   // PLT: a packet with no needed block is skipped unread
                            bool any = false;
                            for (uint32_t bi = 0; bi < R.bands.size() && !any; ++bi) {
                                const PrecG& PG = R.prc[bi][pi];
                                for (uint32_t k = 0; k < PG.cw * PG.ch && !any; ++k) any = need[PG.first_block + k - tb0];
                            }
                            if (!any) { pos += TPt.plt[pk]; continue; }
                        }
                        if (P.p.sop_eph & 2) {   // SOP: FF91 0004 Nsop (T2Decompress::readPacketHeader :226-250)
                            if (tile_end - pos < 6 || BS.be16(pos) != 0xff91) throw GkError("expected SOP marker");
                            if (BS.be16(pos + 4) != (pk & 0xffff)) throw GkError("SOP marker packet counter mismatch");
                            pos += 6;
                        }
                        // the header from the packed headers (PPM / PPT) when the tile has them, else in
                        // front of the body (T2Decompress.cpp:255-270)
                        BitReader br = TPt.packed ? BitReader(HS, hpos, HS.len) : BitReader(BS, pos, tile_end);
                        std::vector<std::pair<uint32_t, uint32_t>> contrib;
                        if (br.read(1)) {
                            for (uint32_t bi = 0; bi < R.bands.size(); ++bi) {
                                const PrecG& PG = R.prc[bi][pi];
                                if (!PG.cw || !PG.ch) continue;
                                auto it = tidx.find(PG.first_block);
                                if (it == tidx.end()) {
                                    trees.emplace_back();
                                    trees.back().incl.build(PG.cw, PG.ch);
                                    trees.back().imsb.build(PG.cw, PG.ch);
                                    it = tidx.emplace(PG.first_block, trees.size() - 1).first;
                                }
                                Trees& T = trees[it->second];
                                for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
                                    const uint32_t b = PG.first_block + k - tb0;
                                    uint32_t inc;
                                    if (!st2.included[b]) inc = T.incl.decode(br, k, l + 1) <= l ? 1 : 0;
                                    else inc = br.read(1);
                                    if (!inc) continue;
                                    if (!st2.included[b]) {
                                        // zero bit-planes: Grok raises the threshold one plane at a time
                                        // until the leaf is known; a tag tree reads a node's bits only
                                        // once its parent is known, so one walk with threshold 64 reads
                                        // exactly the same bits
                                        const uint32_t v = T.imsb.decode(br, k, 64);
                                        const uint32_t kmsbs = v < 64 ? v : 64;
                                        const uint32_t bnb = R.bands[bi].numbps;
                                        st2.numbps[b] = (uint8_t)(kmsbs > bnb ? 0 : bnb - kmsbs);
                                        st2.numlenbits[b] = 3;
                                        st2.included[b] = 1;
                                    }
                                    const uint32_t np = br.numpasses();
                                    st2.numlenbits[b] += br.commacode();
                                    uint32_t sl = 0;
                                    if (!mseg) {
                                        const uint32_t nbits = st2.numlenbits[b] + floorlog2(np);
                                        if (nbits > 32) throw GkError("corrupt packet header (segment length)");
                                        sl = br.read((int)nbits);
                                    } else {
                                        // one length per segment part; a segment continues across
                                        // packets until it holds its maximum pass count
                                        std::vector<uint32_t>& SL = st2.seglens[b];
                                        for (uint32_t left = np; left;) {
                                            if (SL.empty() || st2.segp[b] == seg_max(c, (uint32_t)SL.size() - 1)) {
                                                if (SL.size() >= GK_MAX_PASSES) throw GkError("corrupt packet header (segments)");
                                                SL.push_back(0); st2.segp[b] = 0;
                                            }
                                            const uint32_t n = std::min(seg_max(c, (uint32_t)SL.size() - 1) - st2.segp[b], left);
                                            const uint32_t nbits = st2.numlenbits[b] + floorlog2(n);
                                            if (nbits > 32) throw GkError("corrupt packet header (segment length)");
                                            const uint32_t part = br.read((int)nbits);
                                            if (!skip_l) SL.back() += part;
                                            sl += part;
                                            st2.segp[b] = (uint16_t)(st2.segp[b] + n);
                                            left -= n;
                                        }
                                    }
                                    if (st2.npasses[b] + np > GK_MAX_PASSES) throw GkError("corrupt packet header (pass count)");
                                    if (!skip_l) st2.npasses[b] = (uint16_t)(st2.npasses[b] + np);
                                    contrib.push_back({b, sl});
                                }
                            }
                        }
                        br.align();
                        if (TPt.packed) {
                            hpos = br.off;
                            if (hpos > HS.len) throw GkError("corrupt packed packet headers");
                            if (P.p.sop_eph & 4) {   // EPH after the header, in the packed headers
                                if (HS.len - hpos < 2 || HS.be16(hpos) != 0xff92) throw GkError("expected EPH marker");
                                hpos += 2;
                            }
                        } else {
                        pos = br.off;
                        if (P.p.sop_eph & 4) {   // EPH after the header (:469-486)
                            if (tile_end - pos < 2 || BS.be16(pos) != 0xff92) throw GkError("expected EPH marker");
                            pos += 2;
                        }
                        }
                        for (auto& ct : contrib) {
                            const uint32_t n = (uint32_t)std::min<size_t>(ct.second, tile_end > pos ? tile_end - pos : 0);
                            if (n && need[ct.first] && !skip_l) {
                                st2.chunks.push_back({pos, ct.first, n, st2.len[ct.first]});
                                st2.len[ct.first] += n;
                            }
                            pos += ct.second;
                        }
        }
    };
    const auto h1 = now();
    if (Hd.parts.size() == 1) {
        t2_part(0, S);
    } else {
        host_pool().run(Hd.parts.size(), [&](size_t q) {
            ByteSrc BS = S.fork();   // per-call cursor caches (batched regions are shared read-only)
            t2_part(q, BS);
        });
    }
    const auto h2 = now();
    // ---- the decode table: the needed blocks of the rectangle's tiles, compacted, with offsets
    // into this call's planes and staging slots, band quantisation from QCD (decoder semantics)
    // (written straight into the pinned upload buffer: no vector growth, no extra copy)
    size_t nmax = 0;
    for (const auto& nd : part_need) nmax += (size_t)std::count(nd.begin(), nd.end(), (uint8_t)1);
    GkBlock* blk = (GkBlock*)ctx->hinfo.get(sizeof(GkBlock) * std::max<size_t>(nmax, 1));
    uint32_t nblk = 0;
    std::vector<uint32_t> hseglen;   // BYPASS / TERMALL: segment lengths, a block's at G.data_cap
    std::vector<std::vector<int32_t>> part_idx(Hd.parts.size());   // tile-local block -> table entry
    uint64_t o = 0, t1_bytes = 0;
    // one tile's needed blocks into blk[nb0 ..) with staging offsets from o0 (its blocks in
    // (component, resolution, band, precinct, block) order); count-only when blk is null
    struct TileFill { int32_t q; uint32_t t, nb; uint64_t bytes, t1; };
    // the blocks of one precinct-band (c, r, bi, pi) of a tile, continuing n / oo / t1
    auto fill_prec = [&](const TileFill& tf, uint32_t c, uint32_t r, uint32_t bi, uint32_t pi, uint32_t nb0,
                         bool count_only, uint32_t& n, uint64_t& oo, uint64_t& t1) {
        const TileG& T = P.tiles[tf.t];
        const PartState& st2 = ps[tf.q];
        const std::vector<uint8_t>& need = part_need[tf.q];
        std::vector<int32_t>& idx = part_idx[tf.q];
        const ResG& R = T.comps[c].res[r];
        const PrecG& PG = R.prc[bi][pi];
        for (uint32_t k = 0; k < PG.cw * PG.ch; ++k) {
            const uint32_t lb = PG.first_block + k - T.b0;
            if (!need[lb]) continue;
            const uint32_t len = st2.len[lb];
            if (!count_only) {
                GkBlock& G = blk[nb0 + n];
                G = P.blocks[T.b0 + lb];
                G.band_off = relocate(P, RGg[P.group_of[G.comp]], G.band_off);
                G.stride = RG.stride;
                G.band_numbps = (uint8_t)R.bands[bi].numbps;
                G.step = R.bands[bi].step_dec / 2.0f;
                if (P.p.c_ht(c) && P.p.c_irrev(c)) {   // ScaleHTFilter: stepsize / 2^(31 - numbps) (Quantizer.cpp:52-62)
                    if (R.bands[bi].numbps > 31) throw GkError("unsupported number of band bit-planes");
                    G.step = R.bands[bi].step_dec / (float)(1u << (31 - R.bands[bi].numbps));
                }
                G.numbps = st2.numbps[lb];
                G.npasses = len ? st2.npasses[lb] : 0;
                if (multiseg) {
                    G.data_cap = (uint32_t)hseglen.size();
                    hseglen.insert(hseglen.end(), st2.seglens[lb].begin(), st2.seglens[lb].end());
                }
                G.data_off = oo;
                G.len = len;
                idx[lb] = (int32_t)(nb0 + n);
            }
            t1 += len;
            oo += (((uint64_t)len + 15) & ~15ull) + 32;
            ++n;
        }
    };
    auto fill_tile = [&](const TileFill& tf, uint32_t nb0, uint64_t o0, bool count_only, TileFill* out) {
        const TileG& T = P.tiles[tf.t];
        if (!count_only) part_idx[tf.q].assign(T.b1 - T.b0, -1);
        uint32_t n = 0;
        uint64_t oo = o0, t1 = 0;
        for (uint32_t c = 0; c < P.nc; ++c)
            for (uint32_t r = 0; r < (uint32_t)T.comps[c].res.size(); ++r) {
                const ResG& R = T.comps[c].res[r];
                for (uint32_t bi = 0; bi < R.bands.size(); ++bi)
                    for (uint32_t pi = 0; pi < R.pw * R.ph; ++pi) fill_prec(tf, c, r, bi, pi, nb0, count_only, n, oo, t1);
            }
        if (out) { out->nb = n; out->bytes = oo - o0; out->t1 = t1; }
    };
    std::vector<TileFill> tiles_in;
    for (uint32_t j = jb; j < je; ++j)
        for (uint32_t i = ib; i < ie; ++i) {
            const int32_t q = part_of[(size_t)j * P.ntx + i];
            if (q >= 0) tiles_in.push_back({q, j * P.ntx + i, 0, 0, 0});
        }
    // many tiles (C4: 256) fill in parallel from per-tile counts; BYPASS / TERMALL segment
    // lengths append in table order, so those streams take the serial pass
    const bool par_fill = !multiseg && tiles_in.size() >= 8;
    std::vector<uint32_t> tb0(tiles_in.size() + 1, 0);
    std::vector<uint64_t> to0(tiles_in.size() + 1, 0);
    if (par_fill) {
        host_pool().run(tiles_in.size(), [&](size_t k) { fill_tile(tiles_in[k], 0, 0, true, &tiles_in[k]); });
        for (size_t k = 0; k < tiles_in.size(); ++k) {
            tb0[k + 1] = tb0[k] + tiles_in[k].nb; to0[k + 1] = to0[k] + tiles_in[k].bytes; t1_bytes += tiles_in[k].t1;
        }
        host_pool().run(tiles_in.size(), [&](size_t k) { fill_tile(tiles_in[k], tb0[k], to0[k], false, nullptr); });
        nblk = tb0.back(); o = to0.back();
    } else if (!multiseg) {
        // few tiles (C2 / C3: one, 49 k blocks): the same two passes over precinct-bands
        struct Unit { uint32_t k, c, r, bi, pi, nb; uint64_t bytes, t1; };
        std::vector<Unit> units;
        for (uint32_t k = 0; k < tiles_in.size(); ++k) {
            const TileG& T = P.tiles[tiles_in[k].t];
            part_idx[tiles_in[k].q].assign(T.b1 - T.b0, -1);
            for (uint32_t c = 0; c < P.nc; ++c)
                for (uint32_t r = 0; r < (uint32_t)T.comps[c].res.size(); ++r) {
                    const ResG& R = T.comps[c].res[r];
                    for (uint32_t bi = 0; bi < R.bands.size(); ++bi)
                        for (uint32_t pi = 0; pi < R.pw * R.ph; ++pi)
                            if (R.prc[bi][pi].cw * R.prc[bi][pi].ch) units.push_back({k, c, r, bi, pi, 0, 0, 0});
                }
        }
        auto run_unit = [&](size_t i, uint32_t nb0, uint64_t o0, bool count_only) {
            Unit& u = units[i];
            uint32_t n = 0;
            uint64_t oo = o0, t1 = 0;
            fill_prec(tiles_in[u.k], u.c, u.r, u.bi, u.pi, nb0, count_only, n, oo, t1);
            if (count_only) { u.nb = n; u.bytes = oo - o0; u.t1 = t1; }
        };
        host_pool().run(units.size(), [&](size_t i) { run_unit(i, 0, 0, true); });
        std::vector<uint32_t> ub(units.size());
        std::vector<uint64_t> uo(units.size());
        for (size_t i = 0; i < units.size(); ++i) {
            ub[i] = nblk; uo[i] = o;
            nblk += units[i].nb; o += units[i].bytes; t1_bytes += units[i].t1;
        }
        host_pool().run(units.size(), [&](size_t i) { run_unit(i, ub[i], uo[i], false); });
    } else {
        for (TileFill& tf : tiles_in) {
            fill_tile(tf, nblk, o, false, &tf);
            nblk += tf.nb; o += tf.bytes; t1_bytes += tf.t1;
        }
    }
    const uint32_t nbr = nblk, nbx = std::max(nbr, 1u);
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    // ---- stage compressed bytes on the device.  A host stream of which the selected blocks
    // use a small part (window decode of a large file) is gathered on the host and only those
    // bytes cross PCIe; otherwise the whole stream is copied and gathered on the device.
    const bool host_gather = !cs_on_device && o * 2 < len;
    const uint8_t* dcs = cs;
    if (!cs_on_device && !host_gather) {
        uint8_t* d = (uint8_t*)ctx->dout.get(len + 16);
        HIPCHK(hipMemcpyAsync(d, cs, len, hipMemcpyHostToDevice, st));
        dcs = d;
    }
    // gather every selected block's segments into a 16-byte aligned slot followed by >= 32
    // bytes of 0xFF (the T1 decoders read their bytes through aligned windows; the Part-1
    // decoder takes the padding as the MQ end-of-data bytes)
    // (pos, slot position, length) triples, straight into the pinned upload buffer; a part's
    // chunks are those of its own blocks, so parts fill disjoint ranges
    // (a chunk lands at its block's slot + the block's bytes before it, recorded by the parse, so
    // pieces of one part's chunk list fill in parallel; a chunk of a block the table does not
    // hold becomes an empty triple)
    size_t nseg = 0;
    uint64_t* seg = nullptr;
    {
        std::vector<size_t> sb(ps.size() + 1, 0);
        for (size_t q = 0; q < ps.size(); ++q) sb[q + 1] = sb[q] + (part_idx[q].empty() ? 0 : 3 * ps[q].chunks.size());
        seg = (uint64_t*)ctx->hseg.get(sb.back() * 8 + 8);
        struct Piece { size_t q, b, e; };
        std::vector<Piece> pieces;
        for (size_t q = 0; q < ps.size(); ++q) {
            if (part_idx[q].empty()) continue;
            const size_t n = ps[q].chunks.size(), step = std::max<size_t>(4096, n / 32);
            for (size_t b = 0; b < n; b += step) pieces.push_back({q, b, std::min(n, b + step)});
        }
        host_pool().run(pieces.size(), [&](size_t i) {
            const Piece& pc = pieces[i];
            const std::vector<Chunk>& chs = ps[pc.q].chunks;
            const std::vector<int32_t>& idx = part_idx[pc.q];
            for (size_t j = pc.b; j < pc.e; ++j) {
                const Chunk& ch = chs[j];
                const int32_t k = idx[ch.b];
                uint64_t* w = seg + sb[pc.q] + 3 * j;
                w[0] = ch.pos;
                w[1] = k < 0 ? 0 : blk[k].data_off + ch.boff;
                w[2] = k < 0 ? 0 : ch.len;
            }
        });
        nseg = sb.back();
    }
    uint8_t* stg = (uint8_t*)ctx->bytes.get(o + 256);   // decoder window loads read up to 48 B past a block
    if (host_gather) {
        HIPCHK(hipStreamSynchronize(st));   // the pinned staging buffer may still feed an earlier copy
        uint8_t* hst = (uint8_t*)ctx->hstage2.get(o + 256);
        if (!P.p.ht()) memset(hst, 0xff, o);
        for (size_t k = 0; k < nseg; k += 3) memcpy(hst + seg[k + 1], cs + seg[k], seg[k + 2]);
        HIPCHK(hipMemcpyAsync(stg, hst, o, hipMemcpyHostToDevice, st));
    } else {
    if (!P.p.ht()) HIPCHK(hipMemsetAsync(stg, 0xff, o, st));
    if (nseg) {
        uint64_t* ds = (uint64_t*)ctx->dseg.get(nseg * 8 + 8);
        HIPCHK(hipMemcpyAsync(ds, seg, nseg * 8, hipMemcpyHostToDevice, st));
        gk_launch_gather(st, dcs, stg, ds, (uint32_t)(nseg / 3));
    }
    }
    const uint8_t* src_bytes = stg;
    if (prof)
        fprintf(stderr, "decode host: headers+setup %.3f ms, packet headers %.3f ms, segments %.3f ms (%zu parts, "
                        "%u blocks); %llu page fetches %.3f ms (cumulative)\n",
                ms(h0, h1), ms(h1, h2), ms(h2, now()), Hd.parts.size(), nbr,
                (unsigned long long)ByteSrc::fetch_cnt.load(), ByteSrc::fetch_ns.load() * 1e-6);
    // components coded with different T1 coders (COC: Part-1 / mode switches / HT): the table is
    // grouped by coder class (a stable partition; entries keep their staging offsets and segment
    // lists), one decoder launch per class below
    std::vector<std::pair<uint32_t, uint32_t>> cls_range;   // (first entry, class) per class run
    {
        bool mixed = false;
        for (uint32_t c = 1; c < P.nc; ++c) mixed = mixed || P.p.c_class(c) != P.p.c_class(0);
        if (mixed && nbr) {
            std::vector<GkBlock> tmp(blk, blk + nbr);
            std::vector<uint32_t> classes;
            for (uint32_t c = 0; c < P.nc; ++c)
                if (std::find(classes.begin(), classes.end(), P.p.c_class(c)) == classes.end()) classes.push_back(P.p.c_class(c));
            uint32_t k = 0;
            for (uint32_t cl : classes) {
                const uint32_t k0 = k;
                for (const GkBlock& G : tmp)
                    if (P.p.c_class(G.comp) == cl) blk[k++] = G;
                if (k > k0) cls_range.push_back({k0, cl});
            }
        } else {
            cls_range.push_back({0, P.p.c_class(0)});
        }
    }
    GkBlock* dblk_all = (GkBlock*)ctx->dblocks.get(sizeof(GkBlock) * nbx);
    HIPCHK(hipMemcpyAsync(dblk_all, blk, sizeof(GkBlock) * nbr, hipMemcpyHostToDevice, st));
    ctx->blocks_uploaded = false;   // the encode table must be re-uploaded
    int32_t* arena = (int32_t*)ctx->arena.get(RG.plane * P.nc * 2 * sizeof(int32_t));
    // tiles of the rectangle without a tile part decode as zero; blocks skipped by the window
    // need no clearing (they only feed samples outside the output region)
    if (Hd.parts.size() < (size_t)(ie - ib) * (je - jb))
        HIPCHK(hipMemsetAsync(arena, 0, RG.plane * P.nc * 2 * sizeof(int32_t), st));
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[2], st));
    // one class of the table: entries [s, s + n), decoder class cls (Params::c_class)
    auto t1_class = [&](uint32_t s0, uint32_t n, uint32_t cls) {
        const uint32_t nbr = n, nbx = std::max(n, 1u);
        GkBlock* const blk_all = blk;
        GkBlock* const blk = blk_all + s0;
        GkBlock* const dblk = dblk_all + s0;
        const bool cls_ht = (cls & 3) == 2, cls_generic = (cls & 3) == 1, cls_wide = (cls >> 8) & 1;
        const uint32_t cls_sty = (cls >> 2) & 0x3f;
        (void)blk_all;
        if (nbr == 0) {
            // nothing to decode (all-zero tiles)
        } else if (cls_ht) {
            // HT cleanup pass decode straight into the band windows (T1HT::decompress, T1HT.cpp:134-187)
            uint32_t* dsel = (uint32_t*)ctx->dord.get(4 * (size_t)nbx + 16);
            uint32_t* hsel = (uint32_t*)ctx->hord.get(4 * (size_t)nbx + 16);
            for (uint32_t k = 0; k < nbr; ++k) hsel[k] = k;
            HIPCHK(hipMemcpyAsync(dsel, hsel, 4 * (size_t)nbr, hipMemcpyHostToDevice, st));
            int* derr = (int*)ctx->derr.get(64);
            HIPCHK(hipMemsetAsync(derr, 0, 64, st));
            gk_launch_ht_dec(st, src_bytes, dblk, dsel, arena, nbr, derr, cls_wide);
            launch_check(__LINE__);
            HIPCHK(hipEventRecord(ctx->ev[8], st));
            int herr = 0;
            HIPCHK(hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (herr) throw GkError("corrupt HT code-block segment");
        } else if (cls_generic) {
            // mode switches or wide code-blocks: lane-per-block decoder over the codeword segments
            // (gk_t1ms.hip)
            uint32_t* dsl = nullptr;   // (segment tables for BYPASS / TERMALL classes only: one segment otherwise)
            if ((cls_sty & (GK_STY_LAZY | GK_STY_TERMALL)) && !hseglen.empty()) {
                uint32_t* hsl = (uint32_t*)ctx->hord.get(4 * hseglen.size());
                memcpy(hsl, hseglen.data(), 4 * hseglen.size());
                dsl = (uint32_t*)ctx->dseglen.get(4 * hseglen.size());
                HIPCHK(hipMemcpyAsync(dsl, hsl, 4 * hseglen.size(), hipMemcpyHostToDevice, st));
            }
            uint8_t* mst = (uint8_t*)ctx->dmsstate.get(gk_t1ms_state_bytes(nbx));
            gk_launch_t1_dec_ms(st, src_bytes, dblk, dsl, arena, nbr, mst, cls_sty);
            launch_check(__LINE__);
            HIPCHK(hipEventRecord(ctx->ev[8], st));
            if (dsl) HIPCHK(hipStreamSynchronize(st));   // the pinned table is reused
        } else {
            // lane assignment: blocks bucketed by pass count (descending), so the lanes of a
            // wave decode similar amounts of work and the longest waves start first.  Only
            // `L` lanes of each 64-lane wave carry a block (gk_t1dec_lanes): fewer lanes per wave
            // give more waves, so every SIMD of the chip holds waves and can hide latency.
            const uint32_t L = gk_t1dec_lanes();
            // The heaviest blocks go to solo waves (gk_t1dec.hip solo_block) on the SIMDs the
            // lane-parallel waves leave.  Weight = compressed bytes (decisions follow them within
            // ~10 %).  K, the number of solo blocks, balances the two sides: the lane-parallel
            // waves last as long as the heaviest block left to them (weight w[K]), a solo wave as
            // long as its blocks' sum / ratio; the top K are packed longest-first into the solo
            // waves (LPT) and K is the crossing point of the two (binary search: the first falls,
            // the second grows with K).  GK_T1DEC_SOLO=n: the n heaviest, one per wave.
            GkSoloPlan sp = nbr ? gk_t1dec_solo_plan(nbr, L) : GkSoloPlan{0, -1, 1.f};
            // Device shared with another engine's call in progress (e.g. two images in flight; engines
            // that merely exist, like the bench's C2 + C3 pair run one after the other, do not count):
            // no SIMD is idle, so a solo
            // wave's time is taken from the other decodes; only clear outliers (> 1.3 x the weight of
            // the block at rank 1,024) go solo, one per wave.  C2 (LL blocks 1.06 x the plateau): none,
            // 2,394 -> 2,548 Mpix/s with two images in flight; C3 (LL ~1.6 x): kept (1,761 -> 2,056).
            const bool shared = sp.forced < 0 && engines_busy(ctx->device) > 1;
            uint32_t nsb = 0;
            std::vector<uint32_t> byl;
            std::vector<std::vector<uint32_t>> bins;
            auto weight = [&](uint32_t q) -> uint64_t { return blk[q].npasses ? blk[q].len : 0; };
            if (sp.waves) {
                // (at most 4 blocks per solo wave: the search stays a fraction of a millisecond of host time)
                const uint32_t kmax = sp.forced >= 0 ? (uint32_t)sp.forced : std::min<uint32_t>(nbr / 4, 4u * sp.waves);
                byl.resize(nbr);
                for (uint32_t q = 0; q < nbr; ++q) byl[q] = q;
                auto heavier = [&](uint32_t x, uint32_t y) { return weight(x) != weight(y) ? weight(x) > weight(y) : x < y; };
                const uint32_t top = std::min<uint32_t>(kmax + 1, nbr);
                if (top) {
                    std::nth_element(byl.begin(), byl.begin() + (top - 1), byl.end(), heavier);
                    std::sort(byl.begin(), byl.begin() + top, heavier);
                }
                // longest-first packing of the k heaviest into the solo waves; returns the largest load
                auto pack = [&](uint32_t k, std::vector<std::vector<uint32_t>>* out) -> uint64_t {
                    std::vector<uint64_t> load(sp.waves, 0);
                    std::vector<uint32_t> cnt(sp.waves, 0);
                    if (out) out->assign(sp.waves, {});
                    using E = std::pair<uint64_t, uint32_t>;
                    std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
                    for (uint32_t b = 0; b < sp.waves; ++b) pq.push({0, b});
                    uint64_t mx = 0;
                    for (uint32_t j = 0; j < k && !pq.empty(); ++j) {
                        const E e = pq.top();
                        pq.pop();
                        load[e.second] = e.first + weight(byl[j]);
                        mx = std::max(mx, load[e.second]);
                        if (out) (*out)[e.second].push_back(byl[j]);
                        if (++cnt[e.second] < 64) pq.push({load[e.second], e.second});
                    }
                    return mx;
                };
                uint32_t k = 0;
                if (sp.forced >= 0) {
                    k = (uint32_t)sp.forced;
                    bins.assign(sp.waves, {});
                    for (uint32_t j = 0; j < k; ++j) bins[j].push_back(byl[j]);
                } else if (shared) {
                    const uint32_t r = std::min<uint32_t>(std::max<uint32_t>(1024u, top), nbr - 1);
                    if (r >= top) std::nth_element(byl.begin() + top, byl.begin() + r, byl.end(), heavier);
                    const double ref = 1.3 * (double)weight(byl[r]);
                    while (k < std::min<uint32_t>(kmax, sp.waves) && (double)weight(byl[k]) > ref) ++k;
                    bins.assign(sp.waves, {});
                    for (uint32_t j = 0; j < k; ++j) bins[j].push_back(byl[j]);
                } else {
                    auto lane_side = [&](uint32_t kk) -> double { return kk < nbr ? (double)weight(byl[kk]) : 0.0; };
                    auto solo_side = [&](uint32_t kk) -> double { return (double)pack(kk, nullptr) / sp.ratio; };
                    uint32_t lo = 0, hi = kmax;   // first k with solo_side(k) >= lane_side(k)
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) / 2;
                        if (solo_side(mid) >= lane_side(mid)) hi = mid; else lo = mid + 1;
                    }
                    k = lo;
                    if (k > 0 && std::max(solo_side(k - 1), lane_side(k - 1)) <= std::max(solo_side(k), lane_side(k))) --k;
                    if (k) pack(k, &bins);
                }
                nsb = k;
            }
            uint32_t nsw = 0;   // solo waves holding a block, rounded up to whole workgroups of 12
            for (uint32_t b = 0; b < bins.size(); ++b)
                if (!bins[b].empty()) nsw = b + 1;
            nsw = (nsw + 11) / 12 * 12;
            const uint32_t nw = nsw + (nbr - nsb + L - 1) / L, nslots = nw * 64;
            uint32_t* hord = (uint32_t*)ctx->hord.get(4 * ((size_t)nslots + 2 * (size_t)nbr + 2) + 8 * ((size_t)nw + 1));
            uint32_t* hpos = hord + nslots;               // slot of block k
            uint32_t* hids = hpos + nbr;                  // identity (compact table)
            uint64_t* hwo = (uint64_t*)(hids + nbr + 2);
            {
                std::fill(hord, hord + nslots, 0xffffffffu);
                std::vector<uint8_t> solo(nbr, 0);
                for (uint32_t b = 0; b < bins.size() && b < nsw; ++b)
                    for (uint32_t i = 0; i < bins[b].size(); ++i) {
                        const uint32_t q = bins[b][i];
                        solo[q] = 1;
                        hord[(size_t)b * 64 + i] = q; hpos[q] = b * 64 + i;
                    }
                std::vector<uint32_t> cnt(GK_MAX_PASSES + 2, 0);
                for (uint32_t q = 0; q < nbr; ++q)
                    if (!solo[q]) cnt[std::min<uint32_t>(blk[q].npasses, GK_MAX_PASSES + 1)]++;
                std::vector<uint32_t> start(GK_MAX_PASSES + 2, 0);
                uint32_t acc = 0;
                for (int k = GK_MAX_PASSES + 1; k >= 0; --k) { start[k] = acc; acc += cnt[k]; }
                for (uint32_t q = 0; q < nbr; ++q) {
                    hids[q] = q;
                    if (solo[q]) continue;
                    const uint32_t k = std::min<uint32_t>(blk[q].npasses, GK_MAX_PASSES + 1);
                    const uint32_t idx = start[k]++;
                    const uint32_t slot = (nsw + idx / L) * 64 + idx % L;
                    hord[slot] = q; hpos[q] = slot;
                }
                uint64_t wo = 0;
                for (uint32_t wv = 0; wv < nw; ++wv) {
                    hwo[wv] = wo;
                    uint32_t mp = 0;
                    for (uint32_t i = wv * 64; i < wv * 64 + (wv < nsw ? 64 : L); ++i)
                        if (hord[i] != 0xffffffffu) mp = std::max(mp, (uint32_t)blk[hord[i]].numbps);
                    if (wv < nsw && hord[wv * 64] == 0xffffffffu) continue;   // a solo wave without a block
                    wo += (272 + (uint64_t)mp * 64) * 64;   // per-lane slab: WS_FIXED + planes (gk_t1dec.hip), 128 B lines
                }
                hwo[nw] = wo;
            }
            const size_t obytes = 4 * ((size_t)nslots + 2 * (size_t)nbr + 2) + 8 * ((size_t)nw + 1);
            uint32_t* dord = (uint32_t*)ctx->dord.get(obytes);
            HIPCHK(hipMemcpyAsync(dord, hord, obytes, hipMemcpyHostToDevice, st));
            const uint32_t* dpos = dord + nslots;
            const uint32_t* dids = dpos + nbr;
            const uint64_t* dwo = (const uint64_t*)(dids + nbr + 2);
            uint64_t* dscr = (uint64_t*)ctx->dscratch.get(8 * hwo[nw] + 64);
            // lane-parallel decoder state rows start at zero; solo waves write every row recon reads
            HIPCHK(hipMemsetAsync(dscr + hwo[nsw], 0, 8 * (hwo[nw] - hwo[nsw]), st));
            gk_launch_t1_dec(st, src_bytes, dblk, dord, dscr, dwo, nslots, nsw);
            ctx->tm.t1_steps_max = ctx->tm.t1_steps_total = ctx->tm.t1_symbols = 0;
            ctx->tm.t1_solo_decisions = ctx->tm.t1_solo_decisions_max = 0;
            ctx->tm.t1_solo_blocks = nsb;
            if (getenv("GK_T1_STATS")) {
                uint64_t sv[5];
                gk_t1dec_stats(sv);
                ctx->tm.t1_steps_max = sv[0]; ctx->tm.t1_steps_total = sv[1]; ctx->tm.t1_symbols = sv[2];
                ctx->tm.t1_solo_decisions = sv[3]; ctx->tm.t1_solo_decisions_max = sv[4];
            }
            launch_check(__LINE__);
            HIPCHK(hipEventRecord(ctx->ev[8], st));
            uint32_t maxnp = 1;
            for (uint32_t q = 0; q < nbr; ++q) maxnp = std::max<uint32_t>(maxnp, blk[q].numbps);
            gk_launch_t1_recon(st, dblk, dids, dpos, dscr, dwo, arena, nbr, maxnp);
        }
    };
    for (size_t k = 0; k < cls_range.size(); ++k) {
        const uint32_t s0 = cls_range[k].first, e0 = k + 1 < cls_range.size() ? cls_range[k + 1].first : nbr;
        if (k) HIPCHK(hipStreamSynchronize(st));   // (the pinned staging tables are reused per class)
        t1_class(s0, e0 - s0, cls_range[k].second);
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[3], st));
    // ---- inverse DWT; its last level writes the output region through the inverse MCT + DC
    // shift + clamp into the output planes (without decomposition levels a separate pass does)
    // DC shift and clamp per component (its precision and sign: mct::decompress_dc_shift_* per
    // component); 8 / 16-bit output takes the largest precision and one sign
    std::vector<int32_t> shiftv(P.nc), mnv(P.nc), mxv(P.nc);
    for (uint32_t c = 0; c < P.nc; ++c) {
        const uint32_t pr = P.c_prec(c);
        const bool sg = P.c_sgnd(c) != 0;
        shiftv[c] = sg ? 0 : (1 << (pr - 1));
        mnv[c] = sg ? -(1 << (pr - 1)) : 0;
        mxv[c] = sg ? (1 << (pr - 1)) - 1 : (int32_t)((1u << pr) - 1);
        if ((sample_bytes == 1 || sample_bytes == 2) && sg != (P.sgnd != 0))
            throw GkError("8 / 16-bit output of components with different signs: use int32 planes");
    }
    const int stype = sample_type(sample_bytes, P.prec, P.sgnd != 0);
    const size_t es = gk_sample_size(stype);
    const bool mct3r = P.mct3();
    if (red) {
        // reduced resolution: undo levels L .. red+1; resolution numres-1-red of each tile is
        // then at the tile's corner of plane (red odd ? B : A); the inverse MCT + DC + clamp
        // writes it per tile into the ceil(size / 2^red) output (a tile's reduced origin is
        // ceil(origin / 2^red), B.5).  Subsampled components: the same on each component's grid
        // (tile-component ceil(tile / XRsiz), then reduced), one plane each.
        run_dwt(ctx, RG, false, jb, je, ib, ie, nullptr, red + 1);
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[4], st));
        // reduced canvas: positions ceil(x / 2^red); output index = that less the image origin's.
        // A window (image-relative, full resolution) reduces the same way (the composite
        // component bounds of CodeStreamDecompress.cpp:471-481, rectceildivpow2): the output is
        // the reduced tile rectangle clipped to it, the caller's planes addressing its origin
        std::vector<uint32_t> rox(P.nc), roy(P.nc), qx0(P.nc), qy0(P.nc), qx1(P.nc), qy1(P.nc), wx0(P.nc, 0), wy0(P.nc, 0);
        // (component c: canvas positions on its grid first, ceil(x / dx), then reduced)
        for (uint32_t c = 0; c < P.nc; ++c) {
            const SGroup& G = P.groups[P.group_of[c]];
            auto rx = [&](uint32_t v) { return ceildivpow2(ceildiv(v, G.dx), red); };
            auto ry = [&](uint32_t v) { return ceildivpow2(ceildiv(v, G.dy), red); };
            rox[c] = ceildivpow2(G.ox, red); roy[c] = ceildivpow2(G.oy, red);
            qx0[c] = rx(RG.x0 + P.x0) - rox[c]; qy0[c] = ry(RG.y0 + P.y0) - roy[c];
            qx1[c] = rx(RG.x0 + P.x0 + RG.w) - rox[c]; qy1[c] = ry(RG.y0 + P.y0 + RG.h) - roy[c];
            if (win) {
                qx0[c] = std::max(qx0[c], rx(win[0] + P.x0) - rox[c]); qy0[c] = std::max(qy0[c], ry(win[1] + P.y0) - roy[c]);
                qx1[c] = std::min(qx1[c], rx(win[2] + P.x0) - rox[c]);
                qy1[c] = std::min(qy1[c], ry(win[3] + P.y0) - roy[c]);
                if (qx1[c] <= qx0[c] || qy1[c] <= qy0[c]) throw GkError("the window is empty at this reduction");
            }
            // the caller plane's origin: the window's (a tile pass: the whole call's frame), or the image's
            wx0[c] = rx(ox + P.x0) - rox[c]; wy0[c] = ry(oy + P.y0) - roy[c];
        }
        std::vector<uint8_t*> qd(P.nc);
        std::vector<uint32_t> qs(P.nc);
        if (!out_on_device) {
            size_t tot = 0;
            for (uint32_t c = 0; c < P.nc; ++c) tot += (size_t)(qx1[c] - qx0[c]) * (qy1[c] - qy0[c]);
            uint8_t* stage = (uint8_t*)ctx->dplanes.get(tot * es + 16);
            size_t o2 = 0;
            for (uint32_t c = 0; c < P.nc; ++c) {
                qd[c] = stage + o2 * es; qs[c] = qx1[c] - qx0[c];
                o2 += (size_t)(qx1[c] - qx0[c]) * (qy1[c] - qy0[c]);
            }
        } else {
            for (uint32_t c = 0; c < P.nc; ++c) {
                qd[c] = (uint8_t*)comps[c] + ((size_t)(qy0[c] - wy0[c]) * strides[c] + (qx0[c] - wx0[c])) * es;
                qs[c] = strides[c];
            }
        }
        for (uint32_t j = jb; j < je; ++j)
            for (uint32_t i = ib; i < ie; ++i) {
                const TileG& T = P.tiles[(size_t)j * P.ntx + i];
                for (uint32_t c = 0; c < P.nc;) {
                    const bool m3 = mct3r && c == 0;
                    const SGroup& G = P.groups[P.group_of[c]];
                    // the tile-component and its reduced rectangle on the component's grid
                    const uint32_t cx0 = ceildiv(T.x0, G.dx), cy0 = ceildiv(T.y0, G.dy);
                    const uint32_t tx0 = ceildivpow2(cx0, red) - rox[c], ty0 = ceildivpow2(cy0, red) - roy[c];
                    const uint32_t tx1 = ceildivpow2(ceildiv(T.x1, G.dx), red) - rox[c];
                    const uint32_t ty1 = ceildivpow2(ceildiv(T.y1, G.dy), red) - roy[c];
                    // the part of the tile's reduced rectangle inside the output
                    const uint32_t ix0 = std::max(tx0, qx0[c]), iy0 = std::max(ty0, qy0[c]);
                    const uint32_t ix1 = std::min(tx1, qx1[c]), iy1 = std::min(ty1, qy1[c]);
                    const uint32_t cn = m3 ? 3 : 1;
                    if (ix1 <= ix0 || iy1 <= iy0) { c += cn; continue; }
                    const uint32_t tw = ix1 - ix0, th = iy1 - iy0;
                    const Region& Rg = RGg[P.group_of[c]];
                    auto src = [&](uint32_t k) {
                        return arena + (size_t)k * 2 * RG.plane + ((red & 1) ? RG.plane : 0) +
                               (size_t)(cy0 - G.oy - Rg.y0 + (iy0 - ty0)) * RG.stride + (cx0 - G.ox - Rg.x0 + (ix0 - tx0));
                    };
                    auto srcf = [&](uint32_t k) { return reinterpret_cast<const float*>(src(k)); };
                    auto dst = [&](uint32_t k) { return qd[k] + ((size_t)(iy0 - qy0[k]) * qs[k] + (ix0 - qx0[k])) * es; };
                    if (!P.p.c_irrev(c)) {
                        if (m3) gk_launch_rct_inv_dc(st, src(0), src(1), src(2), RG.stride, stype, dst(0), dst(1), dst(2), qs[0],
                                                     tw, th, shiftv[c], mnv[c], mxv[c]);
                        else gk_launch_dc_inv(st, src(c), RG.stride, stype, dst(c), qs[c], tw, th, shiftv[c], mnv[c], mxv[c]);
                    } else {
                        if (m3) gk_launch_ict_inv_dc(st, srcf(0), srcf(1), srcf(2), RG.stride, stype, dst(0), dst(1), dst(2),
                                                     qs[0], tw, th, shiftv[c], mnv[c], mxv[c]);
                        else gk_launch_dc_inv_f(st, srcf(c), RG.stride, stype, dst(c), qs[c], tw, th, shiftv[c], mnv[c], mxv[c]);
                    }
                    c += cn;
                }
            }
        if (mct3r && (qs[1] != qs[0] || qs[2] != qs[0])) throw GkError("the first three components must share a stride");
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[5], st));
        if (!out_on_device)
            for (uint32_t c = 0; c < P.nc; ++c) {
                const uint32_t qcols = qx1[c] - qx0[c], qrows = qy1[c] - qy0[c];
                HIPCHK(hipMemcpy2DAsync((uint8_t*)comps[c] + ((size_t)(qy0[c] - wy0[c]) * strides[c] + (qx0[c] - wx0[c])) * es,
                                        (size_t)strides[c] * es, qd[c], (size_t)qcols * es, (size_t)qcols * es, qrows,
                                        hipMemcpyDeviceToHost, st));
            }
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[6], st));
        HIPCHK(hipStreamSynchronize(st));
        ctx->tm.t2_ms = ev_ms(ctx, 0, 1); ctx->tm.t1_ms = ev_ms(ctx, 2, 3); ctx->tm.t1_cm_ms = 0.f;
        ctx->tm.t1_coder_ms = ev_ms(ctx, 2, 8); ctx->tm.cs_bytes = len; ctx->tm.t1_bytes = t1_bytes;
        ctx->tm.dwt_ms = ev_ms(ctx, 3, 4); ctx->tm.mct_ms = ev_ms(ctx, 4, 5); ctx->tm.assemble_ms = ev_ms(ctx, 1, 2);
        ctx->tm.total_ms = ev_ms(ctx, 0, 6); ctx->tm.t1_blocks = nbr;
        return;
    }
    // the output rectangle of component c on its grid ([rx0, rx1) x [ry0, ry1) without
    // subsampling), and the caller plane's origin there (the window's, or the image's)
    std::vector<uint32_t> qx0(P.nc), qy0(P.nc), qx1(P.nc), qy1(P.nc), qox(P.nc), qoy(P.nc);
    for (uint32_t c = 0; c < P.nc; ++c) {
        const SGroup& G = P.groups[P.group_of[c]];
        qx0[c] = ceildiv(rx0 + P.x0, G.dx) - G.ox; qx1[c] = ceildiv(rx1 + P.x0, G.dx) - G.ox;
        qy0[c] = ceildiv(ry0 + P.y0, G.dy) - G.oy; qy1[c] = ceildiv(ry1 + P.y0, G.dy) - G.oy;
        qox[c] = ceildiv(ox + P.x0, G.dx) - G.ox; qoy[c] = ceildiv(oy + P.y0, G.dy) - G.oy;
    }
    auto ocols = [&](uint32_t c) { return qx1[c] - qx0[c]; };
    auto orows = [&](uint32_t c) { return qy1[c] - qy0[c]; };
    std::vector<void*> dst(P.nc);
    std::vector<uint32_t> dstr(P.nc);
    if (!out_on_device) {
        size_t tot = 0;
        for (uint32_t c = 0; c < P.nc; ++c) tot += (size_t)ocols(c) * orows(c);
        uint8_t* stage = (uint8_t*)ctx->dplanes.get(tot * es + 16);
        size_t o2 = 0;
        for (uint32_t c = 0; c < P.nc; ++c) {
            dst[c] = stage + o2 * es; dstr[c] = ocols(c);
            o2 += (size_t)ocols(c) * orows(c);
        }
    } else {
        for (uint32_t c = 0; c < P.nc; ++c) {
            dst[c] = (uint8_t*)comps[c] + ((size_t)(qy0[c] - qoy[c]) * strides[c] + (qx0[c] - qox[c])) * es;
            dstr[c] = strides[c];
        }
    }
    auto planeA = [&](uint32_t c) {
        const Region& Rg = RGg[P.group_of[c]];
        return arena + (size_t)c * 2 * RG.plane + (size_t)(qy0[c] - Rg.y0) * RG.stride + (qx0[c] - Rg.x0);
    };
    auto planeAf = [&](uint32_t c) { return reinterpret_cast<const float*>(planeA(c)); };
    const bool mct3 = P.mct3();
    if (P.max_numres() > 1 && !P.l1_fusable) {   // levels first, then the inverse MCT + DC shift + clamp below
        run_dwt(ctx, RG, false, jb, je, ib, ie, nullptr);
    }
    if (P.max_numres() > 1 && P.l1_fusable) {
        L1Io io;
        io.stype = stype; io.mct3 = mct3; io.shift = shiftv; io.mn = mnv; io.mx = mxv;
        io.planes.assign(dst.begin(), dst.end());
        io.strides = dstr;
        io.cx0 = rx0 + P.x0; io.cy0 = ry0 + P.y0; io.cx1 = rx1 + P.x0; io.cy1 = ry1 + P.y0;
        if (mct3 && (dstr[1] != dstr[0] || dstr[2] != dstr[0])) throw GkError("the first three components must share a stride");
        run_dwt(ctx, RG, false, jb, je, ib, ie, &io);
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[4], st));
    } else {
        // (each component by its own transform: COC may differ; the MCT's three share component 0's)
        launch_check(__LINE__);
        HIPCHK(hipEventRecord(ctx->ev[4], st));
        if (mct3 && !P.p.c_irrev(0))
            gk_launch_rct_inv_dc(st, planeA(0), planeA(1), planeA(2), RG.stride, stype, dst[0], dst[1], dst[2], dstr[0],
                                 ocols(0), orows(0), shiftv[0], mnv[0], mxv[0]);
        if (mct3 && P.p.c_irrev(0))
            gk_launch_ict_inv_dc(st, planeAf(0), planeAf(1), planeAf(2), RG.stride, stype, dst[0], dst[1], dst[2], dstr[0],
                                 ocols(0), orows(0), shiftv[0], mnv[0], mxv[0]);
        for (uint32_t c = mct3 ? 3 : 0; c < P.nc; ++c) {
            if (!P.p.c_irrev(c)) gk_launch_dc_inv(st, planeA(c), RG.stride, stype, dst[c], dstr[c], ocols(c), orows(c), shiftv[c], mnv[c], mxv[c]);
            else gk_launch_dc_inv_f(st, planeAf(c), RG.stride, stype, dst[c], dstr[c], ocols(c), orows(c), shiftv[c], mnv[c], mxv[c]);
        }
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[5], st));
    if (!out_on_device) {
        for (uint32_t c = 0; c < P.nc; ++c)
            HIPCHK(hipMemcpy2DAsync((uint8_t*)comps[c] + ((size_t)(qy0[c] - qoy[c]) * strides[c] + (qx0[c] - qox[c])) * es,
                                    (size_t)strides[c] * es, dst[c], (size_t)ocols(c) * es, (size_t)ocols(c) * es, orows(c),
                                    hipMemcpyDeviceToHost, st));
    }
    launch_check(__LINE__);
    HIPCHK(hipEventRecord(ctx->ev[6], st));
    HIPCHK(hipStreamSynchronize(st));
    ctx->tm.t2_ms = ev_ms(ctx, 0, 1);
    ctx->tm.t1_ms = ev_ms(ctx, 2, 3);
    ctx->tm.t1_cm_ms = 0.f;
    ctx->tm.t1_coder_ms = ev_ms(ctx, 2, 8);
    ctx->tm.cs_bytes = len;
    ctx->tm.t1_bytes = t1_bytes;
    ctx->tm.dwt_ms = ev_ms(ctx, 3, 4);
    ctx->tm.mct_ms = ev_ms(ctx, 4, 5);
    ctx->tm.assemble_ms = ev_ms(ctx, 1, 2);
    ctx->tm.total_ms = ev_ms(ctx, 0, 6);
    ctx->tm.t1_blocks = nbr;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

gk_ctx* gk_create(int device_id) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device_id >= n) return nullptr;
    if (hipSetDevice(device_id) != hipSuccess) return nullptr;
    gk_ctx* ctx = new gk_ctx();
    ctx->device = device_id;
    if (hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) { delete ctx; return nullptr; }
    for (auto& a : ctx->aux)
        if (hipStreamCreateWithFlags(&a, hipStreamNonBlocking) != hipSuccess) { gk_destroy(ctx); return nullptr; }
    for (auto& e : ctx->ev) (void)hipEventCreate(&e);
    for (auto& e : ctx->xev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    // nmsedec lookup tables (t1_generate_luts.cpp:338-362): sig, sig0, ref, ref0
    int16_t tab[4][128];
    for (int i = 0; i < 128; ++i) {
        const double F = 64.0;   // 2^T1_NMSEDEC_FRACBITS
        double t = i / F, u = t, v = t - 1.5;
        tab[0][i] = (int16_t)std::max(0, (int)(floor((u * u - v * v) * F + 0.5) / F * 8192.0));
        tab[1][i] = (int16_t)std::max(0, (int)(floor((u * u) * F + 0.5) / F * 8192.0));
        u = t - 1.0;
        v = (i & 64) ? t - 1.5 : t - 0.5;
        tab[2][i] = (int16_t)std::max(0, (int)(floor((u * u - v * v) * F + 0.5) / F * 8192.0));
        tab[3][i] = (int16_t)std::max(0, (int)(floor((u * u) * F + 0.5) / F * 8192.0));
    }
    if (hipMalloc(&ctx->nmse_tab, sizeof tab) != hipSuccess ||
        hipMemcpy(ctx->nmse_tab, tab, sizeof tab, hipMemcpyHostToDevice) != hipSuccess) {
        gk_destroy(ctx);
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> g(g_dev_mu);
        ++g_dev_engines[device_id];
        ctx->registered = true;
    }
    return ctx;
}

void gk_destroy(gk_ctx* ctx) {
    if (!ctx) return;
    if (ctx->registered) {
        std::lock_guard<std::mutex> g(g_dev_mu);
        if (--g_dev_engines[ctx->device] <= 0) g_dev_engines.erase(ctx->device);
    }
    (void)hipSetDevice(ctx->device);
    if (ctx->st) (void)hipStreamSynchronize(ctx->st);
    for (auto& a : ctx->aux)
        if (a) { (void)hipStreamSynchronize(a); (void)hipStreamDestroy(a); }
    for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->xev) if (e) (void)hipEventDestroy(e);
    if (ctx->nmse_tab) (void)hipFree(ctx->nmse_tab);
    if (ctx->st) (void)hipStreamDestroy(ctx->st);
    delete ctx;
}

void gk_set_default_params(gk_cparameters* p) {
    memset(p, 0, sizeof(*p));
    p->numlayers = 1;
    p->numresolution = 6;
    p->cblockw_init = 64; p->cblockh_init = 64;
    p->mct = 0;   // API default (memset in grk_compress_set_default_params, grok.cpp:409); the CLI sets 1 for RGB
    p->numgbits = 2;
    p->write_comment = 1;
    for (int i = 0; i < GK_MAXRLVLS; ++i) { p->prcw_init[i] = 1u << 15; p->prch_init[i] = 1u << 15; }
}

int gk_encode(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
              int comps_on_device, const gk_cparameters* p, uint8_t* out, size_t cap, size_t* out_len,
              int out_on_device) {
    if (!ctx || !info || !comps || !strides || !out) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        DevBusy busy(ctx->device);
        int rc = 0;
        size_t n = encode_impl(ctx, info, comps, strides, comps_on_device, p, out, cap, out_on_device, &rc);
        if (out_len) *out_len = n;
        if (rc == -2) ctx->err = "output capacity too small";
        return rc;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_encode_tiles(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
                    int comps_on_device, const gk_cparameters* p, uint32_t tile_begin, uint32_t tile_end,
                    uint8_t* out, size_t cap, size_t* out_len, uint32_t* part_lens, int out_on_device) {
    if (!ctx || !info || !comps || !strides || !out || !part_lens || tile_end <= tile_begin) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        DevBusy busy(ctx->device);
        int rc = 0;
        size_t n = encode_impl(ctx, info, comps, strides, comps_on_device, p, out, cap, out_on_device, &rc,
                               tile_begin, tile_end, false, part_lens);
        if (out_len) *out_len = n;
        if (rc == -2) ctx->err = "output capacity too small";
        return rc;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_encode_blocks(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
                     int comps_on_device, const gk_cparameters* p, uint32_t* nbands, uint32_t* nblocks,
                     uint64_t* nbytes, uint32_t* npasses) {
    if (!ctx || !info || !comps || !strides) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        DevBusy busy(ctx->device);
        if (p && p->tile_size_on && (p->t_width < info->w || p->t_height < info->h))
            throw GkError("code-block results are produced for single-tile images only (Grok's plugin tile is one tile)");
        int rc = 0;
        uint8_t dummy = 0;
        encode_impl(ctx, info, comps, strides, comps_on_device, p, &dummy, 0, 0, &rc, 0, 0, true, nullptr, true);
        if (nbands) *nbands = (uint32_t)ctx->rb_bands.size();
        if (nblocks) *nblocks = (uint32_t)ctx->rb_blocks.size();
        if (nbytes) *nbytes = ctx->rb_data.size();
        if (npasses) *npasses = (uint32_t)ctx->rb_passes.size();
        return rc;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_encode_blocks_get(gk_ctx* ctx, gk_band_result* bands, gk_block_result* blocks, uint8_t* data,
                         gk_pass_result* passes) {
    if (!ctx) return -1;
    if (bands) std::copy(ctx->rb_bands.begin(), ctx->rb_bands.end(), bands);
    if (blocks) std::copy(ctx->rb_blocks.begin(), ctx->rb_blocks.end(), blocks);
    if (data && !ctx->rb_data.empty()) memcpy(data, ctx->rb_data.data(), ctx->rb_data.size());
    if (passes) std::copy(ctx->rb_passes.begin(), ctx->rb_passes.end(), passes);
    return 0;
}

int gk_main_header(gk_ctx* ctx, const gk_image_info* info, const gk_cparameters* p, uint8_t* out, size_t cap,
                   size_t* out_len, size_t* tlm_offset, uint32_t* num_tiles) {
    if (!ctx || !info || !out) return -1;
    try {
        setup_plan(ctx, info, p);
        std::vector<uint8_t> H;
        size_t tlm = 0;
        write_main_header(H, ctx->plan, &tlm);
        if (out_len) *out_len = H.size();
        if (tlm_offset) *tlm_offset = ctx->plan.p.tlm ? tlm : 0;
        if (num_tiles) *num_tiles = (uint32_t)ctx->plan.tiles.size();
        if (H.size() > cap) { ctx->err = "output capacity too small"; return -2; }
        memcpy(out, H.data(), H.size());
        return 0;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_decode_header(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, gk_image_info* info) {
    if (!ctx || !cs || !info) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        ByteSrc S; S.len = len; S.st = ctx->st;
        if (cs_on_device) S.dev = cs; else S.host = cs;
        size_t joff = 0, jlen = 0;
        if (jp2_locate(S, joff, jlen)) {
            S = ByteSrc(); S.len = jlen; S.st = ctx->st;
            if (cs_on_device) S.dev = cs + joff; else S.host = cs + joff;
        }
        Header Hd;
        parse_header(S, Hd);
        info->w = Hd.want.w; info->h = Hd.want.h; info->numcomps = Hd.want.nc; info->prec = Hd.want.prec;
        info->sgnd = Hd.want.sgnd; info->x0 = Hd.want.x0; info->y0 = Hd.want.y0;
        ctx->hdr_dx.assign(Hd.want.nc, 1); ctx->hdr_dy.assign(Hd.want.nc, 1);
        ctx->hdr_prec.assign(Hd.want.nc, 0); ctx->hdr_sgnd.assign(Hd.want.nc, 0);
        for (uint32_t c = 0; c < Hd.want.nc; ++c) {
            ctx->hdr_dx[c] = Hd.want.sx(c); ctx->hdr_dy[c] = Hd.want.sy(c);
            ctx->hdr_prec[c] = Hd.want.c_prec(c); ctx->hdr_sgnd[c] = Hd.want.c_sgnd(c);
        }
        return 0;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_jp2_header(gk_ctx* ctx, const gk_image_info* info, uint64_t cs_len, uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx || !info || !out) return -1;
    try {
        Plan P;
        P.w = info->w; P.h = info->h; P.nc = info->numcomps; P.prec = info->prec; P.sgnd = info->sgnd;
        if (!P.w || !P.h || !P.nc || P.nc > 255 || !P.prec || P.prec > 31) throw GkError("bad image info");
        std::vector<uint8_t> J;
        write_jp2_prefix(J, P, cs_len);
        if (out_len) *out_len = J.size();
        if (J.size() > cap) { ctx->err = "output capacity too small"; return -2; }
        memcpy(out, J.data(), J.size());
        return 0;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_probe_header(const uint8_t* cs, size_t len, gk_image_info* info, gk_cparameters* coding, char* msg,
                    size_t msg_cap) {
    if (!cs || !info) return -1;
    try {
        ByteSrc S; S.len = len; S.host = cs;
        size_t joff = 0, jlen = 0;
        const bool jp2 = jp2_locate(S, joff, jlen);
        if (jp2) { S = ByteSrc(); S.len = jlen; S.host = cs + joff; }
        Header Hd;
        parse_header(S, Hd);
        info->w = Hd.want.w; info->h = Hd.want.h; info->numcomps = Hd.want.nc; info->prec = Hd.want.prec;
        info->sgnd = Hd.want.sgnd; info->x0 = Hd.want.x0; info->y0 = Hd.want.y0;
        info->sample_bytes = 0;
        if (coding) {
            const Params& p = Hd.want.p;
            gk_set_default_params(coding);
            coding->numlayers = (uint16_t)p.nlayers;
            coding->numresolution = (uint8_t)p.numres;
            coding->cblockw_init = 1u << p.cbw; coding->cblockh_init = 1u << p.cbh;
            coding->cblk_sty = (uint8_t)p.cblk_sty;
            coding->irreversible = (uint8_t)p.irrev;
            coding->mct = (uint8_t)p.mct;
            coding->numgbits = (uint8_t)p.numgbits;
            coding->csty = (uint8_t)((p.custom_prc ? 1 : 0) | p.sop_eph);
            coding->res_spec = p.custom_prc ? p.numres : 0;
            for (uint32_t r = 0; r < p.numres; ++r) {   // highest resolution first, as grk_cparameters
                coding->prcw_init[r] = 1u << p.prcw[p.numres - 1 - r];
                coding->prch_init[r] = 1u << p.prch[p.numres - 1 - r];
            }
            coding->tile_size_on = p.tw != 0;
            coding->t_width = p.tw ? p.tw : Hd.want.x0 + Hd.want.w - Hd.want.gx0;
            coding->t_height = p.th ? p.th : Hd.want.y0 + Hd.want.h - Hd.want.gy0;
            coding->tx0 = Hd.want.gx0; coding->ty0 = Hd.want.gy0;
            coding->writeTLM = !Hd.tlm.empty();
            coding->writePLT = 0;
            coding->cod_format = jp2 ? 2 : 0;
            coding->prog_order = (int32_t)p.prog;
        }
        return 0;
    } catch (const GkError& e) {
        if (msg && msg_cap) snprintf(msg, msg_cap, "%s", e.msg.c_str());
        return -1;
    }
}

int gk_decode(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, void* const* comps,
              const uint32_t* strides, uint32_t sample_bytes, int out_on_device) {
    if (!ctx || !cs || !comps || !strides) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        DevBusy busy(ctx->device);
        decode_impl(ctx, cs, len, cs_on_device, comps, strides, sample_bytes, out_on_device);
        return 0;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_set_subsampling(gk_ctx* ctx, uint32_t numcomps, const uint32_t* dx, const uint32_t* dy) {
    if (!ctx) return -1;
    ctx->enc_dx.clear(); ctx->enc_dy.clear();
    if (!numcomps) return 0;
    if (!dx || !dy || numcomps > 255) { ctx->err = "bad subsampling"; return -1; }
    for (uint32_t c = 0; c < numcomps; ++c) {
        if (!dx[c] || !dy[c] || dx[c] > 255 || dy[c] > 255) { ctx->err = "subsampling factors must be 1..255"; return -1; }
        ctx->enc_dx.push_back((uint8_t)dx[c]); ctx->enc_dy.push_back((uint8_t)dy[c]);
    }
    ctx->plan_key.clear();
    return 0;
}

int gk_probe_components(const uint8_t* cs, size_t len, uint32_t* dx, uint32_t* dy, uint32_t* prec, uint32_t* sgnd,
                        uint32_t cap) {
    if (!cs) return -1;
    try {
        ByteSrc S; S.len = len; S.host = cs;
        size_t joff = 0, jlen = 0;
        if (jp2_locate(S, joff, jlen)) { S = ByteSrc(); S.len = jlen; S.host = cs + joff; }
        Header Hd;
        parse_header(S, Hd);
        for (uint32_t c = 0; c < Hd.want.nc && c < cap; ++c) {
            if (dx) dx[c] = Hd.want.sx(c);
            if (dy) dy[c] = Hd.want.sy(c);
            if (prec) prec[c] = Hd.want.c_prec(c);
            if (sgnd) sgnd[c] = Hd.want.c_sgnd(c);
        }
        return (int)Hd.want.nc;
    } catch (const GkError&) {
        return -1;
    }
}

int gk_header_components(gk_ctx* ctx, uint32_t* dx, uint32_t* dy, uint32_t* prec, uint32_t* sgnd, uint32_t cap) {
    if (!ctx) return -1;
    for (uint32_t c = 0; c < ctx->hdr_dx.size() && c < cap; ++c) {
        if (dx) dx[c] = ctx->hdr_dx[c];
        if (dy) dy[c] = ctx->hdr_dy[c];
        if (prec) prec[c] = ctx->hdr_prec[c];
        if (sgnd) sgnd[c] = ctx->hdr_sgnd[c];
    }
    return (int)ctx->hdr_dx.size();
}

int gk_set_window_rule(gk_ctx* ctx, int whole_tile) {
    if (!ctx) return -1;
    ctx->win_whole_tile = whole_tile != 0;
    return 0;
}

int gk_set_decode_reduce(gk_ctx* ctx, uint32_t reduce) {
    if (!ctx || reduce >= GK_MAXRLVLS) return -1;
    ctx->dec_reduce = reduce;
    return 0;
}

int gk_set_decode_layers(gk_ctx* ctx, uint32_t max_layers) {
    if (!ctx) return -1;
    ctx->dec_layers = max_layers;
    return 0;
}

int gk_decode_window(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, uint32_t x0, uint32_t y0,
                     uint32_t x1, uint32_t y1, void* const* comps, const uint32_t* strides, uint32_t sample_bytes,
                     int out_on_device) {
    if (!ctx || !cs || !comps || !strides) return -1;
    try {
        (void)hipSetDevice(ctx->device);
        DevBusy busy(ctx->device);
        const uint32_t win[4] = {x0, y0, x1, y1};
        decode_impl(ctx, cs, len, cs_on_device, comps, strides, sample_bytes, out_on_device, win);
        return 0;
    } catch (const GkError& e) {
        ctx->err = e.msg;
        return -1;
    }
}

int gk_get_timings(gk_ctx* ctx, gk_timings* t) {
    if (!ctx || !t) return -1;
    *t = ctx->tm;
    return 0;
}

const char* gk_last_error(gk_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

const char* gk_version(void) { return "grok_amd 0.1.0 (MI355X gfx950; codestream-compatible with Grok 9.2.0)"; }

}  // extern "C"
