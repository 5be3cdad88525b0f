// grk_shim.cpp — Grok 9.2.0's public C API (grok.h:1082-1657) over the MI355X engine.
//
// src/bin tools and user programs written against grok.h link this
// library instead of libgrokj2k and run unchanged (include/grk_abi.h holds the
// layout-identical structs; INTEGRATION.md §1 the link recipe).  The grk_* objects keep
// Grok's conventions (grok.cpp:75-870): functions return false / NULL on failure and report
// through the grk_set_*_handler callbacks; codecs, streams and images are ref-counted through
// grk_object::wrapper; the composited image belongs to its codec; calls are synchronous.
//
// What runs where: codestream bytes are produced and consumed by gk_encode / gk_decode*
// (tile pipeline on the GPU, T2 on host threads); this file only moves samples between
// grk_image planes and the engine and bytes between grk_stream and host buffers.
#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/grk_abi.h"
#include "../../include/grok_amd.h"
#include "grk_params.h"

namespace {

// ---------------------------------------------------------------------------- messages
struct Handler { grk_msg_callback cb = nullptr; void* ud = nullptr; };
Handler g_info, g_warn, g_err;
void say(const Handler& h, const char* fmt, va_list ap) {
    if (!h.cb) return;
    char buf[1024];
    vsnprintf(buf, sizeof buf, fmt, ap);
    h.cb(buf, h.ud);
}
void error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); say(g_err, fmt, ap); va_end(ap); }
void warn(const char* fmt, ...) { va_list ap; va_start(ap, fmt); say(g_warn, fmt, ap); va_end(ap); }

// ---------------------------------------------------------------------------- engine
// One engine context per process (device from grk_initialize / the codec parameters);
// calls on it are serialised, as Grok serialises calls on one codec.
std::mutex g_eng_m;
gk_ctx* g_eng = nullptr;
int g_device = 0;
gk_ctx* engine() {
    if (!g_eng) {
        g_eng = gk_create(g_device);
        if (!g_eng) error("no HIP device %d for the JPEG 2000 engine", g_device);
    }
    return g_eng;
}

// ---------------------------------------------------------------------------- objects
// grk_object::wrapper points at an Obj; the public struct lives inside the Obj.
struct Obj {
    std::atomic<int> refs{1};
    virtual ~Obj() {}
};
Obj* obj_of(grk_object* o) { return o ? static_cast<Obj*>(o->wrapper) : nullptr; }

inline uint32_t aligned_stride(uint32_t w) { return (w + 31) / 32 * 32; }   // MemManager.cpp:35-43

struct ImageObj : Obj {
    grk_image img{};
    std::vector<grk_image_comp> comps;
    ~ImageObj() override {
        for (auto& c : comps) free(c.data);
        if (img.meta) grk_object_unref(&img.meta->obj);
    }
};
struct MetaObj : Obj {
    grk_image_meta meta{};
    ~MetaObj() override {
        free(meta.color.icc_profile_buf);
        free(meta.iptc_buf);
        free(meta.xmp_buf);
    }
};
ImageObj* new_image(uint16_t n, const grk_image_cmptparm* p, GRK_COLOR_SPACE cs, bool alloc) {
    auto* o = new ImageObj();
    o->comps.assign(n, grk_image_comp{});
    o->img.obj.wrapper = static_cast<Obj*>(o);
    o->img.numcomps = n;
    o->img.color_space = cs;
    o->img.comps = o->comps.data();
    for (uint16_t i = 0; i < n; ++i) {
        grk_image_comp& c = o->comps[i];
        c.dx = p[i].dx ? p[i].dx : 1; c.dy = p[i].dy ? p[i].dy : 1;
        c.w = p[i].w; c.h = p[i].h; c.x0 = p[i].x0; c.y0 = p[i].y0;
        c.prec = p[i].prec; c.sgnd = p[i].sgnd;
        c.stride = p[i].stride ? p[i].stride : aligned_stride(c.w);
        c.type = GRK_COMPONENT_TYPE_COLOUR;
        c.association = GRK_COMPONENT_ASSOC_WHOLE_IMAGE;
        if (alloc && c.w && c.h) {
            c.data = (int32_t*)aligned_alloc(64, ((size_t)c.stride * c.h * 4 + 63) / 64 * 64);
            if (!c.data) { delete o; return nullptr; }
            memset(c.data, 0, (size_t)c.stride * c.h * 4);
        }
    }
    if (n) {
        o->img.x0 = o->comps[0].x0; o->img.y0 = o->comps[0].y0;
        o->img.x1 = o->comps[0].x0 + o->comps[0].w * o->comps[0].dx;
        o->img.y1 = o->comps[0].y0 + o->comps[0].h * o->comps[0].dy;
    }
    return o;
}

// Streams: a memory buffer (read or write), a file, or user callbacks (grk_stream_new).
struct StreamObj : Obj {
    grk_object obj{};
    bool input = true;
    // memory
    uint8_t* mem = nullptr; size_t mem_len = 0, mem_pos = 0; bool owns = false;
    // file
    std::string path;
    bool is_file = false;
    // callbacks
    grk_stream_read_fn rd = nullptr; grk_stream_write_fn wr = nullptr; grk_stream_seek_fn sk = nullptr;
    void* ud = nullptr; grk_stream_free_user_data_fn ud_free = nullptr; uint64_t ud_len = 0;
    bool is_cb = false;
    ~StreamObj() override {
        if (owns) free(mem);
        if (ud_free) ud_free(ud);
    }
    // the whole input
    bool read_all(std::vector<uint8_t>& out) {
        out.clear();
        if (is_file) {
            FILE* f = fopen(path.c_str(), "rb");
            if (!f) { error("cannot open %s", path.c_str()); return false; }
            fseek(f, 0, SEEK_END);
            const long n = ftell(f);
            fseek(f, 0, SEEK_SET);
            out.resize(n > 0 ? (size_t)n : 0);
            const size_t got = out.empty() ? 0 : fread(out.data(), 1, out.size(), f);
            fclose(f);
            if (got != out.size()) { error("short read of %s", path.c_str()); return false; }
            return true;
        }
        if (is_cb) {
            if (!rd) { error("stream has no read function"); return false; }
            if (sk) sk(0, ud);
            const size_t chunk = 1 << 20;
            for (;;) {
                const size_t at = out.size();
                out.resize(at + chunk);
                const size_t got = rd(out.data() + at, chunk, ud);
                if (got == (size_t)-1 || got == 0) { out.resize(at); break; }
                out.resize(at + got);
                if (ud_len && out.size() >= ud_len) break;
            }
            return !out.empty();
        }
        out.assign(mem, mem + mem_len);
        return true;
    }
    bool write_all(const uint8_t* p, size_t n) {
        if (is_file) {
            FILE* f = fopen(path.c_str(), "wb");
            if (!f) { error("cannot create %s", path.c_str()); return false; }
            const size_t put = fwrite(p, 1, n, f);
            fclose(f);
            if (put != n) { error("short write to %s", path.c_str()); return false; }
            return true;
        }
        if (is_cb) {
            if (!wr) { error("stream has no write function"); return false; }
            size_t done = 0;
            while (done < n) {
                const size_t k = wr((void*)(p + done), n - done, ud);
                if (k == 0 || k == (size_t)-1) { error("stream write failed"); return false; }
                done += k;
            }
            return true;
        }
        if (mem_pos + n > mem_len) { error("memory stream too small (%zu bytes needed)", mem_pos + n); return false; }
        memcpy(mem + mem_pos, p, n);
        mem_pos += n;
        return true;
    }
};
StreamObj* stream_of(grk_stream* s) { return s ? dynamic_cast<StreamObj*>(obj_of(s)) : nullptr; }

// Codecs.
struct CodecObj : Obj {
    grk_object obj{};
    bool compress = false;
    GRK_CODEC_FORMAT fmt = GRK_CODEC_J2K;
    grk_stream* stream = nullptr;
    // compress
    grk_cparameters cp{};
    grk_image* image = nullptr;
    std::vector<uint8_t> tile_buf;           // grk_compress_tile: planar raw samples of the image
    std::vector<uint8_t> tile_seen;
    bool encoded = false;
    // decompress
    grk_dparameters dp{};
    std::vector<uint8_t> data;               // the whole input stream
    gk_image_info info{};
    gk_cparameters coding{};
    bool header_read = false;
    uint32_t win[4] = {0, 0, 0, 0};
    bool has_win = false;
    ImageObj* out = nullptr;                 // composited image (owned by the codec)
    bool tile_decoded = false;               // grk_decompress_tile cropped `out` to a tile
    std::vector<uint32_t> cdx, cdy;          // the stream's component subsampling (SIZ XRsiz / YRsiz)
    std::vector<uint32_t> cprec, csgnd;      // and precision / signedness (Ssiz)
    ~CodecObj() override {
        if (stream) grk_object_unref(stream);
        if (image) grk_object_unref(&image->obj);
        if (out) grk_object_unref(&out->img.obj);
    }
};
CodecObj* codec_of(grk_codec* c) { return c ? dynamic_cast<CodecObj*>(obj_of(c)) : nullptr; }

// grk_cparameters -> gk_cparameters (grk_params.h); a refusal goes to the error callback
bool to_gk(const grk_cparameters& g, GRK_CODEC_FORMAT fmt, gk_cparameters& p, const grk_image* im = nullptr) {
    std::string why;
    uint32_t ntiles = 1;
    if (im && im->numcomps && g.tile_size_on && g.t_width && g.t_height) {   // grid from (tx0, ty0) to the image's far corner
        const uint64_t w = (uint64_t)im->x0 + im->comps[0].w - std::min(g.tx0, im->x0);
        const uint64_t h = (uint64_t)im->y0 + im->comps[0].h - std::min(g.ty0, im->y0);
        ntiles = (uint32_t)(((w + g.t_width - 1) / g.t_width) * ((h + g.t_height - 1) / g.t_height));
    }
    if (grk_params_to_gk(g, fmt == GRK_CODEC_JP2, p, why, ntiles)) return true;
    error("%s", why.c_str());
    return false;
}

inline uint32_t ceil_div(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b - 1) / b); }
bool subsampled(const grk_image* im) {
    for (uint16_t i = 0; i < im->numcomps; ++i)
        if (im->comps[i].dx > 1 || im->comps[i].dy > 1) return true;
    return false;
}

bool image_geometry(const grk_image* im, gk_image_info& info) {
    if (!im || !im->numcomps || !im->comps) { error("empty image"); return false; }
    const grk_image_comp& c0 = im->comps[0];
    // subsampled components (grk_image_comp::dx / dy): component c covers the image area
    // [x0, x1) sampled every dx, ceil(x1 / dx) - ceil(x0 / dx) columns (GrkImage.cpp:74-113)
    const bool sub = subsampled(im);
    if (sub && (im->x1 <= im->x0 || im->y1 <= im->y0)) { error("subsampled image without its area (x1, y1)"); return false; }
    for (uint16_t i = 0; i < im->numcomps; ++i) {
        const grk_image_comp& c = im->comps[i];
        const uint32_t dx = c.dx ? c.dx : 1, dy = c.dy ? c.dy : 1;
        const bool size_ok = sub ? (c.w == ceil_div(im->x1, dx) - ceil_div(im->x0, dx) && c.h == ceil_div(im->y1, dy) - ceil_div(im->y0, dy))
                                 : (c.w == c0.w && c.h == c0.h);
        if (!size_ok || c.prec != c0.prec || c.sgnd != c0.sgnd) {
            error("components must share precision, and their sizes follow the image area and subsampling, on this path");
            return false;
        }
    }
    info.w = sub ? im->x1 - im->x0 : c0.w; info.h = sub ? im->y1 - im->y0 : c0.h;
    info.numcomps = im->numcomps; info.prec = c0.prec; info.sgnd = c0.sgnd;
    info.sample_bytes = 0;
    info.x0 = im->x0; info.y0 = im->y0;   // the image area's canvas origin (SIZ XOsiz / YOsiz)
    return true;
}

bool run_encode(CodecObj* C, const void* const* planes, const uint32_t* strides, uint32_t sample_bytes) {
    gk_cparameters p;
    if (!to_gk(C->cp, C->fmt, p, C->image)) return false;
    gk_image_info info;
    if (!image_geometry(C->image, info)) return false;
    info.sample_bytes = sample_bytes;
    if (C->fmt == GRK_CODEC_JP2 && C->image->color_space != GRK_CLRSPC_UNKNOWN &&
        C->image->color_space != (info.numcomps < 3 ? GRK_CLRSPC_GRAY : GRK_CLRSPC_SRGB)) {
        error("JP2 output supports sRGB (3+ components) or greyscale colour spaces on this path");
        return false;
    }
    std::lock_guard<std::mutex> lk(g_eng_m);
    gk_ctx* e = engine();
    if (!e) return false;
    std::vector<uint32_t> dx(info.numcomps), dy(info.numcomps);
    for (uint32_t c = 0; c < info.numcomps; ++c) {
        dx[c] = C->image->comps[c].dx ? C->image->comps[c].dx : 1; dy[c] = C->image->comps[c].dy ? C->image->comps[c].dy : 1;
    }
    if (gk_set_subsampling(e, subsampled(C->image) ? info.numcomps : 0, dx.data(), dy.data()) != 0) {
        error("%s", gk_last_error(e));
        return false;
    }
    std::vector<uint8_t> out((size_t)info.w * info.h * info.numcomps * 4 + (1 << 20));
    size_t n = 0;
    int rc = gk_encode(e, &info, planes, strides, 0, &p, out.data(), out.size(), &n, 0);
    if (rc == -2) {
        out.resize(n);
        rc = gk_encode(e, &info, planes, strides, 0, &p, out.data(), out.size(), &n, 0);
    }
    gk_set_subsampling(e, 0, nullptr, nullptr);
    if (rc != 0) { error("%s", gk_last_error(e)); return false; }
    StreamObj* s = stream_of(C->stream);
    if (!s || !s->write_all(out.data(), n)) return false;
    C->encoded = true;
    return true;
}

// decode into `o` (its comps sized for the region) — the whole image or the window `w`;
// whole_tile: a tile decode with no window set keeps Grok's whole-tile inverse rule
bool run_decode(CodecObj* C, ImageObj* o, const uint32_t* w, bool whole_tile = false) {
    std::lock_guard<std::mutex> lk(g_eng_m);
    gk_ctx* e = engine();
    if (!e) return false;
    std::vector<void*> planes(o->img.numcomps);
    std::vector<uint32_t> strides(o->img.numcomps);
    for (uint16_t i = 0; i < o->img.numcomps; ++i) { planes[i] = o->comps[i].data; strides[i] = o->comps[i].stride; }
    gk_set_decode_layers(e, C->dp.cp_layer);   // 0 = every layer
    gk_set_decode_reduce(e, C->dp.cp_reduce);
    gk_set_window_rule(e, whole_tile ? 1 : 0);
    int rc = w ? gk_decode_window(e, C->data.data(), C->data.size(), 0, w[0], w[1], w[2], w[3], planes.data(),
                                  strides.data(), 0, 0)
               : gk_decode(e, C->data.data(), C->data.size(), 0, planes.data(), strides.data(), 0, 0);
    gk_set_window_rule(e, 0);
    if (rc != 0) { error("%s", gk_last_error(e)); return false; }
    return true;
}

// The composited image keeps its canvas bounds (the image area, or the window) at full
// resolution while its components take them reduced by cp_reduce, ceil(x / 2^reduce)
// (GrkImage::subsampleAndReduce, GrkImage.cpp:74-113; SIZMarker.cpp:292 for the header image,
// CodeStreamDecompress.cpp:390 after a window)
static inline uint32_t reduced(uint64_t v, uint32_t r) { return (uint32_t)((v + (1ull << r) - 1) >> r); }

ImageObj* region_image(CodecObj* C, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    const uint32_t r = C->dp.cp_reduce;
    std::vector<grk_image_cmptparm> p(C->info.numcomps);
    for (uint32_t k = 0; k < p.size(); ++k) {
        grk_image_cmptparm& q = p[k];
        q = grk_image_cmptparm{};
        // (a subsampled component: the rectangle on its grid, then reduced; GrkImage.cpp:74-113)
        q.dx = C->cdx[k]; q.dy = C->cdy[k];
        q.x0 = reduced(ceil_div(x0, q.dx), r); q.y0 = reduced(ceil_div(y0, q.dy), r);
        q.w = reduced(ceil_div(x1, q.dx), r) - q.x0; q.h = reduced(ceil_div(y1, q.dy), r) - q.y0;
        q.prec = (uint8_t)C->cprec[k]; q.sgnd = C->csgnd[k] != 0;
    }
    GRK_COLOR_SPACE cs = GRK_CLRSPC_UNKNOWN;
    if (C->coding.cod_format == 2) cs = C->info.numcomps < 3 ? GRK_CLRSPC_GRAY : GRK_CLRSPC_SRGB;
    // sample memory is attached by the decompress call (Grok allocates the composite's planes
    // at decompress time too), so a header read of a 32768^2 .jp2 holds no planes
    ImageObj* o = new_image((uint16_t)C->info.numcomps, p.data(), cs, false);
    if (o) { o->img.x0 = x0; o->img.y0 = y0; o->img.x1 = x1; o->img.y1 = y1; }
    return o;
}

// Re-bound the composited image in place and give it planes: callers keep the pointer that
// grk_decompress_get_composited_image returned after the header read (grk_decompress.cpp:1191
// takes it before set_window / decompress), as Grok edits the one composite image in place
// (CodeStreamDecompress.cpp:335-387, :451-481).  (x0, y0, x1, y1): canvas bounds at full
// resolution; the components take them reduced by r.
bool reshape_image(ImageObj* o, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t r) {
    o->img.x0 = x0; o->img.y0 = y0; o->img.x1 = x1; o->img.y1 = y1;
    for (auto& c : o->comps) {
        const uint32_t dx = c.dx ? c.dx : 1, dy = c.dy ? c.dy : 1;
        const uint32_t cx0 = reduced(ceil_div(x0, dx), r), cy0 = reduced(ceil_div(y0, dy), r);
        const uint32_t cw = reduced(ceil_div(x1, dx), r) - cx0, ch = reduced(ceil_div(y1, dy), r) - cy0;
        if (!cw || !ch) { error("the decompress region is empty at reduction %u", r); return false; }
        const uint32_t stride = aligned_stride(cw);
        if (c.data && (c.w != cw || c.h != ch || c.stride != stride)) { free(c.data); c.data = nullptr; }
        c.x0 = cx0; c.y0 = cy0; c.w = cw; c.h = ch; c.stride = stride;
        if (!c.data && c.w && c.h) {
            c.data = (int32_t*)aligned_alloc(64, ((size_t)c.stride * c.h * 4 + 63) / 64 * 64);
            if (!c.data) { error("out of memory for a %ux%u component", c.w, c.h); return false; }
        }
    }
    return true;
}

}  // namespace

extern "C" {

const char* grk_version(void) { return "9.2.0"; }   // the codestream COM text names this version

// grok.cpp:71-86 sizes the thread pool and loads the plugin.  The engine (and its HIP context)
// is created by the first call that codes, so an initialise on a host without a GPU succeeds and
// the refusal comes from that call, as Grok's own CPU path would only fail there.
bool grk_initialize(const char* pluginPath, uint32_t numthreads) {
    (void)pluginPath; (void)numthreads;   // no separate plugin; host T2 threads are sized by the engine
    return true;
}

void grk_deinitialize(void) {
    std::lock_guard<std::mutex> lk(g_eng_m);
    if (g_eng) gk_destroy(g_eng);
    g_eng = nullptr;
}

void grk_object_ref(grk_object* obj) {
    if (Obj* o = obj_of(obj)) o->refs++;
}
void grk_object_unref(grk_object* obj) {
    Obj* o = obj_of(obj);
    if (o && --o->refs == 0) delete o;
}

bool grk_set_info_handler(grk_msg_callback cb, void* ud) { g_info = {cb, ud}; return true; }
bool grk_set_warning_handler(grk_msg_callback cb, void* ud) { g_warn = {cb, ud}; return true; }
bool grk_set_error_handler(grk_msg_callback cb, void* ud) { g_err = {cb, ud}; return true; }

grk_image* grk_image_new(uint16_t numcmpts, grk_image_cmptparm* cmptparms, GRK_COLOR_SPACE clrspc, bool allocData) {
    if (!numcmpts || !cmptparms) return nullptr;
    ImageObj* o = new_image(numcmpts, cmptparms, clrspc, allocData);
    return o ? &o->img : nullptr;
}
grk_image_meta* grk_image_meta_new(void) {
    auto* m = new MetaObj();
    m->meta.obj.wrapper = static_cast<Obj*>(m);
    return &m->meta;
}
void grk_image_single_component_data_free(grk_image_comp* comp) {
    if (!comp) return;
    free(comp->data);
    comp->data = nullptr;
}
void grk_image_all_components_data_free(grk_image* image) {
    if (!image) return;
    for (uint16_t i = 0; i < image->numcomps; ++i) grk_image_single_component_data_free(image->comps + i);
}

grk_stream* grk_stream_new(size_t buffer_size, bool is_input) {
    (void)buffer_size;
    auto* s = new StreamObj();
    s->obj.wrapper = static_cast<Obj*>(s);
    s->input = is_input;
    s->is_cb = true;
    return &s->obj;
}
void grk_stream_set_read_function(grk_stream* st, grk_stream_read_fn f) { if (auto* s = stream_of(st)) s->rd = f; }
void grk_stream_set_write_function(grk_stream* st, grk_stream_write_fn f) { if (auto* s = stream_of(st)) s->wr = f; }
void grk_stream_set_seek_function(grk_stream* st, grk_stream_seek_fn f) { if (auto* s = stream_of(st)) s->sk = f; }
void grk_stream_set_user_data(grk_stream* st, void* data, grk_stream_free_user_data_fn f) {
    if (auto* s = stream_of(st)) { s->ud = data; s->ud_free = f; }
}
void grk_stream_set_user_data_length(grk_stream* st, uint64_t n) { if (auto* s = stream_of(st)) s->ud_len = n; }
grk_stream* grk_stream_create_file_stream(const char* fname, size_t buffer_size, bool is_read_stream) {
    (void)buffer_size;
    if (!fname) return nullptr;
    auto* s = new StreamObj();
    s->obj.wrapper = static_cast<Obj*>(s);
    s->input = is_read_stream;
    s->is_file = true;
    s->path = fname;
    return &s->obj;
}
grk_stream* grk_stream_create_mapped_file_stream(const char* fname, bool read_stream) {
    return grk_stream_create_file_stream(fname, 0, read_stream);
}
grk_stream* grk_stream_create_mem_stream(uint8_t* buf, size_t len, bool ownsBuffer, bool is_read_stream) {
    if (!buf || !len) return nullptr;
    auto* s = new StreamObj();
    s->obj.wrapper = static_cast<Obj*>(s);
    s->input = is_read_stream;
    s->mem = buf; s->mem_len = len; s->owns = ownsBuffer;
    return &s->obj;
}
size_t grk_stream_get_write_mem_stream_length(grk_stream* st) {
    auto* s = stream_of(st);
    return s && !s->input ? s->mem_pos : 0;
}

// ----------------------------------------------------------------------------- compress
grk_codec* grk_compress_create(GRK_CODEC_FORMAT format, grk_stream* stream) {
    if (format != GRK_CODEC_J2K && format != GRK_CODEC_JP2) return nullptr;
    if (!stream_of(stream)) return nullptr;
    auto* c = new CodecObj();
    c->obj.wrapper = static_cast<Obj*>(c);
    c->compress = true;
    c->fmt = format;
    c->stream = stream;
    grk_object_ref(stream);
    return &c->obj;
}

void grk_compress_set_default_params(grk_cparameters* p) {   // grok.cpp:405-435
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->rsiz = GRK_PROFILE_NONE;
    p->numresolution = 6;
    p->cblockw_init = 64; p->cblockh_init = 64;
    p->numgbits = 2;
    p->prog_order = GRK_LRCP;
    p->roi_compno = -1;
    p->subsampling_dx = 1; p->subsampling_dy = 1;
    p->decod_format = GRK_UNK_FMT; p->cod_format = GRK_UNK_FMT;
    p->numThreads = std::max(1u, std::thread::hardware_concurrency());
    p->deviceId = 0;
    p->repeats = 1;
}

bool grk_compress_init(grk_codec* codec, grk_cparameters* parameters, grk_image* image) {
    CodecObj* C = codec_of(codec);
    if (!C || !C->compress || !parameters || !image) return false;
    gk_cparameters probe;
    if (!to_gk(*parameters, C->fmt, probe, image)) return false;
    gk_image_info info;
    if (!image_geometry(image, info)) return false;
    C->cp = *parameters;
    if (C->image) grk_object_unref(&C->image->obj);
    C->image = image;
    grk_object_ref(&image->obj);
    g_device = parameters->deviceId >= 0 ? parameters->deviceId : 0;
    return true;
}

bool grk_compress_start(grk_codec* codec) {
    CodecObj* C = codec_of(codec);
    return C && C->compress && C->image;
}

bool grk_compress_with_plugin(grk_codec* codec, grk_plugin_tile* tile) {
    CodecObj* C = codec_of(codec);
    if (!C || !C->compress || !C->image) return false;
    if (tile) { error("plugin tiles are not used: the tile pipeline runs in this library"); return false; }
    const grk_image* im = C->image;
    std::vector<const void*> planes(im->numcomps);
    std::vector<uint32_t> strides(im->numcomps);
    for (uint16_t i = 0; i < im->numcomps; ++i) {
        if (!im->comps[i].data) { error("image component %u has no data", i); return false; }
        planes[i] = im->comps[i].data;
        strides[i] = im->comps[i].stride ? im->comps[i].stride : im->comps[i].w;
    }
    return run_encode(C, planes.data(), strides.data(), 0);
}

bool grk_compress(grk_codec* codec) { return grk_compress_with_plugin(codec, nullptr); }

// Raw tile samples, planar per component, (prec + 7) / 8 bytes each (TileProcessor::
// ingestUncompressedData, TileProcessor.cpp:779-835); the image is coded once every tile arrived.
bool grk_compress_tile(grk_codec* codec, uint16_t tileIndex, uint8_t* data, uint64_t data_size) {
    CodecObj* C = codec_of(codec);
    if (!C || !C->compress || !C->image || !data) return false;
    gk_image_info info;
    if (!image_geometry(C->image, info)) return false;
    if (subsampled(C->image)) { error("raw tiles of subsampled components are not supported on this path"); return false; }
    const uint32_t es = (info.prec + 7) / 8;
    if (es > 2) { error("raw tiles of more than 16 bits per sample are not supported"); return false; }
    if (C->cp.tile_size_on && (!C->cp.t_width || !C->cp.t_height)) { error("tile size must be non-zero"); return false; }
    // tile grid from (tx0, ty0) over the image area [X0, X1) x [Y0, Y1) (B.3); x0, y0 below are
    // image-relative
    const uint32_t X0 = info.x0, Y0 = info.y0, X1 = X0 + info.w, Y1 = Y0 + info.h;
    const uint32_t gx = std::min(C->cp.tx0, X0), gy = std::min(C->cp.ty0, Y0);
    const uint32_t tw = C->cp.tile_size_on ? C->cp.t_width : X1 - gx;
    const uint32_t th = C->cp.tile_size_on ? C->cp.t_height : Y1 - gy;
    const uint32_t ntx = (X1 - gx + tw - 1) / tw, nty = (Y1 - gy + th - 1) / th;
    if (tileIndex >= ntx * nty) { error("tile index %u out of range", tileIndex); return false; }
    const uint32_t x0 = std::max(gx + (tileIndex % ntx) * tw, X0) - X0, y0 = std::max(gy + (tileIndex / ntx) * th, Y0) - Y0;
    const uint32_t w = std::min(gx + (tileIndex % ntx + 1) * tw, X1) - X0 - x0;
    const uint32_t h = std::min(gy + (tileIndex / ntx + 1) * th, Y1) - Y0 - y0;
    if (data_size != (uint64_t)w * h * info.numcomps * es) { error("tile %u: wrong data size", tileIndex); return false; }
    if (C->tile_buf.empty()) {
        C->tile_buf.assign((size_t)info.w * info.h * info.numcomps * es, 0);
        C->tile_seen.assign((size_t)ntx * nty, 0);
    }
    for (uint32_t c = 0; c < info.numcomps; ++c)
        for (uint32_t y = 0; y < h; ++y)
            memcpy(C->tile_buf.data() + (((size_t)c * info.h + y0 + y) * info.w + x0) * es,
                   data + (((size_t)c * h + y) * w) * es, (size_t)w * es);
    C->tile_seen[tileIndex] = 1;
    if (std::find(C->tile_seen.begin(), C->tile_seen.end(), 0) != C->tile_seen.end()) return true;
    std::vector<const void*> planes(info.numcomps);
    std::vector<uint32_t> strides(info.numcomps, info.w);
    for (uint32_t c = 0; c < info.numcomps; ++c) planes[c] = C->tile_buf.data() + (size_t)c * info.w * info.h * es;
    return run_encode(C, planes.data(), strides.data(), es);
}

bool grk_compress_end(grk_codec* codec) {
    CodecObj* C = codec_of(codec);
    if (!C || !C->compress) return false;
    if (!C->encoded) { error("grk_compress_end before the image was compressed"); return false; }
    return true;
}

bool grk_set_MCT(grk_cparameters* parameters, float* pEncodingMatrix, int32_t* p_dc_shift, uint32_t pNbComp) {
    (void)parameters; (void)pEncodingMatrix; (void)p_dc_shift; (void)pNbComp;
    error("Part-2 array MCT (grk_set_MCT) is not supported on this path");
    return false;
}

// ----------------------------------------------------------------------------- decompress
grk_codec* grk_decompress_create(GRK_CODEC_FORMAT format, grk_stream* stream) {
    if (format != GRK_CODEC_J2K && format != GRK_CODEC_JP2) return nullptr;
    if (!stream_of(stream)) return nullptr;
    auto* c = new CodecObj();
    c->obj.wrapper = static_cast<Obj*>(c);
    c->fmt = format;
    c->stream = stream;
    grk_object_ref(stream);
    return &c->obj;
}

void grk_decompress_set_default_params(grk_dparameters* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->tileCacheStrategy = GRK_TILE_CACHE_NONE;
}

bool grk_decompress_init(grk_codec* codec, grk_dparameters* parameters) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress || !parameters) return false;
    C->dp = *parameters;
    if (parameters->DA_x1 > parameters->DA_x0 && parameters->DA_y1 > parameters->DA_y0) {
        C->win[0] = parameters->DA_x0; C->win[1] = parameters->DA_y0;
        C->win[2] = parameters->DA_x1; C->win[3] = parameters->DA_y1;
        C->has_win = true;
    }
    return true;
}

bool grk_decompress_read_header(grk_codec* codec, grk_header_info* hi) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress) return false;
    if (!C->header_read) {
        StreamObj* s = stream_of(C->stream);
        if (!s || !s->read_all(C->data)) return false;
        char msg[256];
        if (gk_probe_header(C->data.data(), C->data.size(), &C->info, &C->coding, msg, sizeof msg) != 0) {
            error("%s", msg);
            return false;
        }
        C->cdx.assign(C->info.numcomps, 1); C->cdy.assign(C->info.numcomps, 1);
        C->cprec.assign(C->info.numcomps, C->info.prec); C->csgnd.assign(C->info.numcomps, C->info.sgnd);
        if (gk_probe_components(C->data.data(), C->data.size(), C->cdx.data(), C->cdy.data(), C->cprec.data(),
                                C->csgnd.data(), C->info.numcomps) < 0) {
            error("cannot read the component subsampling");
            return false;
        }
        C->header_read = true;
        if (C->dp.cp_reduce >= C->coding.numresolution) {
            error("reduce %u must be less than the number of resolutions %u", C->dp.cp_reduce, C->coding.numresolution);
            return false;
        }
        // the composited image: the image area on the canvas (components reduced by cp_reduce)
        C->out = region_image(C, C->info.x0, C->info.y0, C->info.x0 + C->info.w, C->info.y0 + C->info.h);
        if (!C->out) return false;
    }
    if (hi) {
        const gk_cparameters& k = C->coding;
        hi->cblockw_init = k.cblockw_init; hi->cblockh_init = k.cblockh_init;
        hi->irreversible = k.irreversible != 0;
        hi->mct = k.mct;
        hi->rsiz = (k.cblk_sty & GRK_CBLKSTY_HT) ? GRK_JPH_RSIZ_FLAG : GRK_PROFILE_NONE;
        hi->numresolutions = k.numresolution;
        hi->csty = k.csty;
        hi->cblk_sty = k.cblk_sty;
        for (int r = 0; r < GRK_J2K_MAXRLVLS; ++r) { hi->prcw_init[r] = k.prcw_init[r]; hi->prch_init[r] = k.prch_init[r]; }
        hi->tx0 = k.tx0; hi->ty0 = k.ty0;
        hi->t_width = k.t_width; hi->t_height = k.t_height;
        hi->t_grid_width = (C->info.x0 + C->info.w - k.tx0 + k.t_width - 1) / k.t_width;
        hi->t_grid_height = (C->info.y0 + C->info.h - k.ty0 + k.t_height - 1) / k.t_height;
        hi->numlayers = k.numlayers;
        hi->xml_data = nullptr; hi->xml_data_len = 0;
        hi->num_comments = 0;
        hi->num_asocs = 0;
    }
    return true;
}

// CodeStreamDecompress::setDecompressWindow (CodeStreamDecompress.cpp:295-398): (0,0,0,0) is the
// whole image — grk_decompress.cpp:1259 always calls this, with the -d values or zeros; a left or
// top edge past the image is an error; a right or bottom edge past it is clamped with a warning.
bool grk_decompress_set_window(grk_codec* codec, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress) return false;
    if (!C->header_read) { error("Need to read the main header before setting decompress window"); return false; }
    if (!x0 && !y0 && !x1 && !y1) { C->has_win = false; return true; }
    // the window is relative to the image origin; Grok reports canvas positions (window + origin)
    const uint32_t W = C->info.w, H = C->info.h, OX = C->info.x0, OY = C->info.y0;
    if (x0 > W) { error("Left position of the decompress window (%u) is outside of the image area (Xsiz=%u).", x0 + OX, W + OX); return false; }
    if (y0 > H) { error("Top position of the decompress window (%u) is outside of the image area (Ysiz=%u).", y0 + OY, H + OY); return false; }
    if (x1 > W) { warn("Right position of the decompress window (%u) is outside the image area (Xsiz=%u).", x1 + OX, W + OX); x1 = W; }
    if (y1 > H) { warn("Bottom position of the decompress window (%u) is outside of the image area (Ysiz=%u).", y1 + OY, H + OY); y1 = H; }
    if (x0 >= x1 || y0 >= y1) { error("decompress window (%u,%u,%u,%u) is empty", x0, y0, x1, y1); return false; }
    C->win[0] = x0; C->win[1] = y0; C->win[2] = x1; C->win[3] = y1;
    C->has_win = true;
    return true;
}

bool grk_decompress(grk_codec* codec, grk_plugin_tile* tile) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress) return false;
    if (tile) { error("plugin tiles are not used: the tile pipeline runs in this library"); return false; }
    if (!C->header_read && !grk_decompress_read_header(codec, nullptr)) return false;
    const uint32_t OX = C->info.x0, OY = C->info.y0;   // composited images are canvas rectangles
    if (C->has_win) {
        // (the components: the window's canvas rectangle reduced by cp_reduce)
        if (!reshape_image(C->out, C->win[0] + OX, C->win[1] + OY, C->win[2] + OX, C->win[3] + OY, C->dp.cp_reduce))
            return false;
        return run_decode(C, C->out, C->win);
    }
    if (!reshape_image(C->out, OX, OY, OX + C->info.w, OY + C->info.h, C->dp.cp_reduce)) return false;
    return run_decode(C, C->out, nullptr);
}

// CodeStreamDecompress::decompressTile (CodeStreamDecompress.cpp:416-493): the composited image
// is cropped to the tile (intersected with the window when one is set) and the tile decodes
// into it; grk_decompress_get_tile_image then returns that image.
bool grk_decompress_tile(grk_codec* codec, uint16_t tileIndex) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress) return false;
    if (!C->header_read && !grk_decompress_read_header(codec, nullptr)) return false;
    const uint32_t tw = C->coding.t_width, th = C->coding.t_height;
    const uint32_t OX = C->info.x0, OY = C->info.y0, X1 = OX + C->info.w, Y1 = OY + C->info.h;
    const uint32_t gx = C->coding.tx0, gy = C->coding.ty0;
    const uint32_t ntx = (X1 - gx + tw - 1) / tw, nty = (Y1 - gy + th - 1) / th;
    if (tileIndex >= ntx * nty) {
        error("Tile index %u is greater than maximum tile index %u", tileIndex, ntx * nty - 1);
        return false;
    }
    // the tile's rectangle on the canvas, clipped to the image area, made image-relative
    const uint32_t i = tileIndex % ntx, j = tileIndex / ntx;
    uint32_t w[4] = {std::max(gx + i * tw, OX) - OX, std::max(gy + j * th, OY) - OY, std::min(gx + (i + 1) * tw, X1) - OX,
                     std::min(gy + (j + 1) * th, Y1) - OY};
    if (C->has_win) {
        const uint32_t c[4] = {std::max(w[0], C->win[0]), std::max(w[1], C->win[1]), std::min(w[2], C->win[2]),
                               std::min(w[3], C->win[3])};
        if (c[0] < c[2] && c[1] < c[3]) { w[0] = c[0]; w[1] = c[1]; w[2] = c[2]; w[3] = c[3]; }
        else {
            warn("Decompress bounds <%u,%u,%u,%u> do not overlap with requested tile %u. Decompressing full image",
                 C->win[0], C->win[1], C->win[2], C->win[3], tileIndex);
            w[0] = C->win[0]; w[1] = C->win[1]; w[2] = C->win[2]; w[3] = C->win[3];
        }
    }
    // (with cp_reduce the components take the tile's rectangle reduced, CodeStreamDecompress.cpp:471-481)
    if (!reshape_image(C->out, w[0] + OX, w[1] + OY, w[2] + OX, w[3] + OY, C->dp.cp_reduce)) return false;
    C->tile_decoded = true;
    // wholeTileDecompress stays set unless a window was (CodeStreamDecompress.cpp:389)
    return run_decode(C, C->out, w, !C->has_win);
}

grk_image* grk_decompress_get_tile_image(grk_codec* codec, uint16_t tileIndex) {
    (void)tileIndex;
    CodecObj* C = codec_of(codec);
    return C && C->tile_decoded ? &C->out->img : nullptr;
}

grk_image* grk_decompress_get_composited_image(grk_codec* codec) {
    CodecObj* C = codec_of(codec);
    return C && C->out ? &C->out->img : nullptr;
}

bool grk_decompress_end(grk_codec* codec) {
    CodecObj* C = codec_of(codec);
    return C && !C->compress;
}

void grk_dump_codec(grk_codec* codec, uint32_t info_flag, FILE* f) {
    CodecObj* C = codec_of(codec);
    if (!C || C->compress || !C->header_read || !f) return;
    if (info_flag & GRK_IMG_INFO)
        fprintf(f, "Image info {\n\t x0=%u, y0=%u\n\t x1=%u, y1=%u\n\t numcomps=%u\n\t prec=%u sgnd=%u\n}\n",
                C->info.x0, C->info.y0, C->info.x0 + C->info.w, C->info.y0 + C->info.h, C->info.numcomps, C->info.prec,
                C->info.sgnd);
    if (info_flag & GRK_J2K_MH_INFO)
        fprintf(f, "Codestream info from main header: {\n\t tdx=%u, tdy=%u\n\t numresolutions=%u\n\t cblkw=%u cblkh=%u "
                   "cblksty=0x%x\n\t qmfbid=%u mct=%u numlayers=%u\n}\n",
                C->coding.t_width, C->coding.t_height, C->coding.numresolution, C->coding.cblockw_init,
                C->coding.cblockh_init, C->coding.cblk_sty, C->coding.irreversible ? 0 : 1, C->coding.mct,
                C->coding.numlayers);
}

// ----------------------------------------------------------------------------- plugin management
bool grk_plugin_load(grk_plugin_load_info info) { (void)info; return false; }
void grk_plugin_cleanup(void) {}
uint32_t grk_plugin_get_debug_state(void) { return GRK_PLUGIN_STATE_NO_DEBUG; }
bool grk_plugin_init(grk_plugin_init_info initInfo) { (void)initInfo; return false; }
int32_t grk_plugin_compress(grk_cparameters* p, GRK_PLUGIN_COMPRESS_USER_CALLBACK cb) { (void)p; (void)cb; return -1; }
int32_t grk_plugin_batch_compress(const char* in, const char* out, grk_cparameters* p, GRK_PLUGIN_COMPRESS_USER_CALLBACK cb) {
    (void)in; (void)out; (void)p; (void)cb;
    return -1;
}
bool grk_plugin_is_batch_complete(void) { return true; }
void grk_plugin_stop_batch_compress(void) {}
int32_t grk_plugin_decompress(grk_decompress_parameters* p, grk_plugin_decompress_callback cb) { (void)p; (void)cb; return -1; }
int32_t grk_plugin_init_batch_decompress(const char* in, const char* out, grk_decompress_parameters* p,
                                         grk_plugin_decompress_callback cb) {
    (void)in; (void)out; (void)p; (void)cb;
    return -1;
}
int32_t grk_plugin_batch_decompress(void) { return -1; }
void grk_plugin_stop_batch_decompress(void) {}

}  // extern "C"
