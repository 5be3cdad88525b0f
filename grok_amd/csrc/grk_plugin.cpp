// grk_plugin.cpp — Grok 9.2.0's T1 plugin (libgrokj2k_plugin.so) over
// the MI355X engine, for an unmodified Grok host built with the plugin loader.
//
// Compress (grk_compress -g <dir>, grk_compress.cpp:2171-2289 -> grok.cpp:648-677):
// plugin_encode reads the input image, runs DC shift / MCT / DWT / T1 of the single tile on
// the GPU (gk_encode_blocks) and hands the host the code-block tree (grk_plugin_tile ->
// tileComponents -> resolutions -> band -> precincts -> blocks, grok.h:995-1077) through the
// callback.  The host loads the image itself (info.image = NULL), skips its own DC/MCT/DWT/T1
// (TileProcessor.cpp:217-232) and takes every block's bytes, bit-plane count and passes in
// compress_synch_with_plugin (plugin/plugin_bridge.cpp:146-270), then runs PCRD / T2.  The
// host derives a pass rate as plugin rate + 1, clamped to the block length, minus one if that
// byte is 0xFF (:249-262), so the tree carries Grok's rate - 1; every node and buffer belongs
// to the plugin and lives until the callback returns (the host aliases the bytes until T2
// is done, :213-216).
//
// Decompress (grk_decompress -g <dir>, grk_decompress.cpp:886-990 -> grok.cpp:764-780): the
// GRK_DECODE_* flags select the stages the host runs (TileProcessor.cpp:319-338).  The plugin
// asks the host for the header only (GRK_DECODE_HEADER with init_decompressors_func: the CLI's
// preProcess opens the codec, reads the header, prepares its output writer and returns the
// init function's result, grk_decompress.cpp:1181-1237), decodes the whole codestream on the
// GPU (T2 + T1 + inverse DWT + MCT: gk_decode / gk_decode_window) into an image it owns, and
// hands that image to the host's GRK_DECODE_POST_T1 stage (postProcess writes the output file),
// then GRK_PLUGIN_DECODE_CLEAN releases the host codec.
//
// A configuration outside the GPU path returns -1 ("not handled"): the CLI then runs its CPU
// path (grk_compress.cpp:2281-2289, grk_decompress.cpp:1590-1602).  The plugin tile is one tile
// (B2 is single-tile only).
#include <dirent.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/grk_plugin_abi.h"
#include "../../include/grok_amd.h"
#include "grk_params.h"

namespace {

std::mutex g_m;
gk_ctx* g_eng = nullptr;
int g_device = 0;
bool g_verbose = false;

void note(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "[grok_amd plugin] ");
    vfprintf(stderr, fmt, ap);
    fputc('\n', stderr);
    va_end(ap);
}

gk_ctx* engine() {
    if (!g_eng) g_eng = gk_create(g_device);
    return g_eng;
}

// ---------------------------------------------------------------------------- input images
// Binary PNM, as Grok's PNMFormat reads it (src/bin/image_format/PNMFormat.cpp:398-560): P5 grey
// or P6 RGB, precision floorlog2(maxval) + 1, 16-bit samples big-endian.
struct Raster {
    uint32_t w = 0, h = 0, nc = 0, prec = 0;
    std::vector<uint8_t> planes;   // planar, (prec + 7) / 8 bytes per sample
};

bool read_pnm(const char* path, Raster& R, std::string& why) {
    FILE* f = fopen(path, "rb");
    if (!f) { why = std::string("cannot open ") + path; return false; }
    std::vector<uint8_t> d;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    d.resize(n > 0 ? (size_t)n : 0);
    const size_t got = d.empty() ? 0 : fread(d.data(), 1, d.size(), f);
    fclose(f);
    if (got != d.size() || d.size() < 3 || d[0] != 'P' || (d[1] != '5' && d[1] != '6')) {
        why = "input is not a binary PNM (P5 / P6) image";
        return false;
    }
    size_t i = 2;
    uint32_t v[3];
    for (int k = 0; k < 3; ++k) {
        for (;;) {
            while (i < d.size() && isspace(d[i])) ++i;
            if (i < d.size() && d[i] == '#') { while (i < d.size() && d[i] != '\n') ++i; continue; }
            break;
        }
        uint64_t x = 0;
        const size_t s = i;
        while (i < d.size() && isdigit(d[i])) { x = x * 10 + (d[i] - '0'); if (x > 0xffffffffull) break; ++i; }
        if (i == s || x == 0 || x > 0xffffffffull) { why = "bad PNM header"; return false; }
        v[k] = (uint32_t)x;
    }
    ++i;   // one whitespace byte before the raster
    if (v[2] > 65535) { why = "PNM maxval above 65535"; return false; }
    R.w = v[0]; R.h = v[1]; R.nc = d[1] == '6' ? 3 : 1;
    uint32_t p = 0;
    for (uint32_t m = v[2]; m; m >>= 1) ++p;
    R.prec = p;
    const size_t es = p > 8 ? 2 : 1, npix = (size_t)R.w * R.h;
    if (i > d.size() || d.size() - i < npix * R.nc * es) { why = "truncated PNM raster"; return false; }
    R.planes.resize(npix * R.nc * es);
    const uint8_t* src = d.data() + i;
    for (size_t q = 0; q < npix; ++q)
        for (uint32_t c = 0; c < R.nc; ++c) {
            const uint8_t* s = src + (q * R.nc + c) * es;
            if (es == 1) R.planes[c * npix + q] = s[0];
            else {
                const uint16_t x = (uint16_t)((s[0] << 8) | s[1]);
                memcpy(&R.planes[(c * npix + q) * 2], &x, 2);
            }
        }
    return true;
}

// ---------------------------------------------------------------------------- the block tree
// grk_plugin_tile and its nodes, built from the engine's results in canonical order.  Every
// level is a contiguous array plus the pointer array the parent holds.
struct Tree {
    grk_plugin_tile tile{};
    std::vector<grk_plugin_tile_component> comps;
    std::vector<grk_plugin_tile_component*> comp_p;
    std::vector<grk_plugin_resolution> res;
    std::vector<grk_plugin_resolution*> res_p;
    std::vector<grk_plugin_band> bands;
    std::vector<grk_plugin_band*> band_p;
    std::vector<grk_plugin_precinct> prcs;
    std::vector<grk_plugin_precinct*> prc_p;
    std::vector<grk_plugin_code_block> blocks;
    std::vector<grk_plugin_code_block*> block_p;
    std::vector<uint8_t> data;
};

bool build_tree(Tree& T, uint32_t nc, uint32_t numres, const std::vector<gk_band_result>& B,
                const std::vector<gk_block_result>& K, const std::vector<gk_pass_result>& PS, std::string& why) {
    size_t nprc = 0;
    for (const auto& b : B) nprc += b.num_precincts;
    T.comps.assign(nc, grk_plugin_tile_component{});
    T.comp_p.resize(nc);
    T.res.assign((size_t)nc * numres, grk_plugin_resolution{});
    T.res_p.resize(T.res.size());
    T.bands.assign(B.size(), grk_plugin_band{});
    T.band_p.resize(B.size());
    T.prcs.assign(nprc, grk_plugin_precinct{});
    T.prc_p.resize(nprc);
    T.blocks.assign(K.size(), grk_plugin_code_block{});
    T.block_p.resize(K.size());
    for (size_t i = 0; i < K.size(); ++i) T.block_p[i] = &T.blocks[i];
    T.tile.decompress_flags = 0;
    T.tile.numComponents = nc;
    T.tile.tileComponents = T.comp_p.data();
    size_t bi = 0, pi = 0, ki = 0;
    for (uint32_t c = 0; c < nc; ++c) {
        T.comp_p[c] = &T.comps[c];
        T.comps[c].numResolutions = numres;
        T.comps[c].resolutions = &T.res_p[(size_t)c * numres];
        for (uint32_t r = 0; r < numres; ++r) {
            grk_plugin_resolution& R = T.res[(size_t)c * numres + r];
            T.res_p[(size_t)c * numres + r] = &R;
            R.level = r;
            R.numBands = r ? 3 : 1;
            R.band = &T.band_p[bi];
            for (uint32_t b = 0; b < R.numBands; ++b, ++bi) {
                if (bi >= B.size() || B[bi].comp != c || B[bi].res != r || B[bi].band != b) {
                    why = "band list does not match the tile tree";
                    return false;
                }
                grk_plugin_band& G = T.bands[bi];
                T.band_p[bi] = &G;
                G.orientation = (uint8_t)B[bi].orient;
                G.numPrecincts = B[bi].num_precincts;
                G.precincts = &T.prc_p[pi];
                G.stepsize = B[bi].stepsize;
                for (uint32_t p = 0; p < B[bi].num_precincts; ++p, ++pi) {
                    grk_plugin_precinct& P = T.prcs[pi];
                    T.prc_p[pi] = &P;
                    P.blocks = T.block_p.data() + ki;
                    while (ki < K.size() && K[ki].comp == c && K[ki].res == r && K[ki].band == b && K[ki].precinct == p) {
                        const gk_block_result& k = K[ki];
                        grk_plugin_code_block& o = T.blocks[ki];
                        if (k.npasses > 67) { why = "a code-block has more than the 67 passes of grk_plugin_code_block"; return false; }
                        o.x0 = k.x0; o.y0 = k.y0; o.x1 = k.x1; o.y1 = k.y1;
                        o.contextStream = nullptr;
                        o.numPix = (k.x1 - k.x0) * (k.y1 - k.y0);
                        o.compressedData = T.data.data() + k.data_off;
                        o.compressedDataLength = k.len;
                        o.numBitPlanes = (uint8_t)k.numbps;
                        o.numPasses = k.npasses;
                        for (uint32_t q = 0; q < k.npasses; ++q) {
                            const gk_pass_result& s = PS[k.pass_off + q];
                            o.passes[q].distortionDecrease = s.dist;
                            o.passes[q].rate = (size_t)s.rate - 1;   // the host adds 1 back (plugin_bridge.cpp:249)
                            o.passes[q].length = s.len;
                        }
                        o.sortedIndex = (unsigned)ki;
                        ++ki;
                        ++P.numBlocks;
                    }
                }
            }
        }
    }
    if (ki != K.size() || pi != nprc) { why = "block list does not match the tile tree"; return false; }
    return true;
}

// ---------------------------------------------------------------------------- compress
int32_t encode_file(const char* in, const char* out_name, bool relative, grk_cparameters* params,
                    PLUGIN_ENCODE_USER_CALLBACK cb) {
    Raster img;
    std::string why;
    if (!read_pnm(in, img, why)) { note("%s: %s (not handled)", in, why.c_str()); return -1; }
    gk_cparameters p;
    if (!grk_params_to_gk(*params, false, p, why)) { note("%s (not handled)", why.c_str()); return -1; }
    gk_image_info info{};
    info.w = img.w; info.h = img.h; info.numcomps = img.nc; info.prec = img.prec; info.sgnd = 0;
    info.sample_bytes = img.prec > 8 ? 2 : 1;
    const size_t npix = (size_t)img.w * img.h, es = info.sample_bytes;
    std::vector<const void*> planes(img.nc);
    std::vector<uint32_t> strides(img.nc, img.w);
    for (uint32_t c = 0; c < img.nc; ++c) planes[c] = img.planes.data() + c * npix * es;
    Tree T;
    std::vector<gk_band_result> B;
    std::vector<gk_block_result> K;
    std::vector<gk_pass_result> PS;
    {
        std::lock_guard<std::mutex> lk(g_m);
        gk_ctx* e = engine();
        if (!e) { note("no HIP device %d (not handled)", g_device); return -1; }
        uint32_t nb = 0, nk = 0, np = 0;
        uint64_t nbytes = 0;
        if (gk_encode_blocks(e, &info, planes.data(), strides.data(), 0, &p, &nb, &nk, &nbytes, &np) != 0) {
            note("%s (not handled)", gk_last_error(e));
            return -1;
        }
        B.resize(nb); K.resize(nk); PS.resize(np); T.data.resize(nbytes);
        gk_encode_blocks_get(e, B.data(), K.data(), T.data.data(), PS.data());
    }
    if (!build_tree(T, img.nc, p.numresolution, B, K, PS, why)) { note("%s (not handled)", why.c_str()); return -1; }
    if (g_verbose) note("%s: %zu code-blocks, %zu bytes", in, K.size(), T.data.size());
    plugin_encode_user_callback_info cbi{};
    cbi.input_file_name = in;
    cbi.outputFileNameIsRelative = relative;
    cbi.output_file_name = out_name;
    cbi.compressor_parameters = params;
    cbi.image = nullptr;   // the host loads the image (grk_compress.cpp:1779-1800)
    cbi.tile = &T.tile;
    cb(&cbi);
    return cbi.error_code;
}

bool has_ext(const std::string& n, std::initializer_list<const char*> exts) {
    const size_t dot = n.rfind('.');
    if (dot == std::string::npos) return false;
    std::string e = n.substr(dot + 1);
    for (auto& ch : e) ch = (char)tolower(ch);
    for (const char* x : exts) if (e == x) return true;
    return false;
}
std::vector<std::string> dir_files(const char* dir, std::initializer_list<const char*> exts) {
    std::vector<std::string> out;
    DIR* d = opendir(dir);
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        std::string n = e->d_name;
        if (n == "." || n == ".." || !has_ext(n, exts)) continue;
        out.push_back(n);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}
bool g_batch_done = true;

// ---------------------------------------------------------------------------- decompress
struct OwnedImage {
    grk_image img{};
    std::vector<grk_image_comp> comps;
    ~OwnedImage() { for (auto& c : comps) free(c.data); }
};

int g_hdr_rc = 0;
int hdr_seen(grk_header_info* hi, grk_image* im) {   // GROK_INIT_DECOMPRESSORS
    (void)hi;
    g_hdr_rc = im ? 0 : -1;
    return g_hdr_rc;
}

int32_t decode_file(const std::string& in, const std::string& out, grk_decompress_parameters* params,
                    PLUGIN_DECODE_USER_CALLBACK cb) {
    std::vector<uint8_t> cs;
    {
        FILE* f = fopen(in.c_str(), "rb");
        if (!f) { note("cannot open %s (not handled)", in.c_str()); return -1; }
        fseek(f, 0, SEEK_END);
        const long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        cs.resize(n > 0 ? (size_t)n : 0);
        const size_t got = cs.empty() ? 0 : fread(cs.data(), 1, cs.size(), f);
        fclose(f);
        if (got != cs.size()) { note("short read of %s (not handled)", in.c_str()); return -1; }
    }
    gk_image_info info{};
    gk_cparameters coding{};
    char msg[256] = {0};
    if (gk_probe_header(cs.data(), cs.size(), &info, &coding, msg, sizeof msg) != 0) {
        note("%s: %s (not handled)", in.c_str(), msg);
        return -1;
    }
    if (params->core.cp_reduce || params->core.cp_layer || params->nb_tile_to_decompress) {
        note("reduced-resolution, layer-limited or single-tile decompression is not handled by the plugin");
        return -1;
    }
    uint32_t x0 = 0, y0 = 0, x1 = info.w, y1 = info.h;
    const bool window = params->DA_x1 > params->DA_x0 && params->DA_y1 > params->DA_y0;
    if (window) {
        x0 = std::min(params->DA_x0, info.w); y0 = std::min(params->DA_y0, info.h);
        x1 = std::min(params->DA_x1, info.w); y1 = std::min(params->DA_y1, info.h);
        if (x1 <= x0 || y1 <= y0) { note("window outside the image (not handled)"); return -1; }
    }
    // 1. the host reads the header and prepares its output writer
    PluginDecodeCallbackInfo ci;
    ci.deviceId = (size_t)g_device;
    ci.inputFile = in;
    ci.outputFile = out;
    ci.decod_format = params->decod_format;
    ci.cod_format = params->cod_format;
    ci.decompressor_parameters = params;
    ci.decompress_flags = GRK_DECODE_HEADER;
    ci.init_decompressors_func = hdr_seen;
    g_hdr_rc = -1;
    int32_t rc = cb(&ci);
    if (rc != 0 || g_hdr_rc != 0) { note("host header stage failed (%d)", rc); return rc ? rc : -1; }
    // 2. the whole decode on the GPU into an image the plugin owns
    OwnedImage O;
    O.comps.assign(info.numcomps, grk_image_comp{});
    O.img.x0 = x0; O.img.y0 = y0; O.img.x1 = x1; O.img.y1 = y1;
    O.img.numcomps = (uint16_t)info.numcomps;
    O.img.color_space = coding.cod_format == 2 ? (info.numcomps < 3 ? GRK_CLRSPC_GRAY : GRK_CLRSPC_SRGB)
                                               : GRK_CLRSPC_UNKNOWN;
    O.img.comps = O.comps.data();
    std::vector<void*> planes(info.numcomps);
    std::vector<uint32_t> strides(info.numcomps);
    for (uint32_t c = 0; c < info.numcomps; ++c) {
        grk_image_comp& k = O.comps[c];
        k.dx = k.dy = 1; k.w = x1 - x0; k.h = y1 - y0; k.x0 = x0; k.y0 = y0;
        k.stride = (k.w + 31) / 32 * 32;
        k.prec = (uint8_t)info.prec; k.sgnd = info.sgnd != 0;
        k.type = GRK_COMPONENT_TYPE_COLOUR; k.association = GRK_COMPONENT_ASSOC_WHOLE_IMAGE;
        k.data = (int32_t*)aligned_alloc(64, ((size_t)k.stride * k.h * 4 + 63) / 64 * 64);
        if (!k.data) { note("out of host memory"); return -1; }
        planes[c] = k.data; strides[c] = k.stride;
    }
    {
        std::lock_guard<std::mutex> lk(g_m);
        gk_ctx* e = engine();
        if (!e) { note("no HIP device %d", g_device); return -1; }
        rc = window ? gk_decode_window(e, cs.data(), cs.size(), 0, x0, y0, x1, y1, planes.data(), strides.data(), 0, 0)
                    : gk_decode(e, cs.data(), cs.size(), 0, planes.data(), strides.data(), 0, 0);
        if (rc != 0) { note("%s", gk_last_error(e)); return -1; }
    }
    // 3. the host writes the output file from the plugin's image
    ci.init_decompressors_func = nullptr;
    ci.image = &O.img;
    ci.plugin_owns_image = true;
    ci.decompress_flags = GRK_DECODE_POST_T1;
    rc = cb(&ci);
    // 4. the host releases its codec and stream
    ci.decompress_flags = GRK_PLUGIN_DECODE_CLEAN;
    cb(&ci);
    if (g_verbose) note("%s -> %s: %ux%u x %u", in.c_str(), out.c_str(), x1 - x0, y1 - y0, info.numcomps);
    return rc;
}

const char* out_ext(GRK_SUPPORTED_FILE_FMT f, uint32_t nc) {
    switch (f) {
        case GRK_PXM_FMT: return nc >= 3 ? "ppm" : "pgm";
        case GRK_PGX_FMT: return "pgx";
        case GRK_PAM_FMT: return "pam";
        case GRK_BMP_FMT: return "bmp";
        case GRK_TIF_FMT: return "tif";
        case GRK_RAW_FMT: return "raw";
        case GRK_RAWL_FMT: return "rawl";
        case GRK_PNG_FMT: return "png";
        case GRK_JPG_FMT: return "jpg";
        default: return "raw";
    }
}
struct BatchDecode {
    std::string in_dir, out_dir;
    grk_decompress_parameters* params = nullptr;
    PLUGIN_DECODE_USER_CALLBACK cb = nullptr;
    bool stop = false;
} g_bd;

void* obj_create(minpf_object_params*) { return nullptr; }
int32_t obj_destroy(void*) { return 0; }
int32_t on_exit() {
    std::lock_guard<std::mutex> lk(g_m);
    if (g_eng) { gk_destroy(g_eng); g_eng = nullptr; }
    return 0;
}

}  // namespace

extern "C" {

// minpf_load (minpf_plugin_manager.cpp:140-175): register, return the exit function
minpf_exit_func minpf_post_load_plugin(const char* pluginPath, const minpf_platform_services* services) {
    (void)pluginPath;
    if (!services || !services->registerObject) return nullptr;
    minpf_register_params rp{};
    rp.version.major = 1;
    rp.version.minor = 0;
    rp.createFunc = obj_create;
    rp.destroyFunc = obj_destroy;
    if (services->registerObject("grokj2k_plugin", &rp) != 0) return nullptr;
    return on_exit;
}

// grok.cpp:626-639
bool plugin_init(grk_plugin_init_info initInfo) {
    std::lock_guard<std::mutex> lk(g_m);
    const int dev = initInfo.deviceId < 0 ? 0 : initInfo.deviceId;
    if (g_eng && dev != g_device) { gk_destroy(g_eng); g_eng = nullptr; }
    g_device = dev;
    g_verbose = initInfo.verbose;
    return engine() != nullptr;
}

// called on the host's hot paths (TileProcessor.cpp:99,204,1066,1203): production state
uint32_t plugin_get_debug_state(void) { return GRK_PLUGIN_STATE_NO_DEBUG; }

int32_t plugin_encode(grk_cparameters* encoding_parameters, PLUGIN_ENCODE_USER_CALLBACK callback) {
    if (!encoding_parameters || !callback) return -1;
    return encode_file(encoding_parameters->infile, encoding_parameters->outfile, false, encoding_parameters, callback);
}

// Every PNM of input_dir, in name order, synchronously; output names are relative (the CLI
// places them in its output folder with its output format, grk_compress.cpp:1755-1768).
int32_t plugin_batch_encode(const char* input_dir, const char* output_dir, grk_cparameters* encoding_parameters,
                            PLUGIN_ENCODE_USER_CALLBACK userCallback) {
    (void)output_dir;
    if (!input_dir || !encoding_parameters || !userCallback) return -1;
    g_batch_done = false;
    int32_t rc = 0;
    for (const std::string& n : dir_files(input_dir, {"pgm", "ppm", "pnm"})) {
        const std::string path = std::string(input_dir) + "/" + n;
        if (encode_file(path.c_str(), n.c_str(), true, encoding_parameters, userCallback) != 0) rc = -1;
    }
    g_batch_done = true;
    return rc;
}
bool plugin_is_batch_complete(void) { return g_batch_done; }
void plugin_stop_batch_encode(void) { g_batch_done = true; }

int32_t plugin_decompress(grk_decompress_parameters* decoding_parameters, PLUGIN_DECODE_USER_CALLBACK userCallback) {
    if (!decoding_parameters || !userCallback) return -1;
    return decode_file(decoding_parameters->infile, decoding_parameters->outfile, decoding_parameters, userCallback);
}

int32_t plugin_init_batch_decompress(const char* input_dir, const char* output_dir,
                                     grk_decompress_parameters* decoding_parameters,
                                     PLUGIN_DECODE_USER_CALLBACK userCallback) {
    if (!input_dir || !output_dir || !decoding_parameters || !userCallback) return -1;
    g_bd.in_dir = input_dir; g_bd.out_dir = output_dir;
    g_bd.params = decoding_parameters; g_bd.cb = userCallback; g_bd.stop = false;
    g_batch_done = false;
    return 0;
}
// Every .j2k / .j2c / .jp2 / .jph / .jhc of the input folder, in name order, synchronously.
int32_t plugin_batch_decompress(void) {
    if (!g_bd.cb) return -1;
    int32_t rc = 0;
    for (const std::string& n : dir_files(g_bd.in_dir.c_str(), {"j2k", "j2c", "jp2", "jph", "jhc"})) {
        if (g_bd.stop) break;
        std::vector<uint8_t> hdr;
        const std::string path = g_bd.in_dir + "/" + n;
        const size_t dot = n.rfind('.');
        gk_image_info info{};
        {
            FILE* f = fopen(path.c_str(), "rb");
            if (!f) { rc = -1; continue; }
            hdr.resize(1 << 16);
            hdr.resize(fread(hdr.data(), 1, hdr.size(), f));
            fclose(f);
        }
        char msg[128];
        const uint32_t nc = gk_probe_header(hdr.data(), hdr.size(), &info, nullptr, msg, sizeof msg) == 0 ? info.numcomps : 1;
        const std::string out = g_bd.out_dir + "/" + n.substr(0, dot) + "." + out_ext(g_bd.params->cod_format, nc);
        if (decode_file(path, out, g_bd.params, g_bd.cb) != 0) rc = -1;
    }
    g_batch_done = true;
    return rc;
}
void plugin_stop_batch_decompress(void) { g_bd.stop = true; g_batch_done = true; }

// optional debug hooks the host resolves by name (plugin_bridge.cpp:299-330); no debug state
void plugin_debug_mqc_next_cxd(void* mqc, uint32_t d) { (void)mqc; (void)d; }
void plugin_debug_mqc_next_plane(void* mqc) { (void)mqc; }

}  // extern "C"
