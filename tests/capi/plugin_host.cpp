// A stand-in for an unmodified Grok 9.2.0 host driving a T1 plugin (Grok itself is not built
// here: its build needs cmake-generated headers).  It does what the host does, in the same
// order, with nothing but the plugin ABI:
//   * load: dlopen <dir>/libgrokj2k_plugin.so, minpf_post_load_plugin with platform services
//     whose registerObject applies minpf_register_object's checks (minpf_plugin_manager.cpp:
//     46-71), plugin_get_debug_state, plugin_init (grok.cpp:579-639);
//   * compress: plugin_encode with grk_compress's parameters; in the callback, walk the tile
//     tree and take every block as compress_synch_with_plugin does (plugin_bridge.cpp:146-270:
//     rate + 1, clamped to the length, minus one before a 0xFF byte), dumping the result;
//   * decompress: plugin_decompress with a callback playing grk_decompress's
//     decompress_callback (grk_decompress.cpp:996-1031): the header stage calls
//     init_decompressors_func, the post-T1 stage writes the plugin's image.
//
//   plugin_host DIR enc IN.pnm DUMP [-n N] [-b W,H] [-c [W,H],..] [-I] [-r R1,R2,..] [-M 64] [-t W,H] [-mct 0|1]
//   plugin_host DIR dec IN.j2k OUT.raw [-d X0,Y0,X1,Y1]
//
// DUMP: per block 15 u32 (comp res band prc cblk x0 y0 x1 y1 numbps npasses len numPix orient
// numPrecincts), npasses u32 host pass rates, npasses f64 distortion, then len bytes.
// OUT.raw: planar int32 samples; stdout lists the callback stages seen.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "grk_plugin_abi.h"

namespace {

typedef minpf_exit_func (*post_load_fn)(const char*, const minpf_platform_services*);
typedef bool (*init_fn)(grk_plugin_init_info);
typedef uint32_t (*state_fn)(void);
typedef int32_t (*encode_fn)(grk_cparameters*, PLUGIN_ENCODE_USER_CALLBACK);
typedef int32_t (*decode_fn)(grk_decompress_parameters*, PLUGIN_DECODE_USER_CALLBACK);

int g_registered = 0;
int32_t register_object(const char* id, const minpf_register_params* p) {
    if (!id || !id[0] || !p || !p->createFunc || !p->destroyFunc) return -1;
    if (p->version.major != 1) return -1;
    ++g_registered;
    return 0;
}

FILE* g_dump = nullptr;
int g_blocks = 0, g_bad = 0;
unsigned g_numres = 6;

void encode_cb(plugin_encode_user_callback_info* info) {
    grk_plugin_tile* t = info->tile;
    if (!t || !t->tileComponents) { g_bad = 1; return; }
    for (size_t c = 0; c < t->numComponents; ++c) {
        grk_plugin_tile_component* tc = t->tileComponents[c];
        if (tc->numResolutions != g_numres) g_bad = 2;
        for (size_t r = 0; r < tc->numResolutions; ++r) {
            grk_plugin_resolution* R = tc->resolutions[r];
            if (R->numBands != (r ? 3u : 1u)) g_bad = 3;
            for (size_t b = 0; b < R->numBands; ++b) {
                grk_plugin_band* B = R->band[b];
                if (B->orientation != (r ? b + 1 : 0)) g_bad = 4;
                for (uint64_t p = 0; p < B->numPrecincts; ++p) {
                    grk_plugin_precinct* P = B->precincts[p];
                    for (uint64_t k = 0; k < P->numBlocks; ++k) {
                        grk_plugin_code_block* K = P->blocks[k];
                        uint32_t hdr[15] = {(uint32_t)c, (uint32_t)r, (uint32_t)b, (uint32_t)p, (uint32_t)k,
                                            K->x0, K->y0, K->x1, K->y1, K->numBitPlanes, (uint32_t)K->numPasses,
                                            K->compressedDataLength, K->numPix, B->orientation,
                                            (uint32_t)B->numPrecincts};
                        fwrite(hdr, 4, 15, g_dump);
                        // plugin_bridge.cpp:244-266
                        const uint16_t total = (uint16_t)K->compressedDataLength;
                        std::vector<uint32_t> rates(K->numPasses);
                        std::vector<double> dist(K->numPasses);
                        for (size_t q = 0; q < K->numPasses; ++q) {
                            uint16_t rate = (uint16_t)(K->passes[q].rate + 1);
                            if (rate > total) rate = total;
                            if (rate > 1 && K->compressedData[rate - 1] == 0xFF) rate--;
                            rates[q] = rate;
                            dist[q] = K->passes[q].distortionDecrease;
                        }
                        fwrite(rates.data(), 4, rates.size(), g_dump);
                        fwrite(dist.data(), 8, dist.size(), g_dump);
                        fwrite(K->compressedData, 1, K->compressedDataLength, g_dump);
                        ++g_blocks;
                    }
                }
            }
        }
    }
}

std::vector<std::string> g_stages;
std::string g_out;
int32_t decode_cb(PluginDecodeCallbackInfo* info) {
    int32_t rc = -1;
    if (info->decompress_flags & GRK_PLUGIN_DECODE_CLEAN) { g_stages.push_back("clean"); rc = 0; }
    if (info->decompress_flags & (GRK_DECODE_HEADER | GRK_DECODE_T1 | GRK_DECODE_T2)) {
        // preProcess: open the codec, read the header (the host's composited image carries the
        // geometry), hand it to the plugin's init function and return its result
        g_stages.push_back("header");
        static grk_image host_image;
        memset(&host_image, 0, sizeof host_image);
        if (info->init_decompressors_func) return info->init_decompressors_func(&info->header_info, &host_image);
        rc = 0;
    }
    if (info->decompress_flags & GRK_DECODE_POST_T1) {   // postProcess: write the image
        g_stages.push_back(info->plugin_owns_image ? "post(plugin image)" : "post");
        grk_image* im = info->image;
        if (!im) return -1;
        FILE* f = fopen(info->outputFile.c_str(), "wb");
        if (!f) return -1;
        for (uint32_t k = 0; k < im->numcomps; ++k)
            for (uint32_t y = 0; y < im->comps[k].h; ++y)
                fwrite(im->comps[k].data + (size_t)y * im->comps[k].stride, 4, im->comps[k].w, f);
        fclose(f);
        printf("image %u %u %u %u comps %u prec %u\n", im->x0, im->y0, im->x1, im->y1, im->numcomps,
               im->comps[0].prec);
        rc = 0;
    }
    return rc;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: plugin_host DIR enc IN.pnm DUMP [opts] | plugin_host DIR dec IN OUT.raw [-d ..]\n");
        return 1;
    }
    // grk_plugin_load (grok.cpp:579-605): <pluginPath>/lib + grokj2k_plugin + .so
    const std::string lib = std::string(argv[1]) + "/libgrokj2k_plugin.so";
    void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
    auto post = (post_load_fn)dlsym(h, "minpf_post_load_plugin");
    if (!post) return 3;
    minpf_platform_services ps{};
    ps.version.major = 1;
    ps.registerObject = register_object;
    minpf_exit_func on_exit = post(lib.c_str(), &ps);
    if (!on_exit || g_registered != 1) { fprintf(stderr, "plugin registration failed\n"); return 4; }
    auto dbg = (state_fn)dlsym(h, "plugin_get_debug_state");
    if (!dbg || dbg() != GRK_PLUGIN_STATE_NO_DEBUG) return 5;
    auto init = (init_fn)dlsym(h, "plugin_init");
    grk_plugin_init_info ii{};
    ii.deviceId = 0;
    if (!init || !init(ii)) { fprintf(stderr, "plugin_init failed\n"); return 6; }
    int rc = 0;
    if (!strcmp(argv[2], "enc")) {
        grk_cparameters p;   // grk_compress_set_default_params (grok.cpp:405-435)
        memset(&p, 0, sizeof p);
        p.numresolution = 6; p.cblockw_init = 64; p.cblockh_init = 64; p.numgbits = 2;
        p.prog_order = GRK_LRCP; p.roi_compno = -1; p.subsampling_dx = 1; p.subsampling_dy = 1; p.repeats = 1;
        int mct = -1;
        for (int i = 5; i < argc; ++i) {
            if (!strcmp(argv[i], "-n")) p.numresolution = (uint8_t)atoi(argv[++i]);
            else if (!strcmp(argv[i], "-b")) sscanf(argv[++i], "%u,%u", &p.cblockw_init, &p.cblockh_init);
            else if (!strcmp(argv[i], "-I")) p.irreversible = true;
            else if (!strcmp(argv[i], "-r")) {
                char* s = argv[++i];
                p.numlayers = 0;
                for (char* t = strtok(s, ","); t; t = strtok(nullptr, ",")) p.layer_rate[p.numlayers++] = atof(t);
                p.allocationByRateDistoration = true;
            } else if (!strcmp(argv[i], "-M")) {
                p.cblk_sty = (uint8_t)atoi(argv[++i]);
                p.isHT = (p.cblk_sty & GRK_CBLKSTY_HT) != 0;
                if (p.isHT) p.numgbits = 1;
            } else if (!strcmp(argv[i], "-c")) {   // precincts [W,H],[W,H],.. (grk_compress.cpp parse)
                const char* s = argv[++i];
                uint32_t n = 0;
                char sep;
                do {
                    sep = 0;
                    if (sscanf(s, "[%u,%u]%c", &p.prcw_init[n], &p.prch_init[n], &sep) < 2) break;
                    ++n;
                    s = strchr(s, ']');
                    if (!s) break;
                    s += 2;
                } while (sep == ',' && n < GRK_J2K_MAXRLVLS);
                p.res_spec = n;
                p.csty |= 1;
            } else if (!strcmp(argv[i], "-t")) {
                p.tile_size_on = true;
                sscanf(argv[++i], "%u,%u", &p.t_width, &p.t_height);
            } else if (!strcmp(argv[i], "-mct")) mct = atoi(argv[++i]);
        }
        p.mct = (uint8_t)(mct < 0 ? 255 : mct);   // 255: not set on the command line (grk_compress.cpp:1977)
        g_numres = p.numresolution;
        snprintf(p.infile, sizeof p.infile, "%s", argv[3]);
        snprintf(p.outfile, sizeof p.outfile, "%s.j2k", argv[4]);
        g_dump = fopen(argv[4], "wb");
        auto enc = (encode_fn)dlsym(h, "plugin_encode");
        rc = enc ? enc(&p, encode_cb) : -1;
        fclose(g_dump);
        printf("plugin_encode rc %d blocks %d tree %s\n", rc, g_blocks, g_bad ? "bad" : "ok");
        if (g_bad) rc = 10 + g_bad;
    } else if (!strcmp(argv[2], "dec")) {
        grk_decompress_parameters d;
        memset(&d, 0, sizeof d);
        snprintf(d.infile, sizeof d.infile, "%s", argv[3]);
        snprintf(d.outfile, sizeof d.outfile, "%s", argv[4]);
        d.cod_format = GRK_RAW_FMT;
        for (int i = 5; i < argc; ++i)
            if (!strcmp(argv[i], "-d")) sscanf(argv[++i], "%u,%u,%u,%u", &d.DA_x0, &d.DA_y0, &d.DA_x1, &d.DA_y1);
        auto dec = (decode_fn)dlsym(h, "plugin_decompress");
        rc = dec ? dec(&d, decode_cb) : -1;
        printf("plugin_decompress rc %d stages", rc);
        for (auto& s : g_stages) printf(" %s", s.c_str());
        printf("\n");
    } else {
        rc = 1;
    }
    on_exit();
    dlclose(h);
    return rc;
}
