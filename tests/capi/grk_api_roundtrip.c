/* A minimal grk_compress / grk_decompress written against Grok's public C API (the call
 * sequence of src/bin/jp2/grk_compress.cpp and grk_decompress.cpp: initialize, set handlers,
 * image, stream, codec create / init / start / compress / end, decompress create / init /
 * read_header / [set_window] / decompress / get_composited_image / end, unref).  Built against
 * include/grk_abi.h (layout-identical to grok.h) and linked with libgrok_amd.so by
 * tests/test_gpu_grk_api.py.  Raw files are planar int32 samples, component after component.
 *
 *   enc RAW W H C PREC OUT [-n N] [-b W,H] [-I] [-r R1,R2,..] [-q Q1,Q2,..] [-S] [-E] [-M 64] [-t W,H] [-X] [-L]
 *       [-p PROG] [-P T0=..,PROG/T0=..] [-jp2] [-tiles] [-file]
 *   dec IN RAWOUT [-d X0,Y0,X1,Y1] [-tile T] [-r REDUCE] [-l LAYERS] [-mapped]
 *   dump IN [FLAGS]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "grk_abi.h"

static void on_error(const char* msg, void* ud) { (void)ud; fprintf(stderr, "[grk error] %s\n", msg); }
static void on_warning(const char* msg, void* ud) { (void)ud; fprintf(stderr, "[grk warning] %s\n", msg); }

static GRK_PROG_ORDER prog_of(const char* s) {   /* grk_compress.cpp:331-347 */
    static const char* names[] = {"LRCP", "RLCP", "RPCL", "PCRL", "CPRL"};
    for (int k = 0; k < 5; ++k)
        if (!strncmp(s, names[k], 4)) return (GRK_PROG_ORDER)k;
    return GRK_PROG_UNKNOWN;
}

static int enc(int argc, char** argv) {
    const char* raw = argv[2];
    uint32_t w = (uint32_t)atoi(argv[3]), h = (uint32_t)atoi(argv[4]), c = (uint32_t)atoi(argv[5]);
    uint32_t prec = (uint32_t)atoi(argv[6]);
    const char* out = argv[7];
    grk_cparameters p;
    grk_compress_set_default_params(&p);
    p.mct = 255;                    /* pluginMain (grk_compress.cpp:2180-2184): resolved per image below */
    p.rateControlAlgorithm = 255;
    p.numlayers = 1;                /* :823-828: no -r / -q is one lossless layer (set before -P is read) */
    int to_file = 0;
    GRK_CODEC_FORMAT fmt = GRK_CODEC_J2K;
    int raw_tiles = 0, tile_off = 0, img_off = 0;
    uint32_t sdx[4] = {1, 1, 1, 1}, sdy[4] = {1, 1, 1, 1};
    for (int i = 8; i < argc; ++i) {
        if (!strcmp(argv[i], "-n")) p.numresolution = (uint8_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-b")) sscanf(argv[++i], "%u,%u", &p.cblockw_init, &p.cblockh_init);
        else if (!strcmp(argv[i], "-I")) p.irreversible = true;
        else if (!strcmp(argv[i], "-r")) {
            char* s = argv[++i];
            p.numlayers = 0;
            for (char* t = strtok(s, ","); t; t = strtok(NULL, ",")) p.layer_rate[p.numlayers++] = atof(t);
            p.allocationByRateDistoration = true;
        } else if (!strcmp(argv[i], "-M")) { p.cblk_sty = (uint8_t)atoi(argv[++i]); p.isHT = (p.cblk_sty & GRK_CBLKSTY_HT) != 0; if (p.isHT) p.numgbits = 1; }
        else if (!strcmp(argv[i], "-t")) { p.tile_size_on = true; sscanf(argv[++i], "%u,%u", &p.t_width, &p.t_height); }
        else if (!strcmp(argv[i], "-X")) p.writeTLM = true;
        else if (!strcmp(argv[i], "-L")) p.writePLT = true;
        else if (!strcmp(argv[i], "-jp2")) fmt = GRK_CODEC_JP2;
        else if (!strcmp(argv[i], "-tiles")) raw_tiles = 1;
        else if (!strcmp(argv[i], "-file")) to_file = 1;
        else if (!strcmp(argv[i], "-p")) p.prog_order = prog_of(argv[++i]);
        else if (!strcmp(argv[i], "-P")) {   /* grk_compress.cpp:1001-1057: T<t>=resS,compS,layE,resE,compE,PROG/... */
            char* s = argv[++i];
            uint32_t n = 0, rs, cs, le, re, ce;
            char prog[5];
            while (sscanf(s, "T%u=%u,%u,%u,%u,%u,%4s", &p.progression[n].tileno, &rs, &cs, &le, &re, &ce, prog) == 7) {
                p.progression[n].resS = (uint8_t)rs; p.progression[n].compS = (uint16_t)cs;
                p.progression[n].layE = (uint16_t)le; p.progression[n].resE = (uint8_t)re;
                p.progression[n].compE = (uint16_t)ce;
                p.progression[n].specifiedCompressionPocProg = prog_of(prog);
                if (p.progression[n].layE > p.numlayers) p.progression[n].layE = p.numlayers;
                if (p.progression[n].resE > p.numresolution) p.progression[n].resE = (uint8_t)(p.numresolution - 1);
                ++n;
                while (*s && *s != '/') s++;
                if (!*s) break;
                s++;
            }
            if (n <= 1) return 21;
            p.numpocs = n - 1;
        }
        else if (!strcmp(argv[i], "-S")) p.csty |= 0x02;   /* grk_compress.cpp:529-531: SOP / EPH */
        else if (!strcmp(argv[i], "-E")) p.csty |= 0x04;
        else if (!strcmp(argv[i], "-q")) {   /* :788-800: PSNR per layer, fixed-quality allocation */
            char* s = argv[++i];
            p.numlayers = 0;
            for (char* t = strtok(s, ","); t; t = strtok(NULL, ",")) p.layer_distortion[p.numlayers++] = atof(t);
            p.allocationByQuality = true;
        }
        else if (!strcmp(argv[i], "-T")) { sscanf(argv[++i], "%u,%u", &p.tx0, &p.ty0); tile_off = 1; }   /* :1512-1529 */
        else if (!strcmp(argv[i], "-C")) {   /* grk_compress.cpp:1578-1608: '|'-separated ISO Latin comments */
            char* str = argv[++i];
            char* tok = strtok(str, "|");
            while (tok && p.num_comments < GRK_NUM_COMMENTS_SUPPORTED) {
                if (*tok) {
                    size_t n = strlen(tok);
                    p.is_binary_comment[p.num_comments] = false;
                    p.comment[p.num_comments] = (char*)malloc(n);
                    memcpy(p.comment[p.num_comments], tok, n);
                    p.comment_len[p.num_comments] = (uint16_t)n;
                    p.num_comments++;
                }
                tok = strtok(NULL, "|");
            }
        }
        else if (!strcmp(argv[i], "-sub")) {   /* API-level subsampling (grk_image_comp dx / dy): dx1xdy1:dx2xdy2:...
                                                  (the CLI's raw reader refuses it, RAWFormat.cpp:293-298) */
            char* s = argv[++i];
            for (uint32_t k = 0; k < 4 && *s; ++k) {
                sscanf(s, "%ux%u", &sdx[k], &sdy[k]);
                char* q = strchr(s, ':');
                if (!q) break;
                s = q + 1;
            }
        }
        else if (!strcmp(argv[i], "-d")) {   /* :1530-1545 image offset */
            sscanf(argv[++i], "%u,%u", &p.image_offset_x0, &p.image_offset_y0);
            img_off = 1;
        }
        else if (!strcmp(argv[i], "-c")) {   /* one precinct size for every resolution: [W,H] */
            unsigned pw, ph;
            sscanf(argv[++i], "[%u,%u]", &pw, &ph);
            p.csty |= 1; p.res_spec = 1; p.prcw_init[0] = pw; p.prch_init[0] = ph;
        }
    }
    if (!img_off && tile_off) {   /* :1547-1551: -T alone puts the image at the tile origin */
        p.image_offset_x0 = p.tx0; p.image_offset_y0 = p.ty0;
    } else if (p.tx0 > p.image_offset_x0 || p.ty0 > p.image_offset_y0) {
        return 22;   /* :1554-1562 "Tile offset must be top left of image offset" */
    }
    if (p.mct == 255) p.mct = c >= 3 ? 1 : 0;   /* grk_compress.cpp:1978-1995: RGB input switches the MCT on */
    if (p.rateControlAlgorithm == 255) p.rateControlAlgorithm = 0;
    grk_initialize(NULL, p.numThreads);
    {   /* pluginMain: grk_plugin_init fails without a plugin and the CLI falls back (:2209, :2281-2289) */
        grk_plugin_init_info initInfo;
        initInfo.deviceId = p.deviceId;
        initInfo.verbose = false;
        if (grk_plugin_init(initInfo)) return 20;
    }
    grk_image_cmptparm cp[4];
    memset(cp, 0, sizeof cp);
    /* the image readers place the image at the -d offset (RAWFormat.cpp:309-312, PNMFormat.cpp:474-477);
       a subsampled component holds the image area sampled every (dx, dy): ceil(x1 / dx) - ceil(x0 / dx)
       columns (GrkImage.cpp:74-113) */
    const uint32_t X0 = p.image_offset_x0, Y0 = p.image_offset_y0;
    for (uint32_t k = 0; k < c; ++k) {
        cp[k].dx = sdx[k]; cp[k].dy = sdy[k]; cp[k].prec = (uint8_t)prec;
        cp[k].w = (X0 + w + sdx[k] - 1) / sdx[k] - (X0 + sdx[k] - 1) / sdx[k];
        cp[k].h = (Y0 + h + sdy[k] - 1) / sdy[k] - (Y0 + sdy[k] - 1) / sdy[k];
        cp[k].x0 = X0; cp[k].y0 = Y0;
    }
    grk_image* img = grk_image_new((uint16_t)c, cp, c >= 3 ? GRK_CLRSPC_SRGB : GRK_CLRSPC_GRAY, true);
    if (!img) return 2;
    img->x0 = X0; img->y0 = Y0; img->x1 = X0 + w; img->y1 = Y0 + h;
    FILE* f = fopen(raw, "rb");
    int32_t* row = malloc(sizeof(int32_t) * w);
    for (uint32_t k = 0; k < c; ++k)
        for (uint32_t y = 0; y < cp[k].h; ++y) {
            if (fread(row, 4, cp[k].w, f) != cp[k].w) return 3;
            memcpy(img->comps[k].data + (size_t)y * img->comps[k].stride, row, 4 * cp[k].w);
        }
    fclose(f);
    /* compress() :2055-2066: a memory stream the size of 1.5x the raw image, or the output file */
    size_t cap = (size_t)w * h * c * ((prec + 7) / 8) * 3 / 2 + (1 << 16);
    uint8_t* buf = to_file ? NULL : malloc(cap);
    grk_stream* st = to_file ? grk_stream_create_file_stream(out, 1024 * 1024, false)
                             : grk_stream_create_mem_stream(buf, cap, false, false);
    if (!st) return 4;
    grk_codec* codec = grk_compress_create(fmt, st);
    if (!codec) return 4;
    grk_set_warning_handler(on_warning, NULL);
    grk_set_error_handler(on_error, NULL);
    if (!grk_compress_init(codec, &p, img) || !grk_compress_start(codec)) return 4;
    int ok;
    if (raw_tiles) {   /* grk_compress_tile: planar 8/16-bit samples tile by tile */
        uint32_t tw = p.tile_size_on ? p.t_width : w, th = p.tile_size_on ? p.t_height : h;
        uint32_t ntx = (w + tw - 1) / tw, nty = (h + th - 1) / th, es = (prec + 7) / 8;
        ok = 1;
        for (uint32_t t = 0; t < ntx * nty && ok; ++t) {
            uint32_t x0 = (t % ntx) * tw, y0 = (t / ntx) * th;
            uint32_t tw2 = x0 + tw > w ? w - x0 : tw, th2 = y0 + th > h ? h - y0 : th;
            uint8_t* tb = malloc((size_t)tw2 * th2 * c * es);
            size_t o = 0;
            for (uint32_t k = 0; k < c; ++k)
                for (uint32_t y = 0; y < th2; ++y)
                    for (uint32_t x = 0; x < tw2; ++x) {
                        int32_t v = img->comps[k].data[(size_t)(y0 + y) * img->comps[k].stride + x0 + x];
                        if (es == 1) tb[o++] = (uint8_t)v; else { uint16_t s = (uint16_t)v; memcpy(tb + o, &s, 2); o += 2; }
                    }
            ok = grk_compress_tile(codec, (uint16_t)t, tb, o);
            free(tb);
        }
    } else {
        ok = grk_compress_with_plugin(codec, NULL);   /* :2112, info->tile is NULL without a plugin */
    }
    if (!ok || !grk_compress_end(codec)) return 5;
    if (!to_file) {
        size_t n = grk_stream_get_write_mem_stream_length(st);
        f = fopen(out, "wb");
        fwrite(buf, 1, n, f);
        fclose(f);
    }
    grk_object_unref(codec);
    grk_object_unref(st);
    grk_object_unref(&img->obj);
    free(buf);
    free(row);
    grk_deinitialize();
    return 0;
}

/* grk_decompress's call sequence (GrkDecompress::pluginMain grk_decompress.cpp:897-921, then the
 * CPU fallback main :1590-1613 -> decompress -> preProcess :1041-1295 -> postProcess):
 *   grk_initialize; grk_plugin_init (false: no plugin, fall back); grk_decompress_set_default_params;
 *   -d sets dparameters.DA_*; stream; create; handlers; init; read_header; the composited image is
 *   taken right after the header (:1191) and written out at the end; set_window is called
 *   UNCONDITIONALLY with the DA values, zeros when -d is absent (:1259); then grk_decompress +
 *   grk_decompress_end, or grk_decompress_tile for -t. */
static int dec(int argc, char** argv) {
    const char* in = argv[2];
    const char* out = argv[3];
    grk_decompress_parameters params;
    memset(&params, 0, sizeof params);
    grk_decompress_set_default_params(&params.core);
    int mapped = 0;
    for (int i = 4; i < argc; ++i) {
        if (!strcmp(argv[i], "-d"))
            sscanf(argv[++i], "%u,%u,%u,%u", &params.core.DA_x0, &params.core.DA_y0, &params.core.DA_x1, &params.core.DA_y1);
        else if (!strcmp(argv[i], "-tile")) { params.tileIndex = (uint16_t)atoi(argv[++i]); params.nb_tile_to_decompress = 1; }
        else if (!strcmp(argv[i], "-r")) params.core.cp_reduce = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-l")) params.core.cp_layer = (uint16_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-mapped")) mapped = 1;
    }
    grk_initialize(NULL, 0);
    grk_plugin_init_info initInfo;
    initInfo.deviceId = 0;
    initInfo.verbose = false;
    if (grk_plugin_init(initInfo)) return 20;   /* no plugin: the CLI takes its CPU-API path */
    const size_t L = strlen(in);
    GRK_CODEC_FORMAT fmt = L > 4 && !strcmp(in + L - 4, ".jp2") ? GRK_CODEC_JP2 : GRK_CODEC_J2K;
    grk_stream* st = mapped ? grk_stream_create_mapped_file_stream(in, true) : grk_stream_create_file_stream(in, 1024 * 1024, true);
    if (!st) return 6;
    grk_codec* codec = grk_decompress_create(fmt, st);
    if (!codec) return 6;
    grk_set_warning_handler(on_warning, NULL);
    grk_set_error_handler(on_error, NULL);
    if (!grk_decompress_init(codec, &params.core)) return 6;
    grk_header_info hi;
    memset(&hi, 0, sizeof hi);
    if (!grk_decompress_read_header(codec, &hi)) return 6;
    grk_image* img = grk_decompress_get_composited_image(codec);
    if (!img) return 10;
    fprintf(stdout, "header cblk %ux%u numres %u layers %u irrev %d tiles %ux%u\n", hi.cblockw_init, hi.cblockh_init,
            hi.numresolutions, hi.numlayers, (int)hi.irreversible, hi.t_grid_width, hi.t_grid_height);
    for (uint32_t i = 0; i < img->numcomps; ++i)
        if (img->comps[i].prec > 16) return 11;
    if (!grk_decompress_set_window(codec, params.core.DA_x0, params.core.DA_y0, params.core.DA_x1, params.core.DA_y1))
        return 8;
    if (!params.nb_tile_to_decompress) {
        if (!(grk_decompress(codec, NULL) && grk_decompress_end(codec))) return 9;
    } else {
        if (!grk_decompress_tile(codec, params.tileIndex)) return 7;
        if (grk_decompress_get_tile_image(codec, params.tileIndex) != img) return 12;
    }
    grk_object_unref(st);
    fprintf(stdout, "image %u %u %u %u comps %u\n", img->x0, img->y0, img->x1, img->y1, img->numcomps);
    FILE* f = fopen(out, "wb");
    for (uint32_t k = 0; k < img->numcomps; ++k)
        for (uint32_t y = 0; y < img->comps[k].h; ++y)
            fwrite(img->comps[k].data + (size_t)y * img->comps[k].stride, 4, img->comps[k].w, f);
    fclose(f);
    grk_object_unref(codec);
    grk_deinitialize();
    return 0;
}

/* grk_dump's call sequence (grk_dump.cpp:342-504): initialize, handlers, default params, file
 * stream, create, init, read_header(codec, NULL), grk_dump_codec, unref.  Needs no GPU. */
static int dump(int argc, char** argv) {
    const char* in = argv[2];
    uint32_t flag = argc >= 4 ? (uint32_t)strtoul(argv[3], NULL, 0) : (GRK_IMG_INFO | GRK_J2K_MH_INFO);
    grk_initialize(NULL, 0);
    grk_set_warning_handler(on_warning, NULL);
    grk_set_error_handler(on_error, NULL);
    grk_dparameters parameters;
    grk_decompress_set_default_params(&parameters);
    grk_stream* st = grk_stream_create_file_stream(in, 1024 * 1024, 1);
    if (!st) return 30;
    const size_t L = strlen(in);
    grk_codec* codec = grk_decompress_create(L > 4 && !strcmp(in + L - 4, ".jp2") ? GRK_CODEC_JP2 : GRK_CODEC_J2K, st);
    if (!codec) { grk_object_unref(st); return 31; }
    if (!grk_decompress_init(codec, &parameters)) return 32;
    if (!grk_decompress_read_header(codec, NULL)) return 33;
    grk_dump_codec(codec, flag, stdout);
    grk_object_unref(st);
    grk_object_unref(codec);
    grk_deinitialize();
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 3 && !strcmp(argv[1], "dump")) return dump(argc, argv);
    if (argc >= 8 && !strcmp(argv[1], "enc")) return enc(argc, argv);
    if (argc >= 4 && !strcmp(argv[1], "dec")) return dec(argc, argv);
    fprintf(stderr, "usage: enc RAW W H C PREC OUT [opts] | dec IN RAWOUT [-d x0,y0,x1,y1] [-tile t]\n");
    return 1;
}
