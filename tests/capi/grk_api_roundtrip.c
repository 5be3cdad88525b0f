/* A minimal grk_compress / grk_decompress written against Grok's public C API (the call
 * sequence of src/bin/jp2/grk_compress.cpp and grk_decompress.cpp: initialize, set handlers,
 * image, stream, codec create / init / start / compress / end, decompress create / init /
 * read_header / [set_window] / decompress / get_composited_image / end, unref).  Built against
 * include/grk_abi.h (layout-identical to grok.h) and linked with libgrok_amd.so by
 * tests/test_gpu_grk_api.py.  Raw files are planar int32 samples, component after component.
 *
 *   enc RAW W H C PREC OUT [-n N] [-b W,H] [-I] [-r R1,R2,..] [-M 64] [-t W,H] [-X] [-L] [-jp2] [-tiles]
 *   dec IN RAWOUT [-d X0,Y0,X1,Y1] [-tile T]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "grk_abi.h"

static void on_error(const char* msg, void* ud) { (void)ud; fprintf(stderr, "[grk error] %s\n", msg); }

static int enc(int argc, char** argv) {
    const char* raw = argv[2];
    uint32_t w = (uint32_t)atoi(argv[3]), h = (uint32_t)atoi(argv[4]), c = (uint32_t)atoi(argv[5]);
    uint32_t prec = (uint32_t)atoi(argv[6]);
    const char* out = argv[7];
    grk_cparameters p;
    grk_compress_set_default_params(&p);
    GRK_CODEC_FORMAT fmt = GRK_CODEC_J2K;
    int raw_tiles = 0;
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
        else if (!strcmp(argv[i], "-c")) {   /* one precinct size for every resolution: [W,H] */
            unsigned pw, ph;
            sscanf(argv[++i], "[%u,%u]", &pw, &ph);
            p.csty |= 1; p.res_spec = 1; p.prcw_init[0] = pw; p.prch_init[0] = ph;
        }
    }
    if (c >= 3) p.mct = 1;   /* grk_compress.cpp:1978-1995: RGB input switches the MCT on */
    grk_initialize(NULL, 0);
    grk_set_error_handler(on_error, NULL);
    grk_image_cmptparm cp[4];
    memset(cp, 0, sizeof cp);
    for (uint32_t k = 0; k < c; ++k) { cp[k].dx = cp[k].dy = 1; cp[k].w = w; cp[k].h = h; cp[k].prec = (uint8_t)prec; }
    grk_image* img = grk_image_new((uint16_t)c, cp, c >= 3 ? GRK_CLRSPC_SRGB : GRK_CLRSPC_GRAY, true);
    if (!img) return 2;
    FILE* f = fopen(raw, "rb");
    int32_t* row = malloc(sizeof(int32_t) * w);
    for (uint32_t k = 0; k < c; ++k)
        for (uint32_t y = 0; y < h; ++y) {
            if (fread(row, 4, w, f) != w) return 3;
            memcpy(img->comps[k].data + (size_t)y * img->comps[k].stride, row, 4 * w);
        }
    fclose(f);
    size_t cap = (size_t)w * h * c * 4 + (1 << 20);
    uint8_t* buf = malloc(cap);
    grk_stream* st = grk_stream_create_mem_stream(buf, cap, false, false);
    grk_codec* codec = grk_compress_create(fmt, st);
    if (!codec || !grk_compress_init(codec, &p, img) || !grk_compress_start(codec)) return 4;
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
        ok = grk_compress(codec);
    }
    if (!ok || !grk_compress_end(codec)) return 5;
    size_t n = grk_stream_get_write_mem_stream_length(st);
    f = fopen(out, "wb");
    fwrite(buf, 1, n, f);
    fclose(f);
    grk_object_unref(codec);
    grk_object_unref(st);
    grk_object_unref(&img->obj);
    free(buf);
    free(row);
    grk_deinitialize();
    return 0;
}

static int dec(int argc, char** argv) {
    const char* in = argv[2];
    const char* out = argv[3];
    grk_initialize(NULL, 0);
    grk_set_error_handler(on_error, NULL);
    grk_dparameters dp;
    grk_decompress_set_default_params(&dp);
    int win = 0, tile = -1;
    uint32_t x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    for (int i = 4; i < argc; ++i) {
        if (!strcmp(argv[i], "-d")) { sscanf(argv[++i], "%u,%u,%u,%u", &x0, &y0, &x1, &y1); win = 1; }
        else if (!strcmp(argv[i], "-tile")) tile = atoi(argv[++i]);
    }
    const size_t L = strlen(in);
    GRK_CODEC_FORMAT fmt = L > 4 && !strcmp(in + L - 4, ".jp2") ? GRK_CODEC_JP2 : GRK_CODEC_J2K;
    grk_stream* st = grk_stream_create_file_stream(in, 1 << 20, true);
    grk_codec* codec = grk_decompress_create(fmt, st);
    grk_header_info hi;
    memset(&hi, 0, sizeof hi);
    if (!codec || !grk_decompress_init(codec, &dp) || !grk_decompress_read_header(codec, &hi)) return 6;
    fprintf(stdout, "header cblk %ux%u numres %u layers %u irrev %d tiles %ux%u\n", hi.cblockw_init, hi.cblockh_init,
            hi.numresolutions, hi.numlayers, (int)hi.irreversible, hi.t_grid_width, hi.t_grid_height);
    grk_image* img;
    if (tile >= 0) {
        if (!grk_decompress_tile(codec, (uint16_t)tile)) return 7;
        img = grk_decompress_get_tile_image(codec, (uint16_t)tile);
    } else {
        if (win && !grk_decompress_set_window(codec, x0, y0, x1, y1)) return 8;
        if (!grk_decompress(codec, NULL) || !grk_decompress_end(codec)) return 9;
        img = grk_decompress_get_composited_image(codec);
    }
    if (!img) return 10;
    fprintf(stdout, "image %u %u %u %u comps %u\n", img->x0, img->y0, img->x1, img->y1, img->numcomps);
    FILE* f = fopen(out, "wb");
    for (uint32_t k = 0; k < img->numcomps; ++k)
        for (uint32_t y = 0; y < img->comps[k].h; ++y)
            fwrite(img->comps[k].data + (size_t)y * img->comps[k].stride, 4, img->comps[k].w, f);
    fclose(f);
    grk_object_unref(codec);
    grk_object_unref(st);
    grk_deinitialize();
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 8 && !strcmp(argv[1], "enc")) return enc(argc, argv);
    if (argc >= 4 && !strcmp(argv[1], "dec")) return dec(argc, argv);
    fprintf(stderr, "usage: enc RAW W H C PREC OUT [opts] | dec IN RAWOUT [-d x0,y0,x1,y1] [-tile t]\n");
    return 1;
}
