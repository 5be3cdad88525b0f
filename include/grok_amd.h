/*
 * grok_amd.h — C ABI of the MI355X JPEG 2000 tile-pipeline engine.
 *
 * Drop-in boundary for Grok 9.2.0's hot path.  Plain C types,
 * plain pointers and sizes; no torch/HIP types in any signature.  Every entry
 * point cites the reference interface it replaces (paths relative to
 * /root/reference/src/lib/jp2/).  INTEGRATION.md shows the reference-side
 * binding (ctypes / C call sites) a maintainer would add.
 *
 * Conventions mirror grok.h: functions return 0 / non-NULL on success and a
 * negative code on failure (grok.h returns bool false); messages are
 * retrievable with gk_last_error() (grok.h routes them to grk_set_error_handler
 * callbacks, grok.cpp:116-134).  Calls on one context are synchronous and
 * single-threaded, like calls on one grk_codec (grok.cpp:71-86).
 */
#ifndef GROK_AMD_H
#define GROK_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GK_MAXRLVLS 33
#define GK_MAX_LAYERS 100
#define GK_NUM_COMMENTS 256   /* GRK_NUM_COMMENTS_SUPPORTED */

/* One progression order change (grk_progression's resS, compS, layE, resE, compE, progression;
 * POC marker A.6.6): layers [0, layE), resolutions [resS, resE), components [compS, compE). */
typedef struct gk_poc {
    uint32_t resS, compS, layE, resE, compE;
    int32_t prog;                        /* GRK_PROG_ORDER */
} gk_poc;

/* Coding parameters: the subset of grk_cparameters (grok.h:466-590) the hot
 * path consumes, with the same field names and meaning. */
typedef struct gk_cparameters {
    uint16_t numlayers;                  /* grk_cparameters::numlayers */
    double layer_rate[GK_MAX_LAYERS];    /* grk_cparameters::layer_rate (compression ratio, 0 = lossless) */
    uint8_t numresolution;               /* grk_cparameters::numresolution (default 6) */
    uint32_t cblockw_init, cblockh_init; /* grk_cparameters::cblockw_init / cblockh_init (default 64) */
    uint8_t cblk_sty;                    /* grk_cparameters::cblk_sty: Part-1 mode switches (LAZY 1, RESET 2, TERMALL 4,
                                            VSC 8, PTERM 0x10, SEGSYM 0x20) or 0x40 alone (HTJ2K, GRK_CBLKSTY_HT) */
    uint8_t irreversible;                /* grk_cparameters::irreversible */
    uint8_t mct;                         /* grk_cparameters::mct (RCT/ICT for >= 3 components) */
    uint8_t numgbits;                    /* grk_cparameters::numgbits (default 2) */
    uint8_t csty;                        /* grk_cparameters::csty: bit0 user precincts, 2 SOP before every packet
                                            (grk_compress -S), 4 EPH after every packet header (-E) */
    uint32_t res_spec;                   /* grk_cparameters::res_spec */
    uint32_t prcw_init[GK_MAXRLVLS];     /* grk_cparameters::prcw_init */
    uint32_t prch_init[GK_MAXRLVLS];     /* grk_cparameters::prch_init */
    uint8_t write_comment;               /* write Grok's default COM marker (CodeStreamCompress.cpp:334) */
    uint8_t tile_size_on;                /* grk_cparameters::tile_size_on */
    uint32_t t_width, t_height;          /* grk_cparameters::t_width / t_height (tile origins on the 2^levels grid) */
    uint8_t writeTLM;                    /* grk_cparameters::writeTLM (grk_compress -X) */
    uint8_t writePLT;                    /* grk_cparameters::writePLT (grk_compress -L) */
    int32_t cod_format;                  /* grk_cparameters::cod_format: GRK_CODEC_J2K (0, raw codestream) or
                                            GRK_CODEC_JP2 (2, JP2 file boxes around it; FileFormatCompress.cpp) */
    int32_t prog_order;                  /* grk_cparameters::prog_order: GRK_LRCP 0, RLCP 1, RPCL 2, PCRL 3, CPRL 4 */
    uint8_t enableTilePartGeneration;    /* grk_cparameters::enableTilePartGeneration (grk_compress -u) */
    char newTilePartProgressionDivider;  /* grk_cparameters::newTilePartProgressionDivider: 'L', 'R' or 'C' */
    int32_t roi_compno;                  /* grk_cparameters::roi_compno (-1: none) */
    uint32_t roi_shift;                  /* grk_cparameters::roi_shift: RGN maxshift of that component (Part-1) */
    uint32_t numpocs;                    /* progression order changes, written as a POC marker in each tile's
                                            first tile-part header (CodeStreamCompress::writePoc) */
    gk_poc pocs[32];
    uint8_t allocationByQuality;         /* grk_cparameters::allocationByQuality (grk_compress -q): layers by PSNR */
    double layer_distortion[GK_MAX_LAYERS]; /* grk_cparameters::layer_distortion: PSNR per layer (0 = the rest) */
    uint32_t tx0, ty0;                   /* grk_cparameters::tx0 / ty0 (grk_compress -T): tile grid origin on the
                                            canvas, at or above-left of the image origin (B.3) */
    /* grk_cparameters::comment / comment_len / is_binary_comment / num_comments (grk_compress -C):
       COM markers written instead of Grok's default one (CodeStreamCompress.cpp:303-330 keeps the
       non-empty ones, write_com :1114-1145 writes Rcom 1 (text) or 0 (binary) and the bytes) */
    uint32_t num_comments;
    const char* comment[GK_NUM_COMMENTS];
    uint16_t comment_len[GK_NUM_COMMENTS];
    uint8_t is_binary_comment[GK_NUM_COMMENTS];
} gk_cparameters;

/* Image description: grk_image / grk_image_comp (grok.h:895-959) reduced to
 * what the tile pipeline reads.  Component planes are int32 (grk_image_comp::data),
 * row stride in samples (grk_image_comp::stride). */
typedef struct gk_image_info {
    uint32_t w, h;          /* grk_image::x1 - x0, y1 - y0: the image area (tiles per gk_cparameters) */
    uint32_t numcomps;      /* grk_image::numcomps */
    uint32_t prec;          /* grk_image_comp::prec (same for every component) */
    uint32_t sgnd;          /* grk_image_comp::sgnd */
    uint32_t sample_bytes;  /* the caller's planes: 0 or 4 = int32 (grk_image_comp::data); 1 / 2 = planar
                               8 / 16-bit samples, signed iff sgnd, as grk_compress_tile's buffer
                               (TileProcessor::ingestUncompressedData, TileProcessor.cpp:779-835);
                               must be 4 or (prec + 7) / 8.  Decode writes the same type. */
    uint32_t x0, y0;        /* grk_image::x0 / y0 (grk_compress -d): the image area's canvas origin (SIZ
                               XOsiz / YOsiz); planes hold the area only, windows are relative to it */
} gk_image_info;

/* Per-stage device times of the last call (HIP events on the engine stream). */
typedef struct gk_timings {
    float mct_ms, dwt_ms, t1_ms, t2_ms, assemble_ms, total_ms;
    float t1_cm_ms;         /* encode: context-modelling kernel (k_t1_cm) part of t1_ms */
    float t1_coder_ms;      /* the arithmetic-coder kernel alone: k_t1_mq (encode) / k_t1_dec (decode) */
    uint32_t dwt_launches, t1_blocks;
    uint64_t dwt_bytes;     /* algorithmic bytes moved by the DWT launches */
    uint64_t cs_bytes;      /* codestream bytes produced (encode) / consumed (decode) */
    uint64_t t1_bytes;      /* compressed code-block bytes coded by T1 */
    /* Part-1 decode with GK_T1_STATS set in the environment (0 otherwise): decision steps of
       the longest-running wave, all steps issued, symbols decoded (the T1 chain's work) */
    uint64_t t1_steps_max, t1_steps_total, t1_symbols;
    /* Part-1 decode: code-blocks given to solo waves (one wave per block on the SIMDs the
       lane-parallel waves leave); with GK_T1_STATS, their decisions and the largest per wave */
    uint64_t t1_solo_blocks, t1_solo_decisions, t1_solo_decisions_max;
} gk_timings;

typedef struct gk_ctx gk_ctx;

/* grk_initialize (grok.cpp:75-86): create an engine bound to one MI355X. */
gk_ctx* gk_create(int device_id);
/* grk_deinitialize / grk_object_unref(codec) */
void gk_destroy(gk_ctx* ctx);
/* grk_compress_set_default_params (grok.cpp:405-435) */
void gk_set_default_params(gk_cparameters* p);

/* grk_compress_init + grk_compress_start + grk_compress + grk_compress_end
 * (grok.cpp:382-469; TileProcessor::doCompress TileProcessor.cpp:202-260) for a
 * single- or multi-tile image (all tiles in one pass; one tile part per tile).  comps[c] points at component c's plane (device
 * memory if comps_on_device, host otherwise).  The codestream is written to
 * out (device memory if out_on_device); *out_len receives its size.
 * Returns 0, or < 0 on error (-2: capacity too small, *out_len = needed). */
int gk_encode(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
              int comps_on_device, const gk_cparameters* p, uint8_t* out, size_t cap, size_t* out_len,
              int out_on_device);

/* Tile sharding: encode only tiles [tile_begin, tile_end) of the
 * image described by info / p — grk_compress_tile (grok.h:1082-1657) per tile, without
 * the main header.  comps[c] addresses the image origin; only the sample rows of the
 * selected tiles are read.  out receives their tile parts (SOT [PLT] SOD packets,
 * CodeStreamCompress::writeTilePart :862-900) back to back; part_lens[i] = length
 * of tile tile_begin + i (the TLM Ptlm value).  Returns 0 / < 0 like gk_encode. */
int gk_encode_tiles(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
                    int comps_on_device, const gk_cparameters* p, uint32_t tile_begin, uint32_t tile_end,
                    uint8_t* out, size_t cap, size_t* out_len, uint32_t* part_lens, int out_on_device);

/* Main header alone (SOC SIZ [CAP] COD QCD [TLM] [COM]; CodeStreamCompress::
 * init_header_writing :822-860) for assembling sharded tile parts: codestream =
 * header + tile parts in tile order + EOC (0xFFD9).  With TLM, *tlm_offset is the
 * offset of the first 6-byte entry (Ttlm u16 = tile index, Ptlm u32 = tile-part
 * length, big-endian) for the caller to fill; *num_tiles = tiles in the grid. */
int gk_main_header(gk_ctx* ctx, const gk_image_info* info, const gk_cparameters* p, uint8_t* out, size_t cap,
                   size_t* out_len, size_t* tlm_offset, uint32_t* num_tiles);

/* JP2 boxes for a file wrapping a codestream of cs_len bytes (signature, ftyp, jp2h with
 * ihdr + colr, jp2c box header; FileFormatCompress::startCompress / write_jp2c,
 * FileFormatCompress.cpp:666-693, 59-102): JP2 file = these bytes + the codestream.  Used to
 * assemble sharded tile parts into a .jp2.  Returns 0, -2 if cap is too small (*out_len = needed). */
int gk_jp2_header(gk_ctx* ctx, const gk_image_info* info, uint64_t cs_len, uint8_t* out, size_t cap, size_t* out_len);

/* grk_decompress_read_header (grok.cpp:287-297, CodeStreamDecompress::readHeader) of a raw
 * codestream or a JP2 file (its jp2c box; FileFormatDecompress::read_box_hdr :632-672). */
int gk_decode_header(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, gk_image_info* info);

/* The same header parse on host bytes without an engine (no device needed): image info of a
 * codestream / JP2 file and, when coding != NULL, its coding style in gk_cparameters terms
 * (CodeStreamDecompress main-header markers; what grk_decompress_read_header reports in
 * grk_header_info), or < 0 with the reason in msg. */
int gk_probe_header(const uint8_t* cs, size_t len, gk_image_info* info, gk_cparameters* coding, char* msg,
                    size_t msg_cap);

/* grk_decompress (grok.cpp:287-297; TileProcessor::decompressT2T1 TileProcessor.cpp:384-408):
 * decode into comps[c] (device memory if out_on_device): int32 planes (sample_bytes 0 / 4) or planar
 * (prec + 7) / 8-byte samples (sample_bytes 1 / 2, signed iff the image is; gk_image_info).  Every tile
 * part present in cs is decoded; a stream holding the main header and only some
 * tile parts (tile sharding, window decode) writes only those tiles' samples. */
int gk_decode(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, void* const* comps,
              const uint32_t* strides, uint32_t sample_bytes, int out_on_device);

/* grk_dparameters::cp_layer (CodeStreamDecompress.cpp:2570-2579): later gk_decode /
 * gk_decode_window calls decode only the first max_layers quality layers (0 = all); packets of
 * later layers are skipped through PLT or parsed without their data (T2Decompress.cpp:55-116). */
int gk_set_decode_layers(gk_ctx* ctx, uint32_t max_layers);

/* grk_dparameters::cp_reduce (CodeStreamDecompress / TileComponent resolutions_to_decompress):
 * later gk_decode calls discard the `reduce` highest resolutions: packets of those resolutions
 * are skipped, the inverse DWT stops `reduce` levels early and the output planes are
 * ceil(w / 2^reduce) x ceil(h / 2^reduce) (0 = full resolution); gk_decode_window then returns
 * the window on the reduced canvas (every edge of its canvas rectangle ceil(x / 2^reduce),
 * CodeStreamDecompress.cpp:471-481). */
int gk_set_decode_reduce(gk_ctx* ctx, uint32_t reduce);

/* grk_image_comp::dx / dy of the components of later gk_encode / gk_encode_tiles / gk_main_header calls (SIZ XRsiz /
 * YRsiz, 1..255; numcomps = 0 clears it).  Component c's plane then holds the image area sampled
 * every (dx[c], dy[c]) canvas positions: ceil((x0 + w) / dx) - ceil(x0 / dx) columns and the same
 * in y (grk_image_comp w / h), row stride strides[c].  Its tile-components are the tiles divided
 * by (dx, dy), rounded up (TileProcessor.cpp:116-131); the MCT is cleared unless the first three
 * components share a grid (CodeStreamCompress.cpp:501-512); rate control takes component 0's
 * factors (updateRates :961).  Tiled images need each factor to divide the tile size.  With
 * gk_encode_tiles, comps[c] addresses component c's plane at its row 0 and only the rows of the
 * selected tiles (on that component's grid) are read. */
int gk_set_subsampling(gk_ctx* ctx, uint32_t numcomps, const uint32_t* dx, const uint32_t* dy);

/* A stream's components from its header, no device needed (SIZ XRsiz / YRsiz / Ssiz): fills dx[c],
 * dy[c], prec[c], sgnd[c] (any may be NULL) for the first cap components and returns the component
 * count (< 0 on error).  gk_decode writes component c into a plane of its own size: the image area
 * divided by (dx, dy) as in gk_set_subsampling, then reduced by cp_reduce (ceil of both edges /
 * 2^reduce); windows take the window's rectangle on each component's grid.  Components of
 * different precisions are DC-shifted and clamped each by its own (gk_image_info::prec reports the
 * largest; 8 / 16-bit output needs one sign). */
int gk_probe_components(const uint8_t* cs, size_t len, uint32_t* dx, uint32_t* dy, uint32_t* prec, uint32_t* sgnd,
                        uint32_t cap);

/* The same for the stream the last gk_decode_header read (host or device bytes); returns the
 * component count. */
int gk_header_components(gk_ctx* ctx, uint32_t* dx, uint32_t* dy, uint32_t* prec, uint32_t* sgnd, uint32_t cap);

/* Inverse 5/3 rule of later gk_decode_window calls.  whole_tile = 0 (default): Grok's partial-tile
 * inverse, which a window set through setDecompressWindow selects for every tile
 * (CodeStreamDecompress.cpp:389; a one-sample-wide resolution on an odd coordinate shifts its
 * sample, WaveletReverse.cpp:1551-1554).  whole_tile = 1: the whole-tile rule (that sample halved,
 * WaveletReverse.cpp:583), which CodeStreamDecompress::decompressTile keeps when no window is set
 * (grk_decompress_tile with the CLI's set_window(0,0,0,0), :309-316, 416-493). */
int gk_set_window_rule(gk_ctx* ctx, int whole_tile);

/* grk_decompress_set_window + grk_decompress (grok.h:1082-1657; CodeStreamDecompress
 * window decode): decode the window [x0, x1) x [y0, y1) of the image.
 * Only the tile parts of tiles intersecting the window are read (located through TLM
 * when present, their packet headers through PLT), decoded and inverse-transformed;
 * comps[c][0] receives sample (x0, y0) of component c, row stride strides[c] (with
 * gk_set_decode_reduce: the reduced window's first sample, see there). */
int gk_decode_window(gk_ctx* ctx, const uint8_t* cs, size_t len, int cs_on_device, uint32_t x0, uint32_t y0,
                     uint32_t x1, uint32_t y1, void* const* comps, const uint32_t* strides, uint32_t sample_bytes,
                     int out_on_device);

/* Code-block results of a single-tile encode, for Grok's T1 plugin interface (SURVEY.md
 * §8(b) B2: grk_plugin_tile -> ... -> grk_plugin_code_block, grok.h:995-1077): what the host
 * takes from the plugin in compress_synch_with_plugin (plugin/plugin_bridge.cpp:146-270).
 * Order is canonical: component, resolution, band, precinct, code-block
 * (T1CompressScheduler.cpp:31-94). */
typedef struct gk_band_result {
    uint32_t comp, res, band;   /* position in the tile tree */
    uint32_t orient;            /* 0 LL, 1 HL, 2 LH, 3 HH (grk_plugin_band::orientation) */
    uint32_t num_precincts;     /* grk_plugin_band::numPrecincts (precinct grid of the resolution) */
    float stepsize;             /* the band's quantisation step (Subband::stepsize) */
} gk_band_result;
typedef struct gk_block_result {
    uint32_t comp, res, band, precinct, cblk;   /* position; cblk = raster index in the precinct */
    uint32_t x0, y0, x1, y1;                    /* code-block rectangle in band coordinates */
    uint32_t numbps;                            /* Codeblock::numbps */
    uint32_t npasses;                           /* CompressCodeblock::numPassesTotal */
    uint32_t len;                               /* compressed bytes */
    uint32_t pass_off;                          /* first pass record in the pass array */
    uint64_t data_off;                          /* first byte in the byte array */
} gk_block_result;
typedef struct gk_pass_result {
    uint32_t rate;     /* cumulative bytes after the pass (CodePass::rate, T1.cpp:856-930 rules) */
    uint32_t len;      /* rate - previous rate (CodePass::len) */
    double dist;       /* cumulative distortion decrease (CodePass::distortiondec); 0 unless the
                          parameters ask for rate control (TileProcessor::needsRateControl) */
} gk_pass_result;

/* TileProcessor::doCompress up to and including T1 (TileProcessor.cpp:202-232: DC shift, MCT,
 * DWT, t1_encode) of a single-tile image; the results stay in the context and *nbands,
 * *nblocks, *nbytes, *npasses receive their counts.  Returns 0 / < 0 (error). */
int gk_encode_blocks(gk_ctx* ctx, const gk_image_info* info, const void* const* comps, const uint32_t* strides,
                     int comps_on_device, const gk_cparameters* p, uint32_t* nbands, uint32_t* nblocks,
                     uint64_t* nbytes, uint32_t* npasses);
/* Copies the results of the last gk_encode_blocks into caller arrays of the reported sizes
 * (any pointer may be NULL to skip that array). */
int gk_encode_blocks_get(gk_ctx* ctx, gk_band_result* bands, gk_block_result* blocks, uint8_t* data,
                         gk_pass_result* passes);

/* Stage timings of the last gk_encode / gk_decode. */
int gk_get_timings(gk_ctx* ctx, gk_timings* t);
/* Last error message for this context (grk_set_error_handler equivalent). */
const char* gk_last_error(gk_ctx* ctx);
/* Engine version string (grk_version, grok.cpp). */
const char* gk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GROK_AMD_H */
