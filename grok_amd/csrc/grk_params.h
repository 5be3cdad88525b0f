// grk_params.h — grk_cparameters (grok.h:466-590) -> gk_cparameters, shared by the grk_*
// shim (grk_shim.cpp) and the T1 plugin (grk_plugin.cpp).
//
// Follows CodeStreamCompress::initCompress (CodeStreamCompress.cpp:150-610).  Features outside
// the GPU path are refused with a reason, never approximated.
#pragma once
#include <cstdio>
#include <string>

#include "../../include/grk_abi.h"
#include "../../include/grok_amd.h"

// ntiles: the image's tile count (progression order changes are given per tile).
inline bool grk_params_to_gk(const grk_cparameters& g, bool jp2, gk_cparameters& p, std::string& why,
                             uint32_t ntiles = 1) {
    char msg[256];
    auto refuse = [&](const char* m) { why = m; return false; };
    gk_set_default_params(&p);
    if (g.numresolution < 1 || g.numresolution > GRK_J2K_MAXRLVLS) {
        snprintf(msg, sizeof msg, "Invalid number of resolutions : %u not in range [1,%u]", g.numresolution,
                 GRK_J2K_MAXRLVLS);
        return refuse(msg);
    }
    if (g.prog_order < GRK_LRCP || g.prog_order > GRK_CPRL) return refuse("unknown progression order");
    // tile grid origin (-T); the image origin travels with the image (grk_image::x0 / y0: the CLI's
    // readers set it from image_offset_x0 / y0, which the library itself does not read)
    p.tx0 = g.tx0; p.ty0 = g.ty0;
    if (g.tile_size_on && (!g.t_width || !g.t_height)) return refuse("tile size must be non-zero when tiling is on");
    // mct 255 = not set on the command line: grk_compress resolves it from the component count
    // once the image is loaded (grk_compress.cpp:1977-1981), as the engine does (>= 3 -> RCT/ICT)
    if (g.mct_data || (g.mct > 1 && g.mct != 255)) return refuse("Part-2 array MCT is not supported");
    if (g.num_comments > GK_NUM_COMMENTS) return refuse("too many comments");
    p.num_comments = (uint32_t)g.num_comments;   // grk_compress -C (CodeStreamCompress.cpp:303-330)
    for (size_t i = 0; i < g.num_comments; ++i) {
        p.comment[i] = g.comment[i]; p.comment_len[i] = g.comment_len[i]; p.is_binary_comment[i] = g.is_binary_comment[i];
    }
    if (g.csty & ~7u) return refuse("unknown coding style bits (csty)");
    const uint32_t sty = (g.isHT ? GRK_CBLKSTY_HT : 0) | g.cblk_sty;
    if (sty > 0x7f || ((sty & GRK_CBLKSTY_HT) && sty != GRK_CBLKSTY_HT)) {
        snprintf(msg, sizeof msg, "code-block style 0x%x is not supported on this path", sty);
        return refuse(msg);
    }
    if ((g.rsiz & ~GRK_JPH_RSIZ_FLAG) != GRK_PROFILE_NONE) {
        snprintf(msg, sizeof msg, "profile 0x%x is not supported", g.rsiz);
        return refuse(msg);
    }
    p.numlayers = g.numlayers ? g.numlayers : 1;
    // a tile takes the PSNR targets under allocationByQuality, the compression ratios otherwise
    // (CodeStreamCompress.cpp:387-393)
    const bool q = g.allocationByQuality && g.numlayers;
    p.allocationByQuality = q ? 1 : 0;
    for (uint32_t l = 0; l < p.numlayers && l < GRK_MAX_LAYERS; ++l) {
        p.layer_rate[l] = (g.numlayers && !q) ? g.layer_rate[l] : 0.0;
        p.layer_distortion[l] = q ? g.layer_distortion[l] : 0.0;
    }
    p.numresolution = g.numresolution;
    p.cblockw_init = g.cblockw_init; p.cblockh_init = g.cblockh_init;
    p.cblk_sty = (uint8_t)sty;
    p.irreversible = g.irreversible ? 1 : 0;
    p.mct = g.mct == 255 ? 1 : g.mct;
    p.numgbits = g.numgbits;
    p.csty = g.csty;
    p.res_spec = g.res_spec;
    for (int r = 0; r < GK_MAXRLVLS; ++r) { p.prcw_init[r] = g.prcw_init[r]; p.prch_init[r] = g.prch_init[r]; }
    p.write_comment = 1;
    p.tile_size_on = g.tile_size_on;
    p.t_width = g.t_width; p.t_height = g.t_height;
    p.writeTLM = g.writeTLM; p.writePLT = g.writePLT;
    p.cod_format = jp2 ? 2 : 0;
    p.prog_order = (int32_t)g.prog_order;
    p.roi_compno = g.roi_compno; p.roi_shift = g.roi_shift;
    p.enableTilePartGeneration = g.enableTilePartGeneration ? 1 : 0;
    p.newTilePartProgressionDivider = g.newTilePartProgressionDivider;
    if (g.numpocs) {
        // CodeStreamCompress.cpp:397-427: numpocs + 1 entries (grk_compress -P T<t>=...); tile t
        // takes as many entries as name it - copied from the head of the list (the loop indexes
        // by its own counter) - and a tile named by none is an error.  One entry is no change
        // (tcp->numpocs = 0: the tile keeps prog_order).  The engine codes one list for every tile.
        const uint32_t n = g.numpocs + 1;
        if (n > GRK_J2K_MAXRLVLS || n > 32) return refuse("too many progression order changes");
        uint32_t k = 0;
        for (uint32_t t = 0; t < ntiles; ++t) {
            uint32_t c = 0;
            for (uint32_t i = 0; i < n; ++i) c += g.progression[i].tileno == t;
            if (!c) return refuse("Problem with specified progression order changes");
            if (t && c != k) return refuse("progression order changes that differ between tiles are not supported");
            k = c;
        }
        if (k > 1) {
            p.numpocs = k;
            for (uint32_t i = 0; i < k; ++i) {
                const grk_progression& e = g.progression[i];
                p.pocs[i].resS = e.resS; p.pocs[i].compS = e.compS; p.pocs[i].layE = e.layE;
                p.pocs[i].resE = e.resE; p.pocs[i].compE = e.compE;
                p.pocs[i].prog = (int32_t)e.specifiedCompressionPocProg;
            }
        }
    }
    return true;
}
