// gk_common.h — descriptors shared by the host engine and the HIP kernels.
//
// Layout in HBM (DESIGN.md §Data layout):
//   * a tile component is planar int32 (or f32 for 9/7), row stride = align32(width)
//     samples (Grok's grkMakeAlignedWidth, cache/MemManager.cpp:35-43);
//   * the forward DWT ping-pongs between two full-size work planes per component
//     (A, B); level l writes its four subbands in Mallat placement into plane
//     (l odd ? B : A), so every band is a (ptr, stride, w, h) window;
//   * T1 reads/writes code-blocks straight out of those band windows.
#pragma once
#include <stdint.h>

#define GK_MAX_RES 33
#define GK_CTX 19

// Caller sample types of the image planes (gk_image_info::sample_bytes + sgnd):
// Grok's int32 image components, or the planar 8/16-bit buffers of
// TileProcessor::ingestUncompressedData (TileProcessor.cpp:779-835).
enum GkSample { GK_S32 = 0, GK_U8 = 1, GK_S8 = 2, GK_U16 = 3, GK_S16 = 4 };
static inline __host__ __device__ uint32_t gk_sample_size(int t) { return t == GK_S32 ? 4 : (t <= GK_S8 ? 1 : 2); }

// One code-block job (encode or decode).
struct GkBlock {
    uint64_t band_off;     // element offset of the block's top-left sample in the coefficient arena
    uint32_t stride;       // row stride in elements
    uint16_t w, h;         // block size: 4..1024 per side, w * h <= 4096 (sides above 64: gk_t1ms.hip / wide HT)
    uint8_t orient;        // 0 LL, 1 HL, 2 LH, 3 HH
    uint8_t comp;
    uint8_t band_numbps;   // Quantizer.cpp:45-49 (decode: numbps - k_msbs)
    uint8_t flags;         // bit0: irreversible, bit1: rate control (collect per-pass distortion)
    float step;            // 9/7 encode: band stepsize (divisor, T1Part1.cpp:70-76); decode: stepsize/2 (ScaleFilter)
    double wmse;           // encode + rate control: w1 * w2 * stepsize of T1::getwmsedec (T1.cpp:418-436)
    // encode outputs / decode inputs
    uint64_t data_off;     // byte offset of the block's compressed data (slot) in the byte arena
    uint32_t data_cap;     // slot capacity (encode)
    uint32_t numbps;       // encode: output; decode: input (cblk->numbps)
    uint32_t npasses;      // encode: output; decode: input
    uint32_t len;          // encode: output bytes; decode: input bytes
};

// Pass information written by the encoder (max 3*31-2 passes per block).
// Default code-block style: only the last pass is terminated (T1.cpp:437-458).
#define GK_MAX_PASSES 96
#define GK_HT_MEL_CAP 1024   // MEL staging bytes per HT block (encoder)
struct GkPass {
    uint32_t rate;         // cumulative bytes after the pass (T1.cpp:856-930 rules)
    uint32_t len;          // rate - previous rate
    double dist;           // cumulative distortion decrease, Grok's distortiondec (rate control only)
};

// 2D window for DWT/MCT kernels.
struct GkPlane {
    uint64_t off;          // element offset in arena
    uint32_t stride;
    uint32_t w, h;
};

// A rectangular batch of equally-sized tiles for the level kernels (grid.z =
// tile): tile z of the batch starts at image row (j0 + z / nx) * dy, column
// (i0 + z % nx) * dx; each tile is transformed independently.  The work plane
// holds the image region whose top-left sample is (ox, oy) (a tile rectangle
// for sharded / windowed calls, the whole image otherwise).
struct GkTiles {
    uint32_t nx = 1, ny = 1, i0 = 0, j0 = 0, dx = 0, dy = 0, ox = 0, oy = 0;
    __host__ __device__ uint32_t count() const { return nx * ny; }
    __host__ __device__ uint64_t offset(uint32_t z, uint32_t stride) const {
        return (uint64_t)((j0 + z / nx) * dy - oy) * stride + (uint64_t)((i0 + z % nx) * dx - ox);
    }
    // top-left of tile z in work-plane (region) coordinates
    __host__ __device__ void origin(uint32_t z, int32_t& x, int32_t& y) const {
        x = (int32_t)((i0 + z % nx) * dx - ox);
        y = (int32_t)((j0 + z / nx) * dy - oy);
    }
};

// Components of one level launch: component c's plane at base + c * cstride elements,
// grid.z = component * tiles + tile.
struct GkComps {
    uint64_t cstride = 0;
    uint32_t n = 1;
};
// Caller planes of up to three components (fused level-1 kernels).
struct GkPtr3 {
    const void* p[3] = {nullptr, nullptr, nullptr};
};
// Output window of a fused last inverse level, in work-plane (region) coordinates.
struct GkWin {
    int32_t x0 = 0, y0 = 0, x1 = 0, y1 = 0;
};
