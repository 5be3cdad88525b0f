/*
 * grk_abi.h — the grk_* C API of Grok 9.2.0 as served by libgrok_amd.so.
 *
 * The reference interface is /root/reference/src/lib/jp2/grok.h:1082-1657 (implementation
 * grok.cpp:75-870).  A program compiled against Grok's grok.h and linked against this
 * library instead of libgrokj2k runs unchanged: the entry points below
 * have grok.h's names and signatures, and every struct a caller touches has grok.h's memory
 * layout (field order and C types), checked field by field by tests/test_grk_abi.py against
 * the reference header.  Only the layout is shared; this header is not a copy of grok.h.
 *
 * Implemented by grok_amd/csrc/grk_shim.cpp over the engine of include/grok_amd.h: the
 * tile pipeline runs on the MI355X; streams, images and codecs are host objects.
 */
#ifndef GRK_ABI_H
#define GRK_ABI_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- limits (grok.h:75-104) */
#define GRK_PATH_LEN 4096
#define GRK_MAX_LAYERS 100
#define GRK_J2K_MAX_DECOMP_LVLS 32
#define GRK_J2K_MAXRLVLS (GRK_J2K_MAX_DECOMP_LVLS + 1)
#define GRK_NUM_COMMENTS_SUPPORTED 256
#define GRK_NUM_ASOC_BOXES_SUPPORTED 256
#define GRK_CBLKSTY_HT 0x40
#define GRK_PROFILE_NONE 0x0000
#define GRK_JPH_RSIZ_FLAG 0x4000
#define GRK_IMG_INFO 1
#define GRK_J2K_MH_INFO 2

/* ---- enumerations (values as grok.h) */
typedef enum GRK_SUPPORTED_FILE_FMT {
    GRK_UNK_FMT, GRK_J2K_FMT, GRK_JP2_FMT, GRK_PXM_FMT, GRK_PGX_FMT, GRK_PAM_FMT, GRK_BMP_FMT, GRK_TIF_FMT,
    GRK_RAW_FMT, GRK_PNG_FMT, GRK_RAWL_FMT, GRK_JPG_FMT
} GRK_SUPPORTED_FILE_FMT;
typedef enum _GRK_PROG_ORDER {
    GRK_PROG_UNKNOWN = -1, GRK_LRCP = 0, GRK_RLCP = 1, GRK_RPCL = 2, GRK_PCRL = 3, GRK_CPRL = 4, GRK_NUM_PROGRESSION_ORDERS = 5
} GRK_PROG_ORDER;
typedef enum _GRK_COLOR_SPACE {
    GRK_CLRSPC_UNKNOWN = 0, GRK_CLRSPC_SRGB = 2, GRK_CLRSPC_GRAY = 3, GRK_CLRSPC_SYCC = 4, GRK_CLRSPC_EYCC = 5,
    GRK_CLRSPC_CMYK = 6, GRK_CLRSPC_DEFAULT_CIE = 7, GRK_CLRSPC_CUSTOM_CIE = 8, GRK_CLRSPC_ICC = 9
} GRK_COLOR_SPACE;
typedef enum _GRK_CODEC_FORMAT { GRK_CODEC_UNKNOWN = -1, GRK_CODEC_J2K = 0, GRK_CODEC_JP2 = 2 } GRK_CODEC_FORMAT;
typedef enum GRK_TILE_CACHE_STRATEGY { GRK_TILE_CACHE_NONE, GRK_TILE_CACHE_ALL } GRK_TILE_CACHE_STRATEGY;
typedef enum grk_prec_mode { GRK_PREC_MODE_CLIP, GRK_PREC_MODE_SCALE } grk_precision_mode;
typedef enum GRK_COMPONENT_TYPE {
    GRK_COMPONENT_TYPE_COLOUR = 0, GRK_COMPONENT_TYPE_OPACITY = 1, GRK_COMPONENT_TYPE_PREMULTIPLIED_OPACITY = 2,
    GRK_COMPONENT_TYPE_UNSPECIFIED = 65535U
} GRK_COMPONENT_TYPE;
typedef enum GRK_COMPONENT_ASSOC {
    GRK_COMPONENT_ASSOC_WHOLE_IMAGE = 0, GRK_COMPONENT_ASSOC_COLOUR_1 = 1, GRK_COMPONENT_ASSOC_COLOUR_2 = 2,
    GRK_COMPONENT_ASSOC_COLOUR_3 = 3, GRK_COMPONENT_ASSOC_UNASSOCIATED = 65535U
} GRK_COMPONENT_ASSOC;

typedef void (*grk_msg_callback)(const char* msg, void* client_data);

/* Ref-counted handle: codecs, streams, images (grk_object_ref / grk_object_unref). */
typedef struct _grk_object { void* wrapper; } grk_object;
typedef grk_object grk_codec;
typedef grk_object grk_stream;

/* ---- compression parameters (grok.h:384-590) */
typedef struct _grk_progression {
    uint16_t layS, layE;
    uint8_t resS, resE;
    uint16_t compS, compE;
    uint64_t precS, precE;
    GRK_PROG_ORDER specifiedCompressionPocProg, progression;
    char progressionString[5];
    uint32_t tileno;
    uint32_t tx0, tx1, ty0, ty1;
    uint16_t tpLayE;
    uint8_t tpResS, tpResE;
    uint16_t tpCompS, tpCompE;
    uint64_t tpPrecE;
    uint32_t tp_txS, tp_txE, tp_tyS, tp_tyE;
    uint32_t dx, dy;
    uint16_t lay_temp;
    uint8_t res_temp;
    uint16_t comp_temp;
    uint64_t prec_temp;
    uint32_t tx0_temp, ty0_temp;
} grk_progression;

typedef struct _grk_raw_comp_cparameters { uint32_t dx, dy; } grk_raw_comp_cparameters;
typedef struct _grk_raw_cparameters {
    uint32_t width, height;
    uint16_t numcomps;
    uint8_t prec;
    bool sgnd;
    grk_raw_comp_cparameters* comps;
} grk_raw_cparameters;

typedef struct _grk_cparameters {
    bool tile_size_on;
    uint32_t tx0, ty0;
    uint32_t t_width, t_height;
    uint16_t numlayers;
    bool allocationByRateDistoration;
    double layer_rate[GRK_MAX_LAYERS];
    bool allocationByQuality;
    double layer_distortion[GRK_MAX_LAYERS];
    char* comment[GRK_NUM_COMMENTS_SUPPORTED];
    uint16_t comment_len[GRK_NUM_COMMENTS_SUPPORTED];
    bool is_binary_comment[GRK_NUM_COMMENTS_SUPPORTED];
    size_t num_comments;
    uint8_t csty;
    uint8_t numgbits;
    GRK_PROG_ORDER prog_order;
    grk_progression progression[GRK_J2K_MAXRLVLS];
    uint32_t numpocs;
    uint8_t numresolution;
    uint32_t cblockw_init, cblockh_init;
    uint8_t cblk_sty;
    bool isHT;
    bool irreversible;
    int32_t roi_compno;
    uint32_t roi_shift;
    uint32_t res_spec;
    uint32_t prcw_init[GRK_J2K_MAXRLVLS];
    uint32_t prch_init[GRK_J2K_MAXRLVLS];
    char infile[GRK_PATH_LEN];
    char outfile[GRK_PATH_LEN];
    uint32_t image_offset_x0, image_offset_y0;
    uint32_t subsampling_dx, subsampling_dy;
    GRK_SUPPORTED_FILE_FMT decod_format;
    GRK_SUPPORTED_FILE_FMT cod_format;
    grk_raw_cparameters raw_cp;
    uint32_t max_comp_size;
    bool enableTilePartGeneration;
    uint8_t newTilePartProgressionDivider;
    uint8_t mct;
    void* mct_data;
    uint64_t max_cs_size;
    uint16_t rsiz;
    uint16_t framerate;
    bool write_capture_resolution_from_file;
    double capture_resolution_from_file[2];
    bool write_capture_resolution;
    double capture_resolution[2];
    bool write_display_resolution;
    double display_resolution[2];
    uint32_t rateControlAlgorithm;
    uint32_t numThreads;
    int32_t deviceId;
    uint32_t duration;
    uint32_t kernelBuildOptions;
    uint32_t repeats;
    bool writePLT;
    bool writeTLM;
    bool verbose;
} grk_cparameters;

/* ---- colour and header information (grok.h:596-714) */
typedef struct _grk_channel_description { uint16_t cn, typ, asoc; } grk_channel_description;
typedef struct _grk_channel_definition {
    grk_channel_description* descriptions;
    uint16_t num_channel_descriptions;
} grk_channel_definition;
typedef struct _grk_component_mapping_comp {
    uint16_t component_index;
    uint8_t mapping_type;
    uint8_t palette_column;
} grk_component_mapping_comp;
typedef struct _grk_palette_data {
    int32_t* lut;
    uint16_t num_entries;
    grk_component_mapping_comp* component_mapping;
    uint8_t num_channels;
    bool* channel_sign;
    uint8_t* channel_prec;
} grk_palette_data;
typedef struct grk_color {
    uint8_t* icc_profile_buf;
    uint32_t icc_profile_len;
    grk_channel_definition* channel_definition;
    grk_palette_data* palette;
    bool has_colour_specification_box;
} grk_color;
typedef struct grk_asoc {
    uint32_t level;
    const char* label;
    uint8_t* xml;
    uint32_t xml_len;
} grk_asoc;
typedef struct _grk_header_info {
    uint32_t cblockw_init, cblockh_init;
    bool irreversible;
    uint32_t mct;
    uint16_t rsiz;
    uint32_t numresolutions;
    uint8_t csty;
    uint8_t cblk_sty;
    uint32_t prcw_init[GRK_J2K_MAXRLVLS];
    uint32_t prch_init[GRK_J2K_MAXRLVLS];
    uint32_t tx0, ty0;
    uint32_t t_width, t_height;
    uint32_t t_grid_width, t_grid_height;
    uint16_t numlayers;
    uint8_t* xml_data;
    size_t xml_data_len;
    size_t num_comments;
    char* comment[GRK_NUM_COMMENTS_SUPPORTED];
    uint16_t comment_len[GRK_NUM_COMMENTS_SUPPORTED];
    bool isBinaryComment[GRK_NUM_COMMENTS_SUPPORTED];
    grk_asoc asocs[GRK_NUM_ASOC_BOXES_SUPPORTED];
    uint32_t num_asocs;
} grk_header_info;

/* ---- decompression parameters (grok.h:716-830) */
typedef struct _grk_dparameters {
    uint8_t cp_reduce;
    uint16_t cp_layer;
    char infile[GRK_PATH_LEN];
    char outfile[GRK_PATH_LEN];
    GRK_SUPPORTED_FILE_FMT decod_format;
    GRK_SUPPORTED_FILE_FMT cod_format;
    uint32_t DA_x0, DA_x1, DA_y0, DA_y1;
    bool m_verbose;
    uint16_t tileIndex;
    uint32_t nb_tile_to_decompress;
    uint32_t flags;
    GRK_TILE_CACHE_STRATEGY tileCacheStrategy;
} grk_dparameters;
typedef struct _grk_prec { uint8_t prec; grk_precision_mode mode; } grk_precision;
typedef struct _grk_decompress_params {
    grk_dparameters core;
    char infile[GRK_PATH_LEN];
    char outfile[GRK_PATH_LEN];
    GRK_SUPPORTED_FILE_FMT decod_format;
    GRK_SUPPORTED_FILE_FMT cod_format;
    char indexfilename[GRK_PATH_LEN];
    uint32_t DA_x0, DA_x1, DA_y0, DA_y1;
    bool m_verbose;
    uint16_t tileIndex;
    uint32_t nb_tile_to_decompress;
    grk_precision* precision;
    uint32_t nb_precision;
    bool force_rgb;
    bool upsample;
    bool split_pnm;
    bool serialize_xml;
    uint32_t compression;
    uint32_t compressionLevel;
    int32_t deviceId;
    uint32_t duration;
    uint32_t kernelBuildOptions;
    uint32_t repeats;
    bool verbose;
    uint32_t numThreads;
} grk_decompress_parameters;

/* ---- streams (grok.h:836-851) */
typedef size_t (*grk_stream_read_fn)(void* buffer, size_t numBytes, void* user_data);
typedef size_t (*grk_stream_write_fn)(void* buffer, size_t numBytes, void* user_data);
typedef bool (*grk_stream_seek_fn)(uint64_t numBytes, void* user_data);
typedef void (*grk_stream_free_user_data_fn)(void* user_data);

/* ---- images (grok.h:895-973): component samples are int32 planes, row stride `stride` */
typedef struct _grk_image_comp {
    grk_object obj;
    uint32_t dx, dy;
    uint32_t w;
    uint32_t stride;
    uint32_t h;
    uint32_t x0, y0;
    uint16_t Xcrg, Ycrg;
    uint8_t prec;
    bool sgnd;
    int32_t* data;
    GRK_COMPONENT_TYPE type;
    GRK_COMPONENT_ASSOC association;
} grk_image_comp;
typedef struct _grk_image_meta {
    grk_object obj;
    grk_color color;
    uint8_t* iptc_buf;
    size_t iptc_len;
    uint8_t* xmp_buf;
    size_t xmp_len;
} grk_image_meta;
typedef struct _grk_image {
    grk_object obj;
    uint32_t x0, y0, x1, y1;
    uint16_t numcomps;
    GRK_COLOR_SPACE color_space;
    bool color_applied;
    bool has_capture_resolution;
    double capture_resolution[2];
    bool has_display_resolution;
    double display_resolution[2];
    grk_image_meta* meta;
    grk_image_comp* comps;
} grk_image;
typedef struct _grk_image_comptparm {
    uint32_t dx, dy;
    uint32_t w;
    uint32_t stride;
    uint32_t h;
    uint32_t x0, y0;
    uint8_t prec;
    bool sgnd;
} grk_image_cmptparm;

/* ---- plugin data (grok.h:995-1077): the code-block tree a compress/decompress plugin owns */
typedef struct _grk_plugin_pass {
    double distortionDecrease;
    size_t rate;
    size_t length;
} grk_plugin_pass;
typedef struct _grk_plugin_code_block {
    uint32_t x0, y0, x1, y1;
    unsigned int* contextStream;
    uint32_t numPix;
    uint8_t* compressedData;
    uint32_t compressedDataLength;
    uint8_t numBitPlanes;
    size_t numPasses;
    grk_plugin_pass passes[67];
    unsigned int sortedIndex;
} grk_plugin_code_block;
typedef struct _grk_plugin_precinct {
    uint64_t numBlocks;
    grk_plugin_code_block** blocks;
} grk_plugin_precinct;
typedef struct _grk_plugin_band {
    uint8_t orientation;
    uint64_t numPrecincts;
    grk_plugin_precinct** precincts;
    float stepsize;
} grk_plugin_band;
typedef struct _grk_plugin_resolution {
    size_t level;
    size_t numBands;
    grk_plugin_band** band;
} grk_plugin_resolution;
typedef struct grk_plugin_tile_component {
    size_t numResolutions;
    grk_plugin_resolution** resolutions;
} grk_plugin_tile_component;
#define GRK_DECODE_HEADER (1 << 0)
#define GRK_DECODE_T2 (1 << 1)
#define GRK_DECODE_T1 (1 << 2)
#define GRK_DECODE_POST_T1 (1 << 3)
#define GRK_PLUGIN_DECODE_CLEAN (1 << 4)
#define GRK_DECODE_ALL (GRK_PLUGIN_DECODE_CLEAN | GRK_DECODE_HEADER | GRK_DECODE_T2 | GRK_DECODE_T1 | GRK_DECODE_POST_T1)
typedef struct _grk_plugin_tile {
    uint32_t decompress_flags;
    size_t numComponents;
    grk_plugin_tile_component** tileComponents;
} grk_plugin_tile;

typedef struct _grk_plugin_load_info { const char* pluginPath; } grk_plugin_load_info;
typedef struct _grk_plugin_init_info { int32_t deviceId; bool verbose; } grk_plugin_init_info;
#define GRK_PLUGIN_STATE_NO_DEBUG 0x0
typedef struct grk_plugin_compress_user_callback_info {
    const char* input_file_name;
    bool outputFileNameIsRelative;
    const char* output_file_name;
    grk_cparameters* compressor_parameters;
    grk_image* image;
    grk_plugin_tile* tile;
    uint8_t* compressBuffer;
    size_t compressBufferLen;
    unsigned int error_code;
    bool transferExifTags;
} grk_plugin_compress_user_callback_info;
typedef bool (*GRK_PLUGIN_COMPRESS_USER_CALLBACK)(grk_plugin_compress_user_callback_info* info);
typedef int (*GROK_INIT_DECOMPRESSORS)(grk_header_info* header_info, grk_image* image);
typedef struct _grk_plugin_decompress_callback_info {
    size_t deviceId;
    GROK_INIT_DECOMPRESSORS init_decompressors_func;
    const char* input_file_name;
    const char* output_file_name;
    GRK_SUPPORTED_FILE_FMT decod_format;
    GRK_SUPPORTED_FILE_FMT cod_format;
    grk_stream* stream;
    grk_codec* codec;
    grk_header_info header_info;
    grk_decompress_parameters* decompressor_parameters;
    grk_image* image;
    bool plugin_owns_image;
    grk_plugin_tile* tile;
    unsigned int error_code;
    uint32_t decompress_flags;
    uint32_t full_image_x0;
    uint32_t full_image_y0;
    void* user_data;
} grk_plugin_decompress_callback_info;
typedef int32_t (*grk_plugin_decompress_callback)(grk_plugin_decompress_callback_info* info);

/* ---- entry points (grok.h:1082-1657), same names and signatures */
const char* grk_version(void);
bool grk_initialize(const char* pluginPath, uint32_t numthreads);
void grk_deinitialize(void);
void grk_object_ref(grk_object* obj);
void grk_object_unref(grk_object* obj);
bool grk_set_info_handler(grk_msg_callback p_callback, void* user_data);
bool grk_set_warning_handler(grk_msg_callback p_callback, void* user_data);
bool grk_set_error_handler(grk_msg_callback p_callback, void* user_data);
grk_image* grk_image_new(uint16_t numcmpts, grk_image_cmptparm* cmptparms, GRK_COLOR_SPACE clrspc, bool allocData);
grk_image_meta* grk_image_meta_new(void);
void grk_image_all_components_data_free(grk_image* image);
void grk_image_single_component_data_free(grk_image_comp* image);
grk_stream* grk_stream_new(size_t buffer_size, bool is_input);
void grk_stream_set_read_function(grk_stream* stream, grk_stream_read_fn p_function);
void grk_stream_set_write_function(grk_stream* stream, grk_stream_write_fn p_function);
void grk_stream_set_seek_function(grk_stream* stream, grk_stream_seek_fn p_function);
void grk_stream_set_user_data(grk_stream* stream, void* data, grk_stream_free_user_data_fn p_function);
void grk_stream_set_user_data_length(grk_stream* stream, uint64_t data_length);
grk_stream* grk_stream_create_file_stream(const char* fname, size_t buffer_size, bool is_read_stream);
grk_stream* grk_stream_create_mem_stream(uint8_t* buf, size_t buffer_len, bool ownsBuffer, bool is_read_stream);
size_t grk_stream_get_write_mem_stream_length(grk_stream* stream);
grk_stream* grk_stream_create_mapped_file_stream(const char* fname, bool read_stream);
grk_codec* grk_decompress_create(GRK_CODEC_FORMAT format, grk_stream* stream);
void grk_decompress_set_default_params(grk_dparameters* parameters);
bool grk_decompress_init(grk_codec* codec, grk_dparameters* parameters);
bool grk_decompress_read_header(grk_codec* codec, grk_header_info* header_info);
grk_image* grk_decompress_get_tile_image(grk_codec* codec, uint16_t tileIndex);
grk_image* grk_decompress_get_composited_image(grk_codec* codec);
bool grk_decompress_set_window(grk_codec* codec, uint32_t start_x, uint32_t start_y, uint32_t end_x, uint32_t end_y);
bool grk_decompress(grk_codec* p_decompressor, grk_plugin_tile* tile);
bool grk_decompress_tile(grk_codec* codec, uint16_t tileIndex);
bool grk_decompress_end(grk_codec* codec);
grk_codec* grk_compress_create(GRK_CODEC_FORMAT format, grk_stream* stream);
void grk_compress_set_default_params(grk_cparameters* parameters);
bool grk_compress_init(grk_codec* codec, grk_cparameters* parameters, grk_image* image);
bool grk_compress_start(grk_codec* codec);
bool grk_compress(grk_codec* codec);
bool grk_compress_tile(grk_codec* codec, uint16_t tileIndex, uint8_t* data, uint64_t data_size);
bool grk_compress_with_plugin(grk_codec* codec, grk_plugin_tile* tile);
bool grk_compress_end(grk_codec* codec);
void grk_dump_codec(grk_codec* codec, uint32_t info_flag, FILE* output_stream);
bool grk_set_MCT(grk_cparameters* parameters, float* pEncodingMatrix, int32_t* p_dc_shift, uint32_t pNbComp);
/* plugin management (grok.h:1470-1657): this library is the GPU path itself, so no
 * separate plugin is ever loaded — the calls report "not handled" and callers use the
 * regular entry points above (grk_compress.cpp:2281-2289 falls back the same way) */
bool grk_plugin_load(grk_plugin_load_info info);
void grk_plugin_cleanup(void);
uint32_t grk_plugin_get_debug_state(void);
bool grk_plugin_init(grk_plugin_init_info initInfo);
int32_t grk_plugin_compress(grk_cparameters* compress_parameters, GRK_PLUGIN_COMPRESS_USER_CALLBACK callback);
int32_t grk_plugin_batch_compress(const char* input_dir, const char* output_dir, grk_cparameters* compress_parameters,
                                  GRK_PLUGIN_COMPRESS_USER_CALLBACK callback);
bool grk_plugin_is_batch_complete(void);
void grk_plugin_stop_batch_compress(void);
int32_t grk_plugin_decompress(grk_decompress_parameters* decompress_parameters, grk_plugin_decompress_callback callback);
int32_t grk_plugin_init_batch_decompress(const char* input_dir, const char* output_dir,
                                         grk_decompress_parameters* decompress_parameters,
                                         grk_plugin_decompress_callback callback);
int32_t grk_plugin_batch_decompress(void);
void grk_plugin_stop_batch_decompress(void);

#ifdef __cplusplus
}
#endif
#endif /* GRK_ABI_H */
