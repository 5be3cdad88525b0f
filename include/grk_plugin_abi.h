/*
 * grk_plugin_abi.h — Grok 9.2.0's T1 plugin ABI, served by
 * grok_amd/libgrokj2k_plugin.so.
 *
 * Grok's loader (grok.cpp:579-605, plugin/minpf_plugin_manager.cpp:140-238) opens
 * <pluginPath>/libgrokj2k_plugin.so, calls minpf_post_load_plugin, then resolves the
 * plugin_* entry points below by name on every call.  The callback structs are the
 * plugin-side mirrors of plugin/plugin_interface.h (PluginDecodeCallbackInfo holds
 * std::string members, so this header is C++ and the library is built with the same
 * standard library as Grok).  Tree structs (grk_plugin_tile ... grk_plugin_code_block)
 * and parameters come from grk_abi.h (layout-identical to grok.h).
 */
#ifndef GRK_PLUGIN_ABI_H
#define GRK_PLUGIN_ABI_H

#include <stdint.h>

#include <string>

#include "grk_abi.h"

/* ---- minpf (plugin/minpf_plugin.h) */
struct minpf_platform_services;
typedef struct minpf_object_params {
    const char* id;
    const struct minpf_platform_services* platformServices;
} minpf_object_params;
typedef struct minpf_plugin_api_version { int32_t major; int32_t minor; } minpf_plugin_api_version;
typedef void* (*minpf_create_func)(minpf_object_params*);
typedef int32_t (*minpf_destroy_func)(void*);
typedef struct minpf_register_params {
    minpf_plugin_api_version version;
    minpf_create_func createFunc;
    minpf_destroy_func destroyFunc;
} minpf_register_params;
typedef int32_t (*minpf_register_func)(const char* nodeType, const minpf_register_params* params);
typedef int32_t (*minpf_invoke_service_func)(const char* serviceName, void* serviceParams);
typedef struct minpf_platform_services {
    minpf_plugin_api_version version;
    minpf_register_func registerObject;
    minpf_invoke_service_func invokeService;
} minpf_platform_services;
typedef int32_t (*minpf_exit_func)();

/* ---- compressor interface (plugin/plugin_interface.h) */
struct plugin_encode_user_callback_info {
    const char* input_file_name;
    bool outputFileNameIsRelative;
    const char* output_file_name;
    grk_cparameters* compressor_parameters;
    grk_image* image;
    grk_plugin_tile* tile;
    int32_t error_code;
};
typedef void (*PLUGIN_ENCODE_USER_CALLBACK)(plugin_encode_user_callback_info* info);

/* ---- decompressor interface (plugin/plugin_interface.h) */
struct PluginDecodeCallbackInfo {
    size_t deviceId = 0;
    GROK_INIT_DECOMPRESSORS init_decompressors_func = nullptr;
    std::string inputFile;
    std::string outputFile;
    GRK_SUPPORTED_FILE_FMT decod_format = GRK_UNK_FMT;   /* input file format */
    GRK_SUPPORTED_FILE_FMT cod_format = GRK_UNK_FMT;     /* output file format */
    grk_stream* stream = nullptr;
    grk_codec* codec = nullptr;
    grk_decompress_parameters* decompressor_parameters = nullptr;
    grk_header_info header_info{};
    grk_image* image = nullptr;
    bool plugin_owns_image = false;
    grk_plugin_tile* tile = nullptr;
    int32_t error_code = 0;
    uint32_t decompress_flags = 0;
    void* user_data = nullptr;
};
typedef int32_t (*PLUGIN_DECODE_USER_CALLBACK)(PluginDecodeCallbackInfo* info);

/* ---- exports (resolved by name: grok.cpp:550-567, plugin_bridge.cpp:299-300) */
extern "C" {
minpf_exit_func minpf_post_load_plugin(const char* pluginPath, const minpf_platform_services* services);
bool plugin_init(grk_plugin_init_info initInfo);
uint32_t plugin_get_debug_state(void);
int32_t plugin_encode(grk_cparameters* encoding_parameters, PLUGIN_ENCODE_USER_CALLBACK callback);
int32_t plugin_batch_encode(const char* input_dir, const char* output_dir, grk_cparameters* encoding_parameters,
                            PLUGIN_ENCODE_USER_CALLBACK userCallback);
bool plugin_is_batch_complete(void);
void plugin_stop_batch_encode(void);
int32_t plugin_decompress(grk_decompress_parameters* decoding_parameters, PLUGIN_DECODE_USER_CALLBACK userCallback);
int32_t plugin_init_batch_decompress(const char* input_dir, const char* output_dir,
                                     grk_decompress_parameters* decoding_parameters,
                                     PLUGIN_DECODE_USER_CALLBACK userCallback);
int32_t plugin_batch_decompress(void);
void plugin_stop_batch_decompress(void);
}

#endif /* GRK_PLUGIN_ABI_H */
