/*
 * vptmcm_napi.c — Node N-API shim over the C-ABI (include/vptmcm.h).
 *
 * The product's host is JavaScript, as in the reference (the renderer class
 * js/MCMSpectralComputeRenderer.js mirrors WebGPUMCMSpectralComputeRenderer).
 * This shim is the only bridge: one JS function per C entry point, typed
 * arrays passed as plain pointers + sizes, negative return codes turned into a
 * thrown JS Error carrying `.code` and vptmcm_last_error()'s message (the
 * reference throws synchronously too, e.g. WebGPURendererFactory.js:25).
 * N-API version 8 (Node 12.22); built with plain gcc, no node-gyp.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vptmcm.h"

typedef struct {
    vptmcm* h;
    uint32_t photon_bytes; /* 144 spectral, 64 RGB */
    uint32_t R;            /* the handle's resolution: every output array is sized from it */
} handle_box;

#define NAPI_OK(env, call)                                                   \
    do {                                                                     \
        if ((call) != napi_ok) {                                             \
            const napi_extended_error_info* _ei = NULL;                      \
            napi_get_last_error_info((env), &_ei);                           \
            napi_throw_error((env), "VPTMCM_NAPI",                           \
                             _ei && _ei->error_message ? _ei->error_message  \
                                                       : "N-API call failed"); \
            return NULL;                                                     \
        }                                                                    \
    } while (0)

static napi_value throw_code(napi_env env, int code, const char* msg) {
    char cbuf[16];
    snprintf(cbuf, sizeof cbuf, "%d", code);
    napi_value err, m, c;
    napi_create_string_utf8(env, msg && *msg ? msg : "vptmcm error", NAPI_AUTO_LENGTH, &m);
    napi_create_string_utf8(env, cbuf, NAPI_AUTO_LENGTH, &c);
    napi_create_error(env, c, m, &err);
    napi_value ncode;
    napi_create_int32(env, code, &ncode);
    napi_set_named_property(env, err, "vptmcmCode", ncode);
    napi_throw(env, err);
    return NULL;
}

static napi_value check(napi_env env, vptmcm* h, int rc) {
    if (rc == VPTMCM_OK) {
        napi_value u;
        napi_get_undefined(env, &u);
        return u;
    }
    return throw_code(env, rc, vptmcm_last_error(h));
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return -1;
    if (argc < want) {
        napi_throw_type_error(env, NULL, "too few arguments");
        return -1;
    }
    return 0;
}

static handle_box* get_box(napi_env env, napi_value v) {
    handle_box* box = NULL;
    if (napi_get_value_external(env, v, (void**)&box) != napi_ok || !box || !box->h) {
        napi_throw_error(env, "VPTMCM_HANDLE", "invalid or destroyed renderer handle");
        return NULL;
    }
    return box;
}

static vptmcm* get_handle(napi_env env, napi_value v) {
    handle_box* box = get_box(env, v);
    return box ? box->h : NULL;
}

/* typed array -> pointer + element count (+ element size check) */
static void* get_typed(napi_env env, napi_value v, size_t elem, size_t min_count, size_t* count) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) {
        napi_throw_type_error(env, NULL, "expected a typed array");
        return NULL;
    }
    napi_typedarray_type type;
    size_t length, offset;
    void* data;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &length, &data, &ab, &offset) != napi_ok) {
        napi_throw_error(env, NULL, "typed array info failed");
        return NULL;
    }
    size_t esz = 1;
    switch (type) {
        case napi_int8_array: case napi_uint8_array: case napi_uint8_clamped_array: esz = 1; break;
        case napi_int16_array: case napi_uint16_array: esz = 2; break;
        case napi_int32_array: case napi_uint32_array: case napi_float32_array: esz = 4; break;
        default: esz = 8; break;
    }
    if (esz != elem) {
        napi_throw_type_error(env, NULL, "typed array has the wrong element size");
        return NULL;
    }
    if (length < min_count) {
        char msg[96];
        snprintf(msg, sizeof msg, "typed array too short: %zu < %zu", length, min_count);
        napi_throw_range_error(env, NULL, msg);
        return NULL;
    }
    if (count) *count = length;
    return data;
}

static uint32_t get_u32(napi_env env, napi_value v);

/* An output array of per_pixel elements per pixel of the handle's R x R
 * frame. The caller's R must be the handle's: the library writes R*R*per_pixel
 * elements whatever the caller believes. */
static void* get_frame_out(napi_env env, handle_box* box, napi_value arr, napi_value r,
                           size_t elem, size_t per_pixel) {
    if (get_u32(env, r) != box->R) {
        char msg[96];
        snprintf(msg, sizeof msg, "resolution %u does not match the renderer's %u", get_u32(env, r),
                 box->R);
        napi_throw_range_error(env, NULL, msg);
        return NULL;
    }
    return get_typed(env, arr, elem, (size_t)box->R * box->R * per_pixel, NULL);
}

static uint32_t get_u32(napi_env env, napi_value v) {
    uint32_t x = 0;
    napi_get_value_uint32(env, v, &x);
    return x;
}
static double get_f64(napi_env env, napi_value v) {
    double x = 0;
    napi_get_value_double(env, v, &x);
    return x;
}

static void finalize_box(napi_env env, void* data, void* hint) {
    (void)env; (void)hint;
    handle_box* box = (handle_box*)data;
    if (box && box->h) vptmcm_destroy(box->h);
    free(box);
}

/* create(resolution, device, layout[, renderer[, devices[, transport]]]) -> handle;
 * devices: an array of device ordinals (vptmcm_config::n_devices, one
 * photon-parallel replica per entry, composited on devices[0]) */
static napi_value js_create(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    vptmcm_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.resolution = get_u32(env, argv[0]);
    cfg.max_bins = VPTMCM_MAX_BINS;
    int32_t dev = -1;
    napi_get_value_int32(env, argv[1], &dev);
    cfg.device = dev;
    cfg.volume_layout = get_u32(env, argv[2]);
    cfg.renderer = VPTMCM_RENDERER_SPECTRAL;
    {   /* optional: renderer kind, device list, group transport */
        size_t argc = 6;
        napi_value all[6];
        if (napi_get_cb_info(env, info, &argc, all, NULL, NULL) == napi_ok) {
            napi_valuetype t;
            if (argc >= 4 && napi_typeof(env, all[3], &t) == napi_ok && t == napi_number)
                cfg.renderer = get_u32(env, all[3]);
            bool is_arr = false;
            if (argc >= 5 && napi_is_array(env, all[4], &is_arr) == napi_ok && is_arr) {
                uint32_t n = 0;
                napi_get_array_length(env, all[4], &n);
                if (n < 1 || n > VPTMCM_MAX_DEVICES) {
                    napi_throw_range_error(env, NULL, "devices: 1 to VPTMCM_MAX_DEVICES (8) ordinals");
                    return NULL;
                }
                for (uint32_t k = 0; k < n; k++) {
                    napi_value e;
                    int32_t d = -1;
                    napi_get_element(env, all[4], k, &e);
                    if (napi_get_value_int32(env, e, &d) != napi_ok) {
                        napi_throw_type_error(env, NULL, "devices: expected integer ordinals");
                        return NULL;
                    }
                    cfg.devices[k] = d;
                }
                cfg.n_devices = n;
            }
            if (argc >= 6 && napi_typeof(env, all[5], &t) == napi_ok && t == napi_number)
                cfg.group_transport = get_u32(env, all[5]);
        }
    }
    vptmcm* h = NULL;
    int rc = vptmcm_create(&cfg, &h);
    if (rc) return throw_code(env, rc, vptmcm_last_error(NULL));
    handle_box* box = (handle_box*)malloc(sizeof *box);
    box->h = h;
    box->R = cfg.resolution;
    box->photon_bytes = cfg.renderer == VPTMCM_RENDERER_RGB ? VPTMCM_PHOTON_RGB_BYTES : VPTMCM_PHOTON_BYTES;
    napi_value ext;
    NAPI_OK(env, napi_create_external(env, box, finalize_box, NULL, &ext));
    return ext;
}

static napi_value js_destroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    handle_box* box = NULL;
    napi_get_value_external(env, argv[0], (void**)&box);
    if (box && box->h) {
        vptmcm_destroy(box->h);
        box->h = NULL;
    }
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

/* setVolume(h, Uint8Array, w, h, d) */
static napi_value js_set_volume(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (get_args(env, info, 5, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    uint32_t w = get_u32(env, argv[2]), hh = get_u32(env, argv[3]), d = get_u32(env, argv[4]);
    const uint8_t* p = get_typed(env, argv[1], 1, (size_t)w * hh * d, NULL);
    if (!p) return NULL;
    return check(env, h, vptmcm_set_volume(h, p, w, hh, d));
}

static napi_value js_volume_begin(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (get_args(env, info, 4, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_volume_begin(h, get_u32(env, argv[1]), get_u32(env, argv[2]),
                                             get_u32(env, argv[3])));
}

/* volumeWriteBlock(h, Uint8Array, x, y, z, w, h, d) */
static napi_value js_volume_write_block(napi_env env, napi_callback_info info) {
    napi_value argv[8];
    if (get_args(env, info, 8, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    uint32_t v[6];
    for (int k = 0; k < 6; k++) v[k] = get_u32(env, argv[2 + k]);
    const uint8_t* p = get_typed(env, argv[1], 1, (size_t)v[3] * v[4] * v[5], NULL);
    if (!p) return NULL;
    return check(env, h, vptmcm_volume_write_block(h, p, v[0], v[1], v[2], v[3], v[4], v[5]));
}

static napi_value js_volume_end(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_volume_end(h));
}

static napi_value js_set_material_tf(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (get_args(env, info, 2, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const uint8_t* p = get_typed(env, argv[1], 1, VPTMCM_TF_BYTES, NULL);
    if (!p) return NULL;
    return check(env, h, vptmcm_set_material_tf(h, p));
}

/* setLight(h, Uint8Array(256), Float32Array(3)) */
static napi_value js_set_light(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const uint8_t* spd = get_typed(env, argv[1], 1, VPTMCM_LIGHT_BYTES, NULL);
    if (!spd) return NULL;
    const float* dir = get_typed(env, argv[2], 4, 3, NULL);
    if (!dir) return NULL;
    return check(env, h, vptmcm_set_light(h, spd, dir));
}

static napi_value js_set_spectrum(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (get_args(env, info, 2, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const float* p = get_typed(env, argv[1], 4, VPTMCM_SPECTRUM_FLOATS, NULL);
    if (!p) return NULL;
    return check(env, h, vptmcm_set_spectrum(h, p));
}

/* setParams(h, extinction, anisotropy, bounces, steps, blur) */
static napi_value js_set_params(napi_env env, napi_callback_info info) {
    napi_value argv[6];
    if (get_args(env, info, 6, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    vptmcm_params p;
    p.extinction = (float)get_f64(env, argv[1]);  /* Float32Array([...]) rounding, js:296 */
    p.anisotropy = (float)get_f64(env, argv[2]);
    p.max_bounces = get_u32(env, argv[3]);           /* Uint32Array([...]), js:303 */
    p.steps = get_u32(env, argv[4]);
    p.blur = (float)get_f64(env, argv[5]);
    return check(env, h, vptmcm_set_params(h, &p));
}

static napi_value march_call(napi_env env, napi_callback_info info, int is_reset) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const float* m = get_typed(env, argv[1], 4, 16, NULL);
    if (!m) return NULL;
    uint32_t seed = get_u32(env, argv[2]);
    return check(env, h, is_reset ? vptmcm_reset(h, m, seed) : vptmcm_render(h, m, seed));
}
static napi_value js_reset(napi_env env, napi_callback_info info) { return march_call(env, info, 1); }
static napi_value js_render(napi_env env, napi_callback_info info) { return march_call(env, info, 0); }

/* renderPasses(h, Float32Array(16), Uint32Array seeds) */
static napi_value js_render_passes(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const float* m = get_typed(env, argv[1], 4, 16, NULL);
    if (!m) return NULL;
    size_t n = 0;
    const uint32_t* s = get_typed(env, argv[2], 4, 0, &n);
    if (!s) return NULL;
    return check(env, h, vptmcm_render_passes(h, m, s, (uint32_t)n));
}

static napi_value js_synchronize(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_synchronize(h));
}

/* readRGBA16F(h, Uint16Array(R*R*4), R) */
static napi_value js_read_rgba16f(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    uint16_t* p = get_frame_out(env, box, argv[1], argv[2], 2, 4);
    if (!p) return NULL;
    return check(env, box->h, vptmcm_read_rgba16f(box->h, p));
}

/* readRGB(h, Float32Array(R*R*3), R): the last pass's fp32 radiance_to_rgb
 * image before the f16 store (wgsl:304-326; vptmcm_read_rgb) */
static napi_value js_read_rgb(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    float* p = get_frame_out(env, box, argv[1], argv[2], 4, 3);
    if (!p) return NULL;
    return check(env, box->h, vptmcm_read_rgb(box->h, p));
}

/* setTransferFunction(h, Uint8Array(w*h*4), w, h) / setEnvironment(h, Uint8Array(4), 1, 1) */
static napi_value image_call(napi_env env, napi_callback_info info, int env_map) {
    napi_value argv[4];
    if (get_args(env, info, 4, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    uint32_t w = get_u32(env, argv[2]), hh = get_u32(env, argv[3]);
    const uint8_t* p = get_typed(env, argv[1], 1, (size_t)w * hh * 4, NULL);
    if (!p) return NULL;
    return check(env, h, env_map ? vptmcm_set_environment(h, p, w, hh)
                                 : vptmcm_set_transfer_function(h, p, w, hh));
}
static napi_value js_set_transfer_function(napi_env env, napi_callback_info info) { return image_call(env, info, 0); }
static napi_value js_set_environment(napi_env env, napi_callback_info info) { return image_call(env, info, 1); }

/* tonemapArtistic(h, Float32Array[low, mid, high, saturation, gamma], Uint8Array(R*R*4), R) */
static napi_value js_tonemap_artistic(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (get_args(env, info, 4, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    const float* params = get_typed(env, argv[1], 4, 5, NULL);
    if (!params) return NULL;
    uint8_t* out = get_frame_out(env, box, argv[2], argv[3], 1, 4);
    if (!out) return NULL;
    return check(env, box->h, vptmcm_tonemap_artistic(box->h, params, out));
}

/* readPhotons(h, Uint8Array(R*R*stride), R) / writePhotons(h, Uint8Array, R);
 * stride = 144 (spectral) or 64 (RGB), from the handle's renderer kind */
static napi_value photons_call(napi_env env, napi_callback_info info, int write) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    uint8_t* p = get_frame_out(env, box, argv[1], argv[2], 1, box->photon_bytes);
    if (!p) return NULL;
    return check(env, box->h, write ? vptmcm_write_photons(box->h, p) : vptmcm_read_photons(box->h, p));
}
static napi_value js_read_photons(napi_env env, napi_callback_info info) { return photons_call(env, info, 0); }
static napi_value js_write_photons(napi_env env, napi_callback_info info) { return photons_call(env, info, 1); }

static napi_value js_enable_kernel_timing(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (get_args(env, info, 2, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    bool on = false;
    napi_get_value_bool(env, argv[1], &on);
    return check(env, h, vptmcm_enable_kernel_timing(h, on ? 1 : 0));
}

/* setMacroSkip(h, mode): 0 off, 1 on, 2 auto (vptmcm_set_macro_skip) */
static napi_value js_set_macro_skip(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (get_args(env, info, 2, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    int32_t mode = 0;
    if (napi_get_value_int32(env, argv[1], &mode) != napi_ok) {
        napi_throw_type_error(env, NULL, "mode must be 0, 1 or 2");
        return NULL;
    }
    return check(env, h, vptmcm_set_macro_skip(h, mode));
}

/* kernelTime(h) -> { ms, launches } */
static napi_value js_kernel_time(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    double ms = 0;
    uint64_t n = 0;
    int rc = vptmcm_kernel_time(h, &ms, &n);
    if (rc) return throw_code(env, rc, vptmcm_last_error(h));
    napi_value o, vms, vn;
    napi_create_object(env, &o);
    napi_create_double(env, ms, &vms);
    napi_create_double(env, (double)n, &vn);
    napi_set_named_property(env, o, "ms", vms);
    napi_set_named_property(env, o, "launches", vn);
    return o;
}

static napi_value js_comm_unique_id(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value ab, arr;
    void* data = NULL;
    NAPI_OK(env, napi_create_arraybuffer(env, VPTMCM_UNIQUE_ID_BYTES, &data, &ab));
    int rc = vptmcm_comm_unique_id((uint8_t*)data);
    if (rc) return throw_code(env, rc, vptmcm_last_error(NULL));
    NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, VPTMCM_UNIQUE_ID_BYTES, ab, 0, &arr));
    return arr;
}

/* commInit(h, Uint8Array(128), nranks, rank) */
static napi_value js_comm_init(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (get_args(env, info, 4, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    const uint8_t* uid = get_typed(env, argv[1], 1, VPTMCM_UNIQUE_ID_BYTES, NULL);
    if (!uid) return NULL;
    return check(env, h, vptmcm_comm_init(h, uid, (int)get_u32(env, argv[2]),
                                          (int)get_u32(env, argv[3])));
}

/* commAllreduceRadiance(h[, inline[, sharded]]): inline = true runs the
 * all-reduce on the march stream (VPTMCM_ALLREDUCE_INLINE, for a composite
 * about to be shown); sharded = true reduce-scatters (VPTMCM_ALLREDUCE_SHARDED:
 * the next commReadComposite is collective) */
static napi_value js_comm_allreduce_radiance(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    size_t argc = 3;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
    if (argc < 1) {
        napi_throw_type_error(env, NULL, "too few arguments");
        return NULL;
    }
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    bool inl = false;
    if (argc > 1 && napi_get_value_bool(env, argv[1], &inl) != napi_ok) {
        napi_throw_type_error(env, NULL, "inline must be a boolean");
        return NULL;
    }
    bool shd = false;
    if (argc > 2 && napi_get_value_bool(env, argv[2], &shd) != napi_ok) {
        napi_throw_type_error(env, NULL, "sharded must be a boolean");
        return NULL;
    }
    return check(env, h, vptmcm_comm_allreduce_radiance_ex(
                             h, (inl ? VPTMCM_ALLREDUCE_INLINE : 0u) | (shd ? VPTMCM_ALLREDUCE_SHARDED : 0u)));
}

/* commReadComposite(h, Float32Array(R*R*3), R) */
static napi_value js_comm_read_composite(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    float* rgb = get_frame_out(env, box, argv[1], argv[2], 4, 3);
    if (!rgb) return NULL;
    return check(env, box->h, vptmcm_comm_read_composite(box->h, rgb, NULL));
}

/* setBand(h, y0, y1): Mode B row band (multiples of 8; y1 may be R) */
static napi_value js_set_band(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_set_band(h, get_u32(env, argv[1]), get_u32(env, argv[2])));
}

/* commGatherBands(h, Float32Array(R*R*3), R): every rank's band, composited */
static napi_value js_comm_gather_bands(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (get_args(env, info, 3, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    float* rgb = get_frame_out(env, box, argv[1], argv[2], 4, 3);
    if (!rgb) return NULL;
    return check(env, box->h, vptmcm_comm_gather_bands(box->h, rgb));
}

static napi_value js_comm_barrier(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_comm_barrier(h));
}

/* lastLaunch(h) -> { mode, tpl, spec, passes, macro, launches } (vptmcm_debug_last_launch) */
static napi_value js_last_launch(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    uint32_t v[4];
    uint64_t n = 0;
    int rc = vptmcm_debug_last_launch(h, v, &n);
    if (rc) return throw_code(env, rc, vptmcm_last_error(h));
    static const char* names[5] = {"mode", "tpl", "spec", "passes", "macro"};
    const uint32_t w[5] = {v[0], v[1], v[2] & 1u, v[3], (v[2] >> 1) & 1u};
    napi_value o, x;
    napi_create_object(env, &o);
    for (int k = 0; k < 5; k++) {
        napi_create_uint32(env, w[k], &x);
        napi_set_named_property(env, o, names[k], x);
    }
    napi_create_double(env, (double)n, &x);
    napi_set_named_property(env, o, "launches", x);
    return o;
}

/* composite(h): enqueue the replicas' composite of the current frame */
static napi_value js_composite(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    return check(env, h, vptmcm_composite(h));
}

/* readComposite(h, Uint16Array(R*R*4) | null, Float32Array(R*R*3) | null, R) */
static napi_value js_read_composite(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (get_args(env, info, 4, argv)) return NULL;
    handle_box* box = get_box(env, argv[0]);
    if (!box) return NULL;
    napi_valuetype t1, t2;
    napi_typeof(env, argv[1], &t1);
    napi_typeof(env, argv[2], &t2);
    uint16_t* q = NULL;
    float* rgb = NULL;
    if (t1 != napi_null && t1 != napi_undefined && !(q = get_frame_out(env, box, argv[1], argv[3], 2, 4)))
        return NULL;
    if (t2 != napi_null && t2 != napi_undefined && !(rgb = get_frame_out(env, box, argv[2], argv[3], 4, 3)))
        return NULL;
    return check(env, box->h, vptmcm_read_composite(box->h, q, rgb, NULL));
}

/* groupDevices(h) -> [ordinals] */
static napi_value js_group_devices(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (get_args(env, info, 1, argv)) return NULL;
    vptmcm* h = get_handle(env, argv[0]);
    if (!h) return NULL;
    int32_t d[VPTMCM_MAX_DEVICES];
    uint32_t n = 0;
    int rc = vptmcm_group_devices(h, d, &n);
    if (rc) return throw_code(env, rc, vptmcm_last_error(h));
    napi_value arr, x;
    napi_create_array_with_length(env, n, &arr);
    for (uint32_t k = 0; k < n; k++) {
        napi_create_int32(env, d[k], &x);
        napi_set_element(env, arr, k, x);
    }
    return arr;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value s;
    napi_create_string_utf8(env, vptmcm_version(), NAPI_AUTO_LENGTH, &s);
    return s;
}

#define EXPORT(name, fn)                                                          \
    do {                                                                          \
        napi_value f;                                                             \
        if (napi_create_function(env, name, NAPI_AUTO_LENGTH, fn, NULL, &f) != napi_ok) \
            return NULL;                                                          \
        napi_set_named_property(env, exports, name, f);                           \
    } while (0)

static napi_value init(napi_env env, napi_value exports) {
    EXPORT("create", js_create);
    EXPORT("destroy", js_destroy);
    EXPORT("setVolume", js_set_volume);
    EXPORT("volumeBegin", js_volume_begin);
    EXPORT("volumeWriteBlock", js_volume_write_block);
    EXPORT("volumeEnd", js_volume_end);
    EXPORT("setMaterialTF", js_set_material_tf);
    EXPORT("setLight", js_set_light);
    EXPORT("setSpectrum", js_set_spectrum);
    EXPORT("setParams", js_set_params);
    EXPORT("reset", js_reset);
    EXPORT("render", js_render);
    EXPORT("renderPasses", js_render_passes);
    EXPORT("synchronize", js_synchronize);
    EXPORT("readRGBA16F", js_read_rgba16f);
    EXPORT("readRGB", js_read_rgb);
    EXPORT("readPhotons", js_read_photons);
    EXPORT("tonemapArtistic", js_tonemap_artistic);
    EXPORT("setTransferFunction", js_set_transfer_function);
    EXPORT("setEnvironment", js_set_environment);
    EXPORT("writePhotons", js_write_photons);
    EXPORT("enableKernelTiming", js_enable_kernel_timing);
    EXPORT("kernelTime", js_kernel_time);
    EXPORT("commUniqueId", js_comm_unique_id);
    EXPORT("commInit", js_comm_init);
    EXPORT("commAllreduceRadiance", js_comm_allreduce_radiance);
    EXPORT("commReadComposite", js_comm_read_composite);
    EXPORT("commBarrier", js_comm_barrier);
    EXPORT("setBand", js_set_band);
    EXPORT("commGatherBands", js_comm_gather_bands);
    EXPORT("lastLaunch", js_last_launch);
    EXPORT("setMacroSkip", js_set_macro_skip);
    EXPORT("composite", js_composite);
    EXPORT("readComposite", js_read_composite);
    EXPORT("groupDevices", js_group_devices);
    EXPORT("version", js_version);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
