/*
 * mcm_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline).
 *
 * Scalar C restatement of VPT's spectral MCM march
 * (src/wgsl/renderers/MCMSpectralComputeRenderer.wgsl and its mixins).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product (libvptmcm.so) never links or calls it.
 */
#ifndef MCM_ORACLE_H
#define MCM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The render UBO (wgsl:8-18); the reset UBO (wgsl:187-192) is its prefix. */
typedef struct orc_uniforms {
    float mvp_inverse[16];  /* column-major */
    float inv_res[2];
    uint32_t seed_bits;     /* bitcast<u32>(randSeed) */
    float blur;
    float extinction;
    float anisotropy;       /* unused by the kernel (as in the reference) */
    uint32_t max_bounces;
    uint32_t steps;
    float light_dir[3];
} orc_uniforms;

/* struct PhotonSpectral, wgsl:238-247: 136 bytes of fields, padded to the
 * 16-byte struct alignment (vec3f) => 144-byte array stride (js:131). */
typedef struct orc_photon {
    float position[3];
    uint32_t bounces;
    float direction[3];
    uint32_t samples;
    uint32_t bin;
    float wavelength;
    float radiance[12];
    float transmittance[12];
    uint32_t _pad[2];
} orc_photon;

/* Full reset kernel over the R x R photon buffer (wgsl:213-231). */
void orc_reset(uint32_t R, const orc_uniforms* u, const float* spectrum /*64*/,
               orc_photon* photons, int nthreads);

/* Render pass (wgsl:107-179). rgb32 (R*R*3, may be NULL) receives the f32
 * radiance_to_rgb result, rgba16 (R*R*4, may be NULL) the rgba16float store.
 * Rows [y0, y1) only (y1 = 0 means all rows). */
void orc_render(uint32_t R, const orc_uniforms* u, const float* spectrum,
                const uint8_t* volume, uint32_t W, uint32_t H, uint32_t D,
                const uint8_t* tf /*256*256*4*/, const uint8_t* light /*256*/,
                orc_photon* photons, float* rgb32, uint16_t* rgba16, int nthreads,
                uint32_t y0, uint32_t y1);

/* ---- RGB sibling renderer (MCMComputeRenderer.wgsl, 'mcm-compute') ------ */

/* struct Photon (src/wgsl/mixins/Photon.wgsl): 64-byte stride. */
typedef struct orc_photon_rgb {
    float position[3];
    uint32_t bounces;
    float direction[3];
    uint32_t samples;
    float transmittance[3];
    uint32_t _pad0;
    float radiance[3];
    uint32_t _pad1;
} orc_photon_rgb;

/* sRGB -> linear decode of an rgba8unorm-srgb texel channel (the sampler
 * decodes before filtering): byte/255 <= 0.04045 ? v/12.92 :
 * ((v+0.055)/1.055)^2.4, in double, rounded to f32. */
float orc_srgb_to_linear(uint8_t b);

/* reset compute_main (MCMComputeRenderer.wgsl reset part) / render
 * compute_main (render part). The transfer function is the rgba8unorm-srgb
 * texture (tf_w x tf_h, row-major) of setTransferFunction; the environment is
 * the 1x1 rgba8unorm texel the rendering context creates. */
void orc_reset_rgb(uint32_t R, const orc_uniforms* u, orc_photon_rgb* photons, int nthreads);
void orc_render_rgb(uint32_t R, const orc_uniforms* u, const uint8_t* volume, uint32_t W,
                    uint32_t H, uint32_t D, const uint8_t* tf, uint32_t tf_w, uint32_t tf_h,
                    const uint8_t env[4], orc_photon_rgb* photons, uint16_t* rgba16, int nthreads);

/* Artistic tone mapper (ArtisticToneMapper.wgsl:38-48) over n rgba16float
 * pixels -> rgba8 (alpha 255), evaluated in double precision: the checker of
 * the device's f32 version (tolerance test, see tests/test_gpu_tonemap.py).
 * params = {low, mid, high, saturation, gamma}. */
void orc_tonemap_artistic(const uint16_t* rgba16, uint32_t n, const float params[5],
                          uint8_t* out);

/* Primitives, exported for known-answer and device-parity tests. */
uint32_t orc_hash(uint32_t v);
uint32_t orc_hash3(uint32_t x, uint32_t y, uint32_t z);
float orc_log(float x);
float orc_sin(float x);
float orc_cos(float x);
uint16_t orc_f2h(float f);
float orc_sample_volume(const uint8_t* vol, uint32_t W, uint32_t H, uint32_t D,
                        const float p[3]);
void orc_sample_tf(const uint8_t* tf, float t, float d, float out[3]);
float orc_sample_light(const uint8_t* light, float t);
void orc_eval_batch(int fn, const uint32_t* in, uint32_t* out, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
