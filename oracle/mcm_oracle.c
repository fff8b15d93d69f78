/*
 * mcm_oracle.c — TEST INFRASTRUCTURE ONLY: the parity oracle and the CPU
 * baseline of the spectral MCM march. It is never linked into the product.
 *
 * What it is: a line-by-line scalar C restatement of the reference's hot path,
 *   src/wgsl/renderers/MCMSpectralComputeRenderer.wgsl  (render :107-179,
 *     reset :213-231, PhotonSpectral mixin :234-326)
 *   src/wgsl/mixins/random/hash/pcg.wgsl:3-7, squashlinear.wgsl:7-9,
 *   random/distribution/{uniformdivision,exponential,disk,square,sphere}.wgsl,
 *   src/wgsl/mixins/{unprojectRand,intersectCube,constants}.wgsl
 * Every function cites the WGSL lines it follows.
 *
 * What the WGSL leaves undefined, and how it is fixed here (the same choices
 * are made by the HIP kernels; DESIGN.md "Arithmetic specification"):
 *   - log/sin/cos: WGSL allows 3 ULP / 2^-11 abs error. Here they are
 *     defined as explicit f32 polynomials built only from +,-,*,/ (below),
 *     so CPU and GPU agree to the bit.
 *   - FMA: WGSL lets implementations fuse a*b + c. Here exactly the
 *     products listed in DESIGN.md ("Arithmetic specification") are fused,
 *     written as explicit fmaf() calls (correctly rounded in glibc); nothing
 *     else is contracted (-ffp-contract=off). Everything else is evaluated
 *     left to right as written in the WGSL.
 *   - division: WGSL's f32 `/` is only 2.5-ULP accurate; here a / b is
 *     defined as a * rcp(b) with rcp(b) = RN(1/b), the correctly rounded
 *     reciprocal (<= 1.5 ULP), one reciprocal per divisor value.
 *   - min/max: IEEE minNum/maxNum written with explicit compares; ties keep
 *     the first operand.
 *   - normalize(v) = v / sqrt(dot(v,v)); length = sqrt(dot);
 *     dot = fma(z, z', fma(y, y', x*x')).
 *   - mat4 * vec4 = fma(c3, v.w, fma(c2, v.z, fma(c1, v.y, c0*v.x))).
 *   - sampler (linear, clamp-to-edge; WebGPUVolume.js:61-64,
 *     WebGPUMCMSpectralComputeRenderer.js:150-169): per axis
 *     x = fma(clampc(u), N, -0.5), i0 = floor(x), f = x - i0, indices clamped to
 *     [0,N-1]; lerp(a,b,f) = fma(f, b-a, a) on the raw byte values, x then y
 *     then z; result * f32(1/255). clampc maps NaN to -1 and limits u to
 *     [-1,2] (outside [0,1] only the clamped edge texel is ever read).
 *   - f32 -> f16 for the rgba16float store: round to nearest even.
 *   - pixel (x,y) owns photon y*R + x (the reference's padded-width index
 *     at wgsl:112-113 equals this whenever R % 8 == 0, e.g. R = 64, 512).
 *
 * Parity pinning: the reference publishes no tests or fixtures.
 * The tables this oracle consumes (spectrum buffer from Spectrum.js +
 * compute_spectral_coefficients, mvpInverse from gl-matrix) are golden
 * fixtures produced by running the reference's own JS here
 * (tests/golden/make_golden.js). The march itself cannot be run from the
 * reference (WGSL, no WebGPU runtime here or on the GPU box); it is pinned
 * by the hand-computed known answers in tests/test_oracle.py. See DESIGN.md.
 */
#include "mcm_oracle.h"

#include <math.h>
#include <pthread.h>
#include <string.h>

#define MAX_N_BINS 12 /* wgsl:236 */
_Static_assert(sizeof(orc_photon) == 144, "PhotonSpectral stride");
#define EPS 1e-5f     /* wgsl:6 */
#define TWOPI 6.2831854820251465f /* constants.wgsl:4, 6.28318530718 as f32 */

typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;

/* correctly rounded reciprocal: the only true division of the spec */
static inline float rcp(float x) { return 1.0f / x; }

/* ORC_ALT (liboracle_alt.so, tests/test_statistical_parity.py only): a second,
 * equally legal WGSL arithmetic — libm logf/sinf/cosf, true division, no fused
 * products — whose converged image must agree statistically with the spec's. */
#ifdef ORC_ALT
#define DIVF(a, b) ((a) / (b))
#define fmaf(a, b, c) ((a) * (b) + (c))
#else
#define DIVF(a, b) ((a) * rcp(b)) /* WGSL a / b := a * RN(1/b) */
#endif

static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ---------------------------------------------------------------- spec math */

/* IEEE minNum / maxNum with explicit compares. */
static inline float smin(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return b < a ? b : a;
}
static inline float smax(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return b > a ? b : a;
}

/* log(x): reduce x = 2^e * m, m in [sqrt(1/2), sqrt(2)), s = f/(2+f) with
 * f = m-1, log(m) = 2 atanh(s) = 2s + s*z*(2/3 + z*(2/5 + ...)), z = s*s. */
float orc_log(float x) {
#ifdef ORC_ALT
    return logf(x);
#endif
    uint32_t b = fbits(x);
    if (x != x || (b >> 31)) return (x == 0.0f) ? -INFINITY : NAN; /* -0 -> -inf */
    if (x == 0.0f) return -INFINITY;
    if (b == 0x7f800000u) return x;
    int e = 0;
    if (b < 0x00800000u) { /* subnormal: scale by 2^25 */
        x = x * 33554432.0f;
        b = fbits(x);
        e = -25;
    }
    e += (int)(b >> 23) - 127;
    float m = bitsf((b & 0x007fffffu) | 0x3f800000u);
    if (m > 1.41421353816986083984375f) {
        m = m * 0.5f;
        e = e + 1;
    }
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float z = s * s;
    float P = fmaf(z, fmaf(z, fmaf(z, fmaf(z, 0.1818181872367859f, 0.2222222238779068f),
                                   0.2857142984867096f), 0.4000000059604645f), 0.6666666865348816f);
    float R = z * P;
    float lm = fmaf(s, R, s + s);
    float ef = (float)e;
    return fmaf(ef, 0.693115234375f, fmaf(ef, 3.194618329871446e-05f, lm));
}

/* sin/cos: k = nearest(x * 2/pi); r = x - k*pi/2 (3-part Cody-Waite);
 * Taylor polynomials on |r| <= pi/4; quadrant select. */
static void spec_sincos(float x, float* so, float* co) {
#ifdef ORC_ALT
    *so = sinf(x);
    *co = cosf(x);
    return;
#endif
    float kf = floorf(fmaf(x, 0.6366197466850281f, 0.5f));
    float r = fmaf(-kf, 7.549790126404332e-08f,
                   fmaf(-kf, 0.0004837512969970703f, fmaf(-kf, 1.5703125f, x)));
    float z = r * r;
    float ps = fmaf(z, fmaf(z, fmaf(z, fmaf(z, -2.5052107943679403e-08f, 2.7557318844628753e-06f),
                                    -0.00019841270113829523f), 0.008333333767950535f),
                    -0.1666666716337204f);
    float s = fmaf(r * z, ps, r);
    float pc = fmaf(z, fmaf(z, fmaf(z, -2.755731998149713e-07f, 2.4801587642286904e-05f),
                            -0.0013888889225199819f), 0.0416666679084301f);
    float c = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    int k = ((int)kf) & 3;
    switch (k) {
        case 0: *so = s; *co = c; break;
        case 1: *so = c; *co = -s; break;
        case 2: *so = -s; *co = -c; break;
        default: *so = -c; *co = s; break;
    }
}
float orc_sin(float x) { float s, c; spec_sincos(x, &s, &c); return s; }
float orc_cos(float x) { float s, c; spec_sincos(x, &s, &c); return c; }

uint16_t orc_f2h(float f) {
    uint32_t x = fbits(f);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u) return sign | 0x7e00u;           /* NaN */
    if (ax >= 0x477ff000u) return sign | 0x7c00u;          /* >= 65520 -> inf */
    if (ax < 0x38800000u) {                                /* below 2^-14 */
        float a = bitsf(ax) * 16777216.0f;                 /* exact */
        return sign | (uint16_t)nearbyintf(a);             /* RTE; 1024 = min normal */
    }
    uint32_t h = (((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13);
    uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return sign | (uint16_t)h;
}

static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline float len3(v3 a) { return sqrtf(dot3(a, a)); }
static inline v3 norm3(v3 a) {
    float l = len3(a);
    v3 r = {DIVF(a.x, l), DIVF(a.y, l), DIVF(a.z, l)};
    return r;
}

/* ------------------------------------------------------------------- RNG */

/* pcg.wgsl:3-7 (PCG-RXS-M-XS) */
uint32_t orc_hash(uint32_t v) {
    uint32_t x = v * 747796405u + 2891336453u;
    x = ((x >> ((x >> 28u) + 4u)) ^ x) * 277803737u;
    return (x >> 22u) ^ x;
}
/* squashlinear.wgsl:7-9 */
uint32_t orc_hash3(uint32_t x, uint32_t y, uint32_t z) {
    return orc_hash(19u * x + 47u * y + 101u * z + 131u);
}
/* uniformdivision.wgsl:3-6: f32(state) / f32(~0u); f32(~0u) == 2^32. */
static inline float rnd_uniform(uint32_t* st) {
    *st = orc_hash(*st);
    return (float)(*st) / 4294967296.0f;
}
/* exponential.wgsl:3-5 */
static inline float rnd_exponential(uint32_t* st, float rate) {
    return DIVF(-orc_log(rnd_uniform(st)), rate);
}
/* disk.wgsl:3-7 */
static inline v2 rnd_disk(uint32_t* st) {
    float radius = sqrtf(rnd_uniform(st));
    float angle = TWOPI * rnd_uniform(st);
    float s, c;
    spec_sincos(angle, &s, &c);
    v2 r = {radius * c, radius * s};
    return r;
}
/* square.wgsl:3-7 */
static inline v2 rnd_square(uint32_t* st) {
    float x = rnd_uniform(st);
    float y = rnd_uniform(st);
    v2 r = {x, y};
    return r;
}
/* sphere.wgsl:4-10 (Marsaglia) */
static inline v3 rnd_sphere(uint32_t* st) {
    v2 d = rnd_disk(st);
    float nrm = fmaf(d.y, d.y, d.x * d.x);
    float radius = 2.0f * sqrtf(1.0f - nrm);
    float z = 1.0f - 2.0f * nrm;
    v3 r = {radius * d.x, radius * d.y, z};
    return r;
}

/* --------------------------------------------------------------- sampling */

static inline float clampc(float u) { return u >= -1.0f ? (u <= 2.0f ? u : 2.0f) : -1.0f; }
static inline void axis(float u, uint32_t n, uint32_t* i0, uint32_t* i1, float* f) {
    float x = fmaf(clampc(u), (float)n, -0.5f);
    float fl = floorf(x);
    *f = x - fl;
    int i = (int)fl;
    int a = i < 0 ? 0 : (i > (int)n - 1 ? (int)n - 1 : i);
    int b = i + 1 < 0 ? 0 : (i + 1 > (int)n - 1 ? (int)n - 1 : i + 1);
    *i0 = (uint32_t)a;
    *i1 = (uint32_t)b;
}
static inline float lerp(float a, float b, float f) { return fmaf(f, b - a, a); }
#define INV255 0.003921568859368563f

/* textureSampleLevel(uVolume, linear, clamp-to-edge, p).r — wgsl:76 */
float orc_sample_volume(const uint8_t* vol, uint32_t W, uint32_t H, uint32_t D,
                        const float p[3]) {
    uint32_t x0, x1, y0, y1, z0, z1;
    float fx, fy, fz;
    axis(p[0], W, &x0, &x1, &fx);
    axis(p[1], H, &y0, &y1, &fy);
    axis(p[2], D, &z0, &z1, &fz);
#define V(i, j, k) ((float)vol[((size_t)(k) * H + (j)) * W + (i)])
    float c00 = lerp(V(x0, y0, z0), V(x1, y0, z0), fx);
    float c10 = lerp(V(x0, y1, z0), V(x1, y1, z0), fx);
    float c01 = lerp(V(x0, y0, z1), V(x1, y0, z1), fx);
    float c11 = lerp(V(x0, y1, z1), V(x1, y1, z1), fx);
#undef V
    float c0 = lerp(c00, c10, fy);
    float c1 = lerp(c01, c11, fy);
    return lerp(c0, c1, fz) * INV255;
}

/* textureSampleLevel(uTransferFunction, (t, d)).rgb — wgsl:77-79.
 * Memory row = density (v), column = wavelength (u). */
void orc_sample_tf(const uint8_t* tf, float t, float d, float out[3]) {
    uint32_t c0, c1, r0, r1;
    float fx, fy;
    axis(t, 256, &c0, &c1, &fx);
    axis(d, 256, &r0, &r1, &fy);
    for (int ch = 0; ch < 3; ch++) {
#define T(c, r) ((float)tf[((size_t)(r) * 256 + (c)) * 4 + ch])
        float a = lerp(T(c0, r0), T(c1, r0), fx);
        float b = lerp(T(c0, r1), T(c1, r1), fx);
#undef T
        out[ch] = lerp(a, b, fy) * INV255;
    }
}

/* textureSampleLevel(uLightSpectrum, (t, 0.5)).r on a 256x1 texture:
 * v = 0.5 selects row 0 for both taps, so it is a 1D lerp (wgsl:65). */
float orc_sample_light(const uint8_t* light, float t) {
    uint32_t c0, c1;
    float fx;
    axis(t, 256, &c0, &c1, &fx);
    return lerp((float)light[c0], (float)light[c1], fx) * INV255;
}

/* ------------------------------------------------------------ tone mapping */

static double h2d(uint16_t h) { /* IEEE binary16 -> double */
    int s = h >> 15, e = (h >> 10) & 31, m = h & 1023;
    double v;
    if (e == 0) v = ldexp((double)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = ldexp((double)(m | 1024), e - 25);
    return s ? -v : v;
}
static uint8_t unorm8d(double v) {
    if (!(v > 0.0)) return 0;        /* NaN and <= 0 */
    if (v >= 1.0) return 255;
    return (uint8_t)floor(v * 255.0 + 0.5);
}
/* ArtisticToneMapper.wgsl:38-48: textureSample at the texel centre (exact),
 * (c - low)/(high - low), mix(dot(c, g) g, c, saturation) with g =
 * normalize(vec3(1)), pow(c, -log2(midpoint)/gamma), rgba8unorm store. */
void orc_tonemap_artistic(const uint16_t* rgba16, uint32_t n, const float params[5],
                          uint8_t* out) {
    const double low = params[0], mid = params[1], high = params[2];
    const double sat = params[3], gamma = params[4];
    const double g = 1.0 / sqrt(3.0);
    const double e = -log((mid - low) / (high - low)) / log(2.0) / gamma;
    for (uint32_t i = 0; i < n; i++) {
        double c[3];
        for (int k = 0; k < 3; k++) c[k] = (h2d(rgba16[i * 4 + k]) - low) / (high - low);
        double d = c[0] * g + c[1] * g + c[2] * g;
        for (int k = 0; k < 3; k++) {
            double m = d * g + (c[k] - d * g) * sat;
            double p = (e == 0.0) ? 1.0 : exp2(e * log2(m));
            out[i * 4 + k] = unorm8d(p);
        }
        out[i * 4 + 3] = 255;
    }
}

/* ------------------------------------------------------------- kernel body */

typedef struct ctx {
    const orc_uniforms* u;
    const float* spec;
    const uint8_t* vol;
    uint32_t W, H, D;
    const uint8_t* tf;
    const uint8_t* light;
} ctx;

/* sample_light, wgsl:62-73 */
static float sample_light(const ctx* c, v3 d, float wavelength) {
    float t = DIVF(wavelength - 400.0f, 700.0f - 400.0f);
    float intensity = orc_sample_light(c->light, t) * 5.0f;
    v3 ld = {c->u->light_dir[0], c->u->light_dir[1], c->u->light_dir[2]};
    if (len3(ld) < EPS) return intensity;
    v3 l = norm3(ld);
    return smax(dot3(d, l) * intensity, 0.0f);
}

/* sampleHenyeyGreenstein{AngleCosine}, wgsl:82-97 */
static v3 sample_hg(uint32_t* st, float g, v3 dir) {
    v3 u = rnd_sphere(st);
    if (fabsf(g) < EPS) return u;
    float g2 = g * g;
    float c = DIVF(1.0f - g2, fmaf(2.0f * g, rnd_uniform(st), 1.0f - g));
    float hgcos = DIVF(fmaf(-c, c, 1.0f + g2), 2.0f * g);
    float ud = dot3(u, dir);
    v3 w = {fmaf(-ud, dir.x, u.x), fmaf(-ud, dir.y, u.y), fmaf(-ud, dir.z, u.z)};
    v3 circle = norm3(w);
    float sn = sqrtf(fmaf(-hgcos, hgcos, 1.0f));
    v3 r = {fmaf(sn, circle.x, hgcos * dir.x), fmaf(sn, circle.y, hgcos * dir.y),
            fmaf(sn, circle.z, hgcos * dir.z)};
    return r;
}

/* mat4x4f * vec4f, column-major */
static inline void mat_vec(const float* m, const float v[4], float o[4]) {
    for (int r = 0; r < 4; r++)
        o[r] = fmaf(m[12 + r], v[3], fmaf(m[8 + r], v[2], fmaf(m[4 + r], v[1], m[0 + r] * v[0])));
}

/* unprojectRand.wgsl:3-25 */
static void unproject_rand(uint32_t* st, v2 screen, const float* m, const float* inv_res,
                           float blur, v3* from, v3* to) {
    v2 disk = rnd_disk(st);
    float nearp[4] = {fmaf(disk.x, blur, screen.x), fmaf(disk.y, blur, screen.y), -1.0f, 1.0f};
    v2 sq = rnd_square(st);
    float farp[4] = {fmaf(fmaf(sq.x, 2.0f, -1.0f), inv_res[0], screen.x),
                     fmaf(fmaf(sq.y, 2.0f, -1.0f), inv_res[1], screen.y), 1.0f, 1.0f};
    float fd[4], td[4];
    mat_vec(m, nearp, fd);
    mat_vec(m, farp, td);
    from->x = DIVF(fd[0], fd[3]); from->y = DIVF(fd[1], fd[3]); from->z = DIVF(fd[2], fd[3]);
    to->x = DIVF(td[0], td[3]); to->y = DIVF(td[1], td[3]); to->z = DIVF(td[2], td[3]);
}

/* intersectCube.wgsl:3-11 (only tnear is used by the caller) */
static float intersect_cube_near(v3 o, v3 d) {
    float tminx = DIVF(0.0f - o.x, d.x), tminy = DIVF(0.0f - o.y, d.y), tminz = DIVF(0.0f - o.z, d.z);
    float tmaxx = DIVF(1.0f - o.x, d.x), tmaxy = DIVF(1.0f - o.y, d.y), tmaxz = DIVF(1.0f - o.z, d.z);
    float t1x = smin(tminx, tmaxx), t1y = smin(tminy, tmaxy), t1z = smin(tminz, tmaxz);
    return smax(smax(t1x, t1y), t1z);
}

static inline uint32_t n_bins_of(const float* spec) { /* u32(spec[0] + 0.5) */
    float v = spec[0] + 0.5f;
    if (!(v > 0.0f)) return 0;
    return (uint32_t)v;
}

/* PhotonSpectral_set_wavelength, wgsl:276-290 */
static void set_wavelength(orc_photon* p, const float* spec, float wavelength) {
    p->wavelength = wavelength;
    uint32_t nb = n_bins_of(spec);
    p->bin = nb - 1u;
    for (uint32_t i = 1u; i < nb; i++) {
        if (wavelength < spec[i + 1]) {
            p->bin = i - 1u;
            break;
        }
    }
}

/* PhotonSpectral_reset, wgsl:249-266 */
static void photon_reset(const ctx* c, orc_photon* p, v2 screen, uint32_t* st) {
    v3 from, to;
    unproject_rand(st, screen, c->u->mvp_inverse, c->u->inv_res, c->u->blur, &from, &to);
    v3 diff = {to.x - from.x, to.y - from.y, to.z - from.z};
    v3 dir = norm3(diff);
    p->direction[0] = dir.x; p->direction[1] = dir.y; p->direction[2] = dir.z;
    p->bounces = 0u;
    float tn = smax(intersect_cube_near(from, dir), 0.0f);
    p->position[0] = fmaf(tn, dir.x, from.x);
    p->position[1] = fmaf(tn, dir.y, from.y);
    p->position[2] = fmaf(tn, dir.z, from.z);
    for (int i = 0; i < MAX_N_BINS; i++) p->transmittance[i] = 1.0f;
    uint32_t nb = n_bins_of(c->spec);
    float min_lam = c->spec[1];
    float max_lam = c->spec[nb + 1];
    set_wavelength(p, c->spec, fmaf(rnd_uniform(st), max_lam - min_lam, min_lam));
}

/* PhotonSpectral_full_reset, wgsl:268-274 */
static void photon_full_reset(const ctx* c, orc_photon* p, v2 screen, uint32_t* st) {
    photon_reset(c, p, screen, st);
    p->samples = 0u;
    for (int i = 0; i < MAX_N_BINS; i++) p->radiance[i] = 1.0f;
}

/* PhotonSpectral_add_radiance, wgsl:292-302 */
static void add_radiance(const ctx* c, orc_photon* p, float radiance) {
    uint32_t nb = n_bins_of(c->spec);
    for (uint32_t i = 0u; i < nb && i < MAX_N_BINS; i++) {
        float tgt = (i == p->bin) ? radiance : 0.0f;
#ifdef ORC_ALT
        p->radiance[i] = p->radiance[i] + (tgt - p->radiance[i]) / (float)p->samples;
#else
        p->radiance[i] = fmaf(tgt - p->radiance[i], rcp((float)p->samples), p->radiance[i]);
#endif
    }
}

/* PhotonSpectral_radiance_to_xyz / _to_rgb, wgsl:304-326 */
static void radiance_to_rgb(const ctx* c, const orc_photon* p, float rgb[3]) {
    uint32_t nb = n_bins_of(c->spec);
    float X = 0.0f, Y = 0.0f, Z = 0.0f;
    for (uint32_t i = 0u; i < nb && i < MAX_N_BINS; i++) {
        X = fmaf(p->radiance[i], c->spec[2 + nb + i], X);
        Y = fmaf(p->radiance[i], c->spec[2 + 2 * nb + i], Y);
        Z = fmaf(p->radiance[i], c->spec[2 + 3 * nb + i], Z);
    }
    rgb[0] = fmaf(-0.498536f, Z, fmaf(-1.537150f, Y, 3.240479f * X));
    rgb[1] = fmaf(0.041556f, Z, fmaf(1.875990f, Y, -0.969255f * X));
    rgb[2] = fmaf(1.057311f, Z, fmaf(-0.204041f, Y, 0.055647f * X));
}

static inline v2 screen_pos(uint32_t x, uint32_t y, const float* inv_res) { /* wgsl:118 */
    v2 s = {fmaf((float)x + 0.5f, inv_res[0], -0.5f) * 2.0f,
            fmaf((float)y + 0.5f, inv_res[1], -0.5f) * -2.0f};
    return s;
}

/* Analysis hook (tools/march_stats.c): per-step outcome of a photon,
 * 0 null collision, 1 scatter, 2 absorption, 3 exit. No-op in the oracle. */
#ifndef ORC_EVENT
#define ORC_EVENT(x, y, step, kind) ((void)0)
#endif

/* render compute_main body for one pixel, wgsl:118-168 */
static void render_pixel(const ctx* c, uint32_t R, uint32_t x, uint32_t y, orc_photon* photons,
                         float* rgb32, uint16_t* rgba16) {
    const orc_uniforms* u = c->u;
    v2 screen = screen_pos(x, y, u->inv_res);
    orc_photon p = photons[(size_t)y * R + x];
    uint32_t st = orc_hash3(x, y, u->seed_bits);
    for (uint32_t i = 0u; i < u->steps; i++) {
        float dist = rnd_exponential(&st, u->extinction);
        p.position[0] = fmaf(dist, p.direction[0], p.position[0]);
        p.position[1] = fmaf(dist, p.direction[1], p.position[1]);
        p.position[2] = fmaf(dist, p.direction[2], p.position[2]);

        float dens = orc_sample_volume(c->vol, c->W, c->H, c->D, p.position);
        float smp[3];
        orc_sample_tf(c->tf, DIVF(p.wavelength - 400.0f, 700.0f - 400.0f), dens, smp);
        float albedo = smp[0], alpha = smp[1];
        float aniso = smp[2] * 2.0f - 1.0f;

        float pnull = 1.0f - alpha;
        float pscat = (p.bounces >= u->max_bounces) ? 0.0f : alpha * albedo;
        float pabs = (1.0f - pnull) - pscat;

        float wheel = rnd_uniform(&st);
        int oob = p.position[0] > 1.0f || p.position[1] > 1.0f || p.position[2] > 1.0f ||
                  p.position[0] < 0.0f || p.position[1] < 0.0f || p.position[2] < 0.0f;
        ORC_EVENT(x, y, i, oob ? 3 : wheel < pabs ? 2 : wheel < pabs + pscat ? 1 : 0);
        if (oob) {
            v3 d = {p.direction[0], p.direction[1], p.direction[2]};
            float rad = sample_light(c, d, p.wavelength);
            p.samples++;
            add_radiance(c, &p, rad);
            photon_reset(c, &p, screen, &st);
        } else if (wheel < pabs) {
            p.samples++;
            add_radiance(c, &p, 0.0f);
            photon_reset(c, &p, screen, &st);
        } else if (wheel < pabs + pscat) {
            v3 d = {p.direction[0], p.direction[1], p.direction[2]};
            v3 nd = sample_hg(&st, aniso, d);
            p.direction[0] = nd.x; p.direction[1] = nd.y; p.direction[2] = nd.z;
            p.bounces++;
        }
    }
    photons[(size_t)y * R + x] = p;
    float rgb[3];
    radiance_to_rgb(c, &p, rgb);
    size_t pix = (size_t)y * R + x;
    if (rgb32) { rgb32[pix * 3 + 0] = rgb[0]; rgb32[pix * 3 + 1] = rgb[1]; rgb32[pix * 3 + 2] = rgb[2]; }
    if (rgba16) {
        rgba16[pix * 4 + 0] = orc_f2h(rgb[0]);
        rgba16[pix * 4 + 1] = orc_f2h(rgb[1]);
        rgba16[pix * 4 + 2] = orc_f2h(rgb[2]);
        rgba16[pix * 4 + 3] = 0x3c00u; /* 1.0 */
    }
}

/* ------------------------------------------------------------ drivers */

typedef struct job {
    const ctx* c;
    uint32_t R, y0, y1;
    int is_reset;
    orc_photon* photons;
    float* rgb32;
    uint16_t* rgba16;
} job;

static void* run_job(void* arg) {
    job* j = (job*)arg;
    for (uint32_t y = j->y0; y < j->y1; y++) {
        for (uint32_t x = 0; x < j->R; x++) {
            if (j->is_reset) { /* reset compute_main, wgsl:224-230 */
                v2 screen = screen_pos(x, y, j->c->u->inv_res);
                orc_photon p;
                memset(&p, 0, sizeof p);
                uint32_t st = orc_hash3(x, y, j->c->u->seed_bits);
                photon_full_reset(j->c, &p, screen, &st);
                j->photons[(size_t)y * j->R + x] = p;
            } else {
                render_pixel(j->c, j->R, x, y, j->photons, j->rgb32, j->rgba16);
            }
        }
    }
    return NULL;
}

static void run_rows(const ctx* c, uint32_t R, uint32_t y0, uint32_t y1, int is_reset,
                     orc_photon* photons, float* rgb32, uint16_t* rgba16, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    uint32_t rows = y1 - y0;
    if ((uint32_t)nthreads > rows) nthreads = rows ? (int)rows : 1;
    pthread_t th[256];
    job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t].c = c;
        jobs[t].R = R;
        jobs[t].y0 = y0 + (uint32_t)((uint64_t)rows * t / nthreads);
        jobs[t].y1 = y0 + (uint32_t)((uint64_t)rows * (t + 1) / nthreads);
        jobs[t].is_reset = is_reset;
        jobs[t].photons = photons;
        jobs[t].rgb32 = rgb32;
        jobs[t].rgba16 = rgba16;
    }
    if (nthreads == 1) {
        run_job(&jobs[0]);
        return;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orc_reset(uint32_t R, const orc_uniforms* u, const float* spectrum, orc_photon* photons,
               int nthreads) {
    ctx c = {u, spectrum, NULL, 0, 0, 0, NULL, NULL};
    run_rows(&c, R, 0, R, 1, photons, NULL, NULL, nthreads);
}

void orc_render(uint32_t R, const orc_uniforms* u, const float* spectrum, const uint8_t* volume,
                uint32_t W, uint32_t H, uint32_t D, const uint8_t* tf, const uint8_t* light,
                orc_photon* photons, float* rgb32, uint16_t* rgba16, int nthreads, uint32_t y0,
                uint32_t y1) {
    ctx c = {u, spectrum, volume, W, H, D, tf, light};
    if (y1 == 0 || y1 > R) y1 = R;
    run_rows(&c, R, y0, y1, 0, photons, rgb32, rgba16, nthreads);
}

/* ===================================================== RGB sibling renderer
 * MCMComputeRenderer.wgsl ('mcm-compute', WebGPUMCMComputeRenderer.js): the
 * same Woodcock march with an RGB photon (Photon.wgsl), the TF sampled at
 * (density, 0) of an rgba8unorm-srgb texture (WebGPUAbstractComputeRenderer.js:
 * 23-28, :62-69), scattering probability alpha * max3(rgb), transmittance
 * tinting, HG with the anisotropy uniform, and the environment texel on exit. */

float orc_srgb_to_linear(uint8_t b) {
    double v = b / 255.0;
    return (float)(v <= 0.04045 ? v / 12.92 : pow((v + 0.055) / 1.055, 2.4));
}

typedef struct rgb_ctx {
    const orc_uniforms* u;
    const uint8_t* vol;
    uint32_t W, H, D;
    float tf[4096][4]; /* row 0 of the TF, decoded (row v = 0 is all a (d, 0) lookup reads) */
    uint32_t tf_w;
    float env[4];
} rgb_ctx;

/* textureSampleLevel(uTransferFunction, (d, g=0)): the v axis at 0 clamps to
 * row 0 for both taps (lerp(a, a, f) = a), the u axis is a linear lerp of the
 * decoded texels. */
static void rgb_sample_tf(const rgb_ctx* c, float d, float out[4]) {
    uint32_t i0, i1;
    float f;
    axis(d, c->tf_w, &i0, &i1, &f);
    for (int k = 0; k < 4; k++) out[k] = lerp(c->tf[i0][k], c->tf[i1][k], f);
}

/* resetPhoton, MCMComputeRenderer.wgsl:38-47 */
static void rgb_reset_photon(const rgb_ctx* c, orc_photon_rgb* p, v2 screen, uint32_t* st) {
    v3 from, to;
    unproject_rand(st, screen, c->u->mvp_inverse, c->u->inv_res, c->u->blur, &from, &to);
    v3 diff = {to.x - from.x, to.y - from.y, to.z - from.z};
    v3 dir = norm3(diff);
    p->direction[0] = dir.x; p->direction[1] = dir.y; p->direction[2] = dir.z;
    p->bounces = 0u;
    float tn = smax(intersect_cube_near(from, dir), 0.0f);
    p->position[0] = fmaf(tn, dir.x, from.x);
    p->position[1] = fmaf(tn, dir.y, from.y);
    p->position[2] = fmaf(tn, dir.z, from.z);
    p->transmittance[0] = p->transmittance[1] = p->transmittance[2] = 1.0f;
}

static inline void rgb_add_radiance(orc_photon_rgb* p, const float L[3]) {
    float in = rcp((float)p->samples);
    for (int k = 0; k < 3; k++) p->radiance[k] = fmaf(L[k] - p->radiance[k], in, p->radiance[k]);
}

/* render compute_main, MCMComputeRenderer.wgsl:97-162 */
static void rgb_render_pixel(const rgb_ctx* c, uint32_t R, uint32_t x, uint32_t y,
                             orc_photon_rgb* photons, uint16_t* rgba16) {
    const orc_uniforms* u = c->u;
    v2 screen = screen_pos(x, y, u->inv_res);
    orc_photon_rgb p = photons[(size_t)y * R + x];
    uint32_t st = orc_hash3(x, y, u->seed_bits);
    for (uint32_t i = 0u; i < u->steps; i++) {
        float dist = rnd_exponential(&st, u->extinction);
        p.position[0] = fmaf(dist, p.direction[0], p.position[0]);
        p.position[1] = fmaf(dist, p.direction[1], p.position[1]);
        p.position[2] = fmaf(dist, p.direction[2], p.position[2]);
        float vs[4];
        rgb_sample_tf(c, orc_sample_volume(c->vol, c->W, c->H, c->D, p.position), vs);
        float pnull = 1.0f - vs[3];
        float pscat = (p.bounces >= u->max_bounces) ? 0.0f : vs[3] * smax(smax(vs[0], vs[1]), vs[2]);
        float pabs = (1.0f - pnull) - pscat;
        float wheel = rnd_uniform(&st);
        int oob = p.position[0] > 1.0f || p.position[1] > 1.0f || p.position[2] > 1.0f ||
                  p.position[0] < 0.0f || p.position[1] < 0.0f || p.position[2] < 0.0f;
        if (oob) { /* environment texel (1x1 map: every coordinate reads it) */
            float L[3] = {p.transmittance[0] * c->env[0], p.transmittance[1] * c->env[1],
                          p.transmittance[2] * c->env[2]};
            p.samples++;
            rgb_add_radiance(&p, L);
            rgb_reset_photon(c, &p, screen, &st);
        } else if (wheel < pabs) {
            float L[3] = {0.0f, 0.0f, 0.0f};
            p.samples++;
            rgb_add_radiance(&p, L);
            rgb_reset_photon(c, &p, screen, &st);
        } else if (wheel < pabs + pscat) {
            for (int k = 0; k < 3; k++) p.transmittance[k] = p.transmittance[k] * vs[k];
            v3 d = {p.direction[0], p.direction[1], p.direction[2]};
            v3 nd = sample_hg(&st, u->anisotropy, d);
            p.direction[0] = nd.x; p.direction[1] = nd.y; p.direction[2] = nd.z;
            p.bounces++;
        }
    }
    photons[(size_t)y * R + x] = p;
    if (rgba16) {
        size_t pix = (size_t)y * R + x;
        for (int k = 0; k < 3; k++) rgba16[pix * 4 + k] = orc_f2h(p.radiance[k]);
        rgba16[pix * 4 + 3] = 0x3c00u;
    }
}

typedef struct rgb_job {
    const rgb_ctx* c;
    uint32_t R, y0, y1;
    int is_reset;
    orc_photon_rgb* photons;
    uint16_t* rgba16;
} rgb_job;

static void* rgb_run_job(void* arg) {
    rgb_job* j = (rgb_job*)arg;
    for (uint32_t y = j->y0; y < j->y1; y++)
        for (uint32_t x = 0; x < j->R; x++) {
            if (j->is_reset) { /* reset compute_main */
                v2 screen = screen_pos(x, y, j->c->u->inv_res);
                orc_photon_rgb p;
                memset(&p, 0, sizeof p);
                uint32_t st = orc_hash3(x, y, j->c->u->seed_bits);
                rgb_reset_photon(j->c, &p, screen, &st);
                p.radiance[0] = p.radiance[1] = p.radiance[2] = 1.0f;
                p.samples = 0u;
                j->photons[(size_t)y * j->R + x] = p;
            } else {
                rgb_render_pixel(j->c, j->R, x, y, j->photons, j->rgba16);
            }
        }
    return NULL;
}

static void rgb_run(const rgb_ctx* c, uint32_t R, int is_reset, orc_photon_rgb* photons,
                    uint16_t* rgba16, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((uint32_t)nthreads > R) nthreads = R ? (int)R : 1;
    pthread_t th[256];
    rgb_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        rgb_job j = {c, R, (uint32_t)((uint64_t)R * t / nthreads),
                     (uint32_t)((uint64_t)R * (t + 1) / nthreads), is_reset, photons, rgba16};
        jobs[t] = j;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, rgb_run_job, &jobs[t]);
    rgb_run_job(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orc_reset_rgb(uint32_t R, const orc_uniforms* u, orc_photon_rgb* photons, int nthreads) {
    static rgb_ctx c; /* large; the oracle is not re-entrant across threads of the caller */
    memset(&c, 0, sizeof c);
    c.u = u;
    rgb_run(&c, R, 1, photons, NULL, nthreads);
}

void orc_render_rgb(uint32_t R, const orc_uniforms* u, const uint8_t* volume, uint32_t W,
                    uint32_t H, uint32_t D, const uint8_t* tf, uint32_t tf_w, uint32_t tf_h,
                    const uint8_t env[4], orc_photon_rgb* photons, uint16_t* rgba16, int nthreads) {
    static rgb_ctx c;
    (void)tf_h;
    memset(&c, 0, sizeof c);
    c.u = u;
    c.vol = volume;
    c.W = W; c.H = H; c.D = D;
    c.tf_w = tf_w > 4096 ? 4096 : tf_w;
    for (uint32_t i = 0; i < c.tf_w; i++) {
        for (int k = 0; k < 3; k++) c.tf[i][k] = orc_srgb_to_linear(tf[i * 4 + k]);
        c.tf[i][3] = (float)tf[i * 4 + 3] * INV255;
    }
    for (int k = 0; k < 4; k++) c.env[k] = (float)env[k] * INV255;
    rgb_run(&c, R, 0, photons, rgba16, nthreads);
}

/* Batch evaluation of the primitives (fn as in vptmcm_debug_eval). */
void orc_eval_batch(int fn, const uint32_t* in, uint32_t* out, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        float x = bitsf(in[i]);
        switch (fn) {
            case 0: out[i] = fbits(orc_log(x)); break;
            case 1: out[i] = fbits(orc_sin(x)); break;
            case 2: out[i] = fbits(orc_cos(x)); break;
            case 3: out[i] = orc_hash(in[i]); break;
            case 4: out[i] = orc_f2h(x); break;
            default: out[i] = 0u;
        }
    }
}
