// mcm_device.h — device-side arithmetic of the spectral MCM march (gfx950).
//
// Implements the arithmetic specification of DESIGN.md ("Arithmetic
// specification"): the WGSL operations of MCMSpectralComputeRenderer.wgsl with
// every implementation-defined choice (log/sin/cos, which products are fused
// into FMAs (explicit fmaf below, nothing else contracted), min/max,
// normalize, mat*vec order, sampler filtering, f16 rounding) fixed, so the
// kernels agree bit for bit with the CPU oracle. Compiled with
// -ffp-contract=off; f32 division and sqrt are hipcc's correctly rounded
// defaults (never -ffast-math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vpt {

constexpr float kEps = 1e-5f;                     // wgsl:6
constexpr float kTwoPi = 6.2831854820251465f;     // constants.wgsl:4 as f32
constexpr float kInv255 = 0.003921568859368563f;  // unorm8 scale
constexpr int kMaxBins = 12;                      // wgsl:236

struct f3 { float x, y, z; };

__device__ __forceinline__ float as_f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t as_u(float f) { return __float_as_uint(f); }

// IEEE minNum/maxNum with explicit compares; ties keep the first operand:
// a NaN -> b; b NaN -> a; else (b < a ? b : a). Written as one select so it
// stays branch-free (the if-chain form compiles to exec-mask branches).
__device__ __forceinline__ float smin(float a, float b) { return (b < a || a != a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (b > a || a != a) ? b : a; }

// ---- correctly rounded reciprocal / sqrt / log division, fast -------------
// The arithmetic spec needs RN(1/x), RN(sqrt x) and RN(a/b). hipcc's default
// IEEE sequences are ~12 dependent instructions plus denorm-mode switches; the
// sequences below use the hardware estimate + one FMA correction and are
// PROVEN equal to the correctly rounded result for every u32 input by
// tests/test_gpu_fastmath.py (exhaustive, on the GPU, through
// vptmcm_debug_verify). Inputs outside the proven-exact ranges take the
// default IEEE path.
__device__ __forceinline__ float rcp_slow(float x) { return 1.0f / x; }
__device__ __forceinline__ float sqrt_slow(float x) { return __builtin_sqrtf(x); }

// Rare-input fix-up as a wave-uniform branch: one compare into an SGPR mask
// and a scalar branch on it, instead of an exec-mask region (saveexec + the
// exec restore, whose hazards cost ~2x a plain instruction each). Inside the
// branch the slow value is selected per lane.
#ifndef VPT_UNIFORM_GUARDS
#define VPT_UNIFORM_GUARDS 1
#endif
#if VPT_UNIFORM_GUARDS
#define VPT_FIXUP(bad, y, slow)                                                  \
  do {                                                                           \
    const bool _bad = (bad);                                                     \
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(_bad) != 0ull, 0)) {        \
      (y) = _bad ? (slow) : (y);                                                 \
    }                                                                            \
  } while (0)
#else
#define VPT_FIXUP(bad, y, slow)                     \
  do {                                              \
    if (__builtin_expect((bad), 0)) (y) = (slow);   \
  } while (0)
#endif

// RN(1/x): v_rcp_f32 + one Newton step is exact for biased exponent 1..252.
__device__ __forceinline__ float rcp_cr(float x) {
  float y = __builtin_amdgcn_rcpf(x);
  float e = __builtin_fmaf(-x, y, 1.0f);
  y = __builtin_fmaf(e, y, y);
  uint32_t ex = (__float_as_uint(x) >> 23) & 0xffu;
  VPT_FIXUP(ex - 1u >= 252u, y, rcp_slow(x));
  return y;
}

// RN(1/x) for x known to have biased exponent 1..252 (e.g. a sample count
// converted to f32): the proven fast path without the range guard.
__device__ __forceinline__ float rcp_in_range(float x) {
  float y = __builtin_amdgcn_rcpf(x);
  float e = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

// RN(1/x) for finite |x| < 2^126 or NaN (e.g. a unit-vector component or a
// HG denominator in [0, 2]): the only inputs outside the fast path's proven
// range are then zero and denormals (and NaN, harmlessly), which one compare
// with an abs modifier detects (vs the 3-instruction exponent range test).
__device__ __forceinline__ float rcp_small(float x) {
  float y = rcp_in_range(x);
  VPT_FIXUP(!(__builtin_fabsf(x) >= 1.17549435e-38f), y, rcp_slow(x));
  return y;
}

// RN(sqrt x) from the rsq estimate alone: s0 = x * rsq(x), then one Newton
// correction with the same estimate, s = fma(x - s0^2, rsq/2, s0) — exact for
// positive x with biased exponent 32..254 (one transcendental instead of the
// v_sqrt + v_rsq pair; proven like the pair, tests/test_gpu_fastmath.py).
__device__ __forceinline__ float sqrt_rsq(float x) {
  float y = __builtin_amdgcn_rsqf(x);
  float s = x * y;
  float e = __builtin_fmaf(-s, s, x);
  return __builtin_fmaf(e, 0.5f * y, s);
}

__device__ __forceinline__ float sqrt_cr(float x) {
  float s = sqrt_rsq(x);
  uint32_t ex = __float_as_uint(x) >> 23;  // sign bit included: negatives excluded
  VPT_FIXUP(ex - 32u > 222u, s, sqrt_slow(x));
  return s;
}

// RN(sqrt x) for x that is +-0, NaN, a normal negative, or positive with
// biased exponent 32..254 (e.g. 1 - y for y in [0, 1] (0 or >= 2^-24 by
// Sterbenz), or f32(h) * 2^-32 (0 or >= 2^-32)): the fast path is exact there
// for everything but +-0 (where the Newton step makes 0 * inf), which one
// select returns as is.
__device__ __forceinline__ float sqrt_z(float x) {
  float s = sqrt_rsq(x);
  return x == 0.0f ? x : s;
}

// RN(f / (2 + f)) for f = m - 1, m in [sqrt(.5), sqrt(2)] (spec_log's only
// division): exact over that whole domain (proven exhaustively).
__device__ __forceinline__ float log_div(float f) {
  float d = 2.0f + f;
  float y = __builtin_amdgcn_rcpf(d);
  float e = __builtin_fmaf(-d, y, 1.0f);
  y = __builtin_fmaf(e, y, y);
  float q = f * y;
  float r = __builtin_fmaf(-q, d, f);
  return __builtin_fmaf(r, y, q);
}

// log(x) = e*ln2 + 2*atanh(s), s = (m-1)/(m+1), m in [sqrt(.5), sqrt(2)).
// Core for a normal positive x given as bit pattern b plus extra exponent e0.
__device__ __forceinline__ float spec_log_normal(uint32_t b, int e0) {
  int e = e0 + (int)(b >> 23) - 127;
  float m = as_f((b & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421353816986083984375f) {
    m = m * 0.5f;
    e = e + 1;
  }
  float f = m - 1.0f;
  float s = log_div(f);
  float z = s * s;
  float Pz = fmaf(z, fmaf(z, fmaf(z, fmaf(z, 0.1818181872367859f, 0.2222222238779068f),
                                  0.2857142984867096f), 0.4000000059604645f), 0.6666666865348816f);
  float R = z * Pz;
  float lm = fmaf(s, R, s + s);
  float ef = (float)e;
  return fmaf(ef, 0.693115234375f, fmaf(ef, 3.194618329871446e-05f, lm));
}

__device__ __forceinline__ float spec_log(float x) {
  uint32_t b = as_u(x);
  if (!(x > 0.0f)) return (x == 0.0f) ? -__builtin_inff() : __builtin_nanf("");
  if (b == 0x7f800000u) return x;
  int e = 0;
  if (b < 0x00800000u) {
    x = x * 33554432.0f;
    b = as_u(x);
    e = -25;
  }
  return spec_log_normal(b, e);
}

// spec_log(f32(h) * 2^-32): the argument is 0 or a normal number in
// [2^-32, 1], so the zero/denormal/inf/NaN paths reduce to one select.
// Equal to spec_log on all 2^32 h (tests/test_gpu_fastmath.py, fn 9).
__device__ __forceinline__ float spec_log_unit(uint32_t h) {
  float r = spec_log_normal(as_u((float)h * 2.3283064365386963e-10f), 0);
  return h == 0u ? -__builtin_inff() : r;
}

// sin/cos: 3-part Cody-Waite reduction by pi/2, Taylor on |r| <= pi/4.
__device__ __forceinline__ void spec_sincos(float x, float* so, float* co) {
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
  float sa = (k & 1) ? c : s;
  float ca = (k & 1) ? s : c;
  *so = (k & 2) ? -sa : sa;
  *co = ((k + 1) & 2) ? -ca : ca;
}

// PCG-RXS-M-XS, pcg.wgsl:3-7
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
  uint32_t x = v * 747796405u + 2891336453u;
  x = ((x >> ((x >> 28u) + 4u)) ^ x) * 277803737u;
  return (x >> 22u) ^ x;
}
// squashlinear.wgsl:7-9
__device__ __forceinline__ uint32_t hash3(uint32_t x, uint32_t y, uint32_t z) {
  return pcg_hash(19u * x + 47u * y + 101u * z + 131u);
}
// uniformdivision.wgsl:3-6; f32(~0u) == 2^32, so the division is exact scaling.
__device__ __forceinline__ float rnd_uniform(uint32_t& st) {
  st = pcg_hash(st);
  return (float)st * 2.3283064365386963e-10f;
}

// The spec's division: WGSL `a / b` (2.5 ULP allowed) is a * rcp(b) with
// rcp(b) = RN(1/b), one correctly rounded reciprocal per divisor value.
__device__ __forceinline__ float rcp(float x) { return rcp_cr(x); }

__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// RN(1 / RN(sqrt x)) with ONE range guard: where sqrt_cr's fast path is exact
// (x > 0 with biased exponent 32..254) the root lies in [2^-48, 2^64), inside
// rcp_in_range's exact range, so its own guard is redundant; every other x
// takes the IEEE pair. Equal to rcp_cr(sqrt_cr(x)) for all 2^32 x
// (tests/test_gpu_fastmath.py, fn 17).
__device__ __forceinline__ float inv_len(float x) {
  float y = rcp_in_range(sqrt_rsq(x));
  uint32_t ex = __float_as_uint(x) >> 23;
  VPT_FIXUP(ex - 32u > 222u, y, rcp_slow(sqrt_slow(x)));
  return y;
}

__device__ __forceinline__ f3 norm3(f3 a) {
  float il = inv_len(dot3(a, a));
  return f3{a.x * il, a.y * il, a.z * il};
}

// float -> half, round to nearest even (v_cvt_f16_f32 under the default mode).
// The empty asm pins f to a VGPR as an f32 value: without it the backend folds
// fptrunc(fma(a, b, c)) into v_fma_mix*_f16, which rounds once to f16 instead
// of f32 then f16 (a tie of the f32 result then rounds differently).
__device__ __forceinline__ uint16_t f2h(float f) {
  asm volatile("" : "+v"(f));
  _Float16 h = (_Float16)f;
  return __builtin_bit_cast(uint16_t, h);
}

// ---- sampler (linear, clamp-to-edge) ---------------------------------------
__device__ __forceinline__ float clampc(float u) {
  return u >= -1.0f ? (u <= 2.0f ? u : 2.0f) : -1.0f;
}
// texel-space coordinate: x = clampc(u)*N - 0.5; returns floor as int and f.
__device__ __forceinline__ int axis_floor(float u, float n, float* f) {
  float x = fmaf(clampc(u), n, -0.5f);
  float fl = floorf(x);
  *f = x - fl;
  return (int)fl;
}
// clampc for a quiet (arithmetic-result) input: minNum(maxNum(u, -1), 2), a
// quiet NaN yielding the other operand (NaN -> -1 like clampc). The backend
// emits a canonicalising v_max + v_med3_f32 (the earlier inline-asm v_max/
// v_min pair cost the same plus hazard s_nops). Exact equality with clampc on
// every non-signalling bit pattern is proven exhaustively
// (tests/test_gpu_fastmath.py, fn 15).
__device__ __forceinline__ float clampc_q(float u) {
  return __builtin_fminf(__builtin_fmaxf(u, -1.0f), 2.0f);
}
__device__ __forceinline__ int axis_floor_q(float u, float n, float* f) {
  float x = fmaf(clampc_q(u), n, -0.5f);
  float fl = floorf(x);
  *f = x - fl;
  return (int)fl;
}
// axis_floor for u known to lie in [-1, 2] (e.g. a filtered texel value in
// [0, 1]): clampc is the identity there.
__device__ __forceinline__ int axis_floor_in(float u, float n, float* f) {
  float x = fmaf(u, n, -0.5f);
  float fl = floorf(x);
  *f = x - fl;
  return (int)fl;
}
// IEEE minNum/maxNum (v_min_f32 / v_max_f32 / v_max3_f32; the backend adds a
// canonicalising v_max only for operands it cannot prove quiet). They equal
// smin/smax whenever no operand is a signalling NaN and the operands are not a
// (+0, -0) pair (fn 16 checks the pairing rule over every bit pattern of one
// operand against special and neighbouring values of the other).
__device__ __forceinline__ float hw_min(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float hw_max(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float hw_max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}

// max(min(i, hi), 0) for hi >= 0 (the same value as i < 0 ? 0 : i > hi ? hi : i): one v_med3_i32
__device__ __forceinline__ int clampi(int i, int hi) { return __builtin_elementwise_max(__builtin_elementwise_min(i, hi), 0); }
__device__ __forceinline__ float lerp(float a, float b, float f) { return fmaf(f, b - a, a); }

}  // namespace vpt
