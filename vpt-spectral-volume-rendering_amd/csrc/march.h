// march.h — the spectral MCM photon march and photon reset for gfx950.
//
// One lane owns one photon (= one pixel), exactly like the reference's
// compute_main (MCMSpectralComputeRenderer.wgsl:107-179 render, :213-231
// reset). What is MI355X-specific is the data layout and mapping:
//   * photon state is stored as 22 SoA planes of 32-bit words in
//     "wave-tile" order — wave w of the grid owns an 8x8 pixel tile and lane
//     l = 8*ly + lx its pixel — so every plane load/store is one fully
//     coalesced 256-B wave access and a wave's rays start in a compact
//     screen-space footprint (volume gathers hit the same cache lines);
//   * the volume is either x-fastest u8 (LINEAR) or CORNER8: one u64 per
//     trilinear cell holding its 8 corner voxels, so the 2x2x2 stencil is a
//     single 8-B load instead of 8 byte gathers;
//   * blocks are remapped so consecutive tiles run on the same XCD (shared
//     L2 for neighbouring rays);
//   * per-photon constants of the current wavelength (TF column taps and
//     weight, light intensity) are computed once per (re)set and kept in
//     registers instead of once per step — bit-identical by construction.
#pragma once

#include "mcm_device.h"

namespace vpt {

enum : uint32_t { kLayoutLinear = 0, kLayoutCorner8 = 1 };

// Plane indices of the SoA photon buffer.
enum Plane : uint32_t {
  kPx = 0, kPy, kPz, kDx, kDy, kDz, kBounces, kSamples, kBin, kLambda, kRad0, kNumPlanes = kRad0 + kMaxBins
};

struct MarchParams {
  float m[16];           // mvpInverse, column-major
  float inv_res[2];      // 1/R as f32 (js:297)
  uint32_t seed;         // bitcast<u32>(randSeed)
  float blur;
  float extinction;
  uint32_t max_bounces;
  uint32_t steps;
  uint32_t nb;           // u32(spectrum[0] + 0.5)
  float lam[13];         // spectrum[1 .. 13]: bin boundaries
  float min_lam, max_lam; // spectrum[1], spectrum[nb + 1] (wgsl:262-263)
  float xb[kMaxBins], yb[kMaxBins], zb[kMaxBins];  // CMF bin means (0 past nb)
  float light_dir[3];    // normalize(light_direction) (host-computed, IEEE)
  uint32_t light_iso;    // length(light_direction) < EPS
  uint32_t R, tiles_x, n_tiles, npad;
  uint32_t W, H, D;
};

// ---------------------------------------------------------------- RNG draws
__device__ __forceinline__ void rnd_disk(uint32_t& st, float& dx, float& dy) {  // disk.wgsl
  float radius = __builtin_sqrtf(rnd_uniform(st));
  float angle = kTwoPi * rnd_uniform(st);
  float s, c;
  spec_sincos(angle, &s, &c);
  dx = radius * c;
  dy = radius * s;
}
__device__ __forceinline__ f3 rnd_sphere(uint32_t& st) {  // sphere.wgsl:4-10
  float dx, dy;
  rnd_disk(st, dx, dy);
  float nrm = dx * dx + dy * dy;
  float radius = 2.0f * __builtin_sqrtf(1.0f - nrm);
  float z = 1.0f - 2.0f * nrm;
  return f3{radius * dx, radius * dy, z};
}

// sampleHenyeyGreenstein{AngleCosine}, wgsl:82-97
__device__ __forceinline__ f3 sample_hg(uint32_t& st, float g, f3 dir) {
  f3 u = rnd_sphere(st);
  if (__builtin_fabsf(g) < kEps) return u;
  float g2 = g * g;
  float c = (1.0f - g2) / ((1.0f - g) + (2.0f * g) * rnd_uniform(st));
  float hgcos = ((1.0f + g2) - c * c) / (2.0f * g);
  float ud = dot3(u, dir);
  f3 circle = norm3(f3{u.x - ud * dir.x, u.y - ud * dir.y, u.z - ud * dir.z});
  float sn = __builtin_sqrtf(1.0f - hgcos * hgcos);
  return f3{sn * circle.x + hgcos * dir.x, sn * circle.y + hgcos * dir.y,
            sn * circle.z + hgcos * dir.z};
}

// Per-photon wavelength constants: TF column taps + weight, and the light
// intensity textureSampleLevel(uLightSpectrum, (t, .5)).r * 5 (wgsl:64-65).
struct WaveConst {
  int c0, c1;
  float fc;
  float intensity;
};
__device__ __forceinline__ WaveConst wave_const(float lambda, const float* s_light) {
  float t = (lambda - 400.0f) / (700.0f - 400.0f);  // wgsl:64 == wgsl:77
  WaveConst w;
  int ic = axis_floor(t, 256.0f, &w.fc);
  w.c0 = clampi(ic, 255);
  w.c1 = clampi(ic + 1, 255);
  w.intensity = lerp(s_light[w.c0], s_light[w.c1], w.fc) * kInv255 * 5.0f;
  return w;
}

// PhotonSpectral_set_wavelength, wgsl:276-290 (bin search over lam[])
__device__ __forceinline__ uint32_t bin_of(const MarchParams& P, float lambda) {
  uint32_t bin = P.nb - 1u;
#pragma unroll
  for (uint32_t i = 1u; i < (uint32_t)kMaxBins; i++) {
    if (i < P.nb && bin == P.nb - 1u && lambda < P.lam[i]) bin = i - 1u;
  }
  return bin;
}

struct Photon {
  f3 pos, dir;
  uint32_t bounces, samples, bin;
  float lambda;
  float rad[kMaxBins];
};

// PhotonSpectral_reset, wgsl:249-266 (+ unprojectRand.wgsl, intersectCube.wgsl)
__device__ __forceinline__ void photon_reset(const MarchParams& P, Photon& p, float sx, float sy,
                                             uint32_t& st) {
  float dx, dy;
  rnd_disk(st, dx, dy);
  float n0 = sx + dx * P.blur, n1 = sy + dy * P.blur;
  float q0 = rnd_uniform(st);
  float q1 = rnd_uniform(st);
  float f0 = sx + (q0 * 2.0f - 1.0f) * P.inv_res[0];
  float f1 = sy + (q1 * 2.0f - 1.0f) * P.inv_res[1];
  const float* m = P.m;
  float fd[4], td[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    fd[r] = ((m[r] * n0 + m[4 + r] * n1) + m[8 + r] * -1.0f) + m[12 + r] * 1.0f;
    td[r] = ((m[r] * f0 + m[4 + r] * f1) + m[8 + r] * 1.0f) + m[12 + r] * 1.0f;
  }
  f3 from{fd[0] / fd[3], fd[1] / fd[3], fd[2] / fd[3]};
  f3 to{td[0] / td[3], td[1] / td[3], td[2] / td[3]};
  f3 dir = norm3(f3{to.x - from.x, to.y - from.y, to.z - from.z});
  p.dir = dir;
  p.bounces = 0u;
  float t1x = smin((0.0f - from.x) / dir.x, (1.0f - from.x) / dir.x);
  float t1y = smin((0.0f - from.y) / dir.y, (1.0f - from.y) / dir.y);
  float t1z = smin((0.0f - from.z) / dir.z, (1.0f - from.z) / dir.z);
  float tn = smax(smax(smax(t1x, t1y), t1z), 0.0f);
  p.pos = f3{from.x + tn * dir.x, from.y + tn * dir.y, from.z + tn * dir.z};
  float lambda = rnd_uniform(st) * (P.max_lam - P.min_lam) + P.min_lam;
  p.lambda = lambda;
  p.bin = bin_of(P, lambda);
}

__device__ __forceinline__ void screen_of(const MarchParams& P, uint32_t x, uint32_t y, float& sx,
                                          float& sy) {  // wgsl:118
  sx = (((float)x + 0.5f) * P.inv_res[0] - 0.5f) * 2.0f;
  sy = (((float)y + 0.5f) * P.inv_res[1] - 0.5f) * -2.0f;
}

// Consecutive logical blocks -> same XCD (blocks are dealt round-robin over 8).
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nblocks) {
  if ((nblocks & 7u) != 0u) return b;
  return (b & 7u) * (nblocks >> 3) + (b >> 3);
}

}  // namespace vpt
