// kernels.hip — gfx950 kernels of the spectral MCM path.
//
//   k_reset<>     PhotonSpectral_full_reset for every photon  (wgsl:213-231)
//   k_march<L>    one progressive pass: `steps` Woodcock delta-tracking steps
//                 per photon + radiance_to_rgb + rgba16float store
//                 (wgsl:107-179); L = volume layout
//   k_corner8     LINEAR u8 volume -> CORNER8 (one u64 of 8 corners per cell)
//   k_pack        (rgb*n, n) float4 per pixel for the cross-rank all-reduce
//   k_debug_eval  spec-math primitives, for device-vs-oracle parity tests
#include "kernels.h"

namespace vpt {

// ------------------------------------------------------------- photon I/O
__device__ __forceinline__ void load_photon(const float* __restrict__ ph, size_t S, size_t i,
                                            Photon& p) {
  p.pos = f3{ph[kPx * S + i], ph[kPy * S + i], ph[kPz * S + i]};
  p.dir = f3{ph[kDx * S + i], ph[kDy * S + i], ph[kDz * S + i]};
  p.bounces = as_u(ph[kBounces * S + i]);
  p.samples = as_u(ph[kSamples * S + i]);
  p.bin = as_u(ph[kBin * S + i]);
  p.lambda = ph[kLambda * S + i];
#pragma unroll
  for (int b = 0; b < kMaxBins; b++) p.rad[b] = ph[(kRad0 + b) * S + i];
}

__device__ __forceinline__ void store_state(float* __restrict__ ph, size_t S, size_t i,
                                            const Photon& p) {
  ph[kPx * S + i] = p.pos.x;
  ph[kPy * S + i] = p.pos.y;
  ph[kPz * S + i] = p.pos.z;
  ph[kDx * S + i] = p.dir.x;
  ph[kDy * S + i] = p.dir.y;
  ph[kDz * S + i] = p.dir.z;
  ph[kBounces * S + i] = as_f(p.bounces);
  ph[kSamples * S + i] = as_f(p.samples);
  ph[kBin * S + i] = as_f(p.bin);
  ph[kLambda * S + i] = p.lambda;
}

template <uint32_t BLOCK = kBlock>
__device__ __forceinline__ bool tile_pixel(const MarchParams& P, uint32_t& x, uint32_t& y,
                                           size_t& idx) {
  uint32_t b = xcd_swizzle(blockIdx.x, gridDim.x);
  uint32_t tile = b * (BLOCK / 64) + (threadIdx.x >> 6);
  uint32_t lane = threadIdx.x & 63u;
  if (tile >= P.n_tiles) return false;
  x = (tile % P.tiles_x) * 8u + (lane & 7u);
  y = (tile / P.tiles_x) * 8u + (lane >> 3);
  idx = (size_t)tile * 64u + lane;
  return x < P.R && y < P.R;
}

// -------------------------------------------------------------- reset kernel
__device__ __forceinline__ bool near_fixed(const MarchParams& P, float sx, float sy, f3& from) {
  bool fixed = P.blur == 0.0f && sx != 0.0f && sy != 0.0f;
  if (fixed) from = unproject(P.m, sx, sy, -1.0f);
  return fixed;
}

__global__ __launch_bounds__(kBlock) void k_reset(const MarchParams P, float* __restrict__ ph) {
  uint32_t x, y;
  size_t i;
  if (!tile_pixel(P, x, y, i)) return;
  const size_t S = P.npad;
  float sx, sy;
  screen_of(P, x, y, sx, sy);
  f3 from{0.0f, 0.0f, 0.0f};
  bool fixed = near_fixed(P, sx, sy, from);
  uint32_t st = hash3(x, y, P.seed);
  Photon p;
  photon_reset(P, p, sx, sy, fixed, from, st);
  p.samples = 0u;
  store_state(ph, S, i, p);
#pragma unroll
  for (int b = 0; b < kMaxBins; b++) ph[(kRad0 + b) * S + i] = 1.0f;
}

// ------------------------------------------------------------ volume sample
// textureSampleLevel(uVolume, linear, clamp-to-edge, p).r (wgsl:76), split in
// two so the gather can be issued early and filtered after other work.
struct VolTap {
  float fx, fy, fz;
  uint32_t lo, hi;  // the 8 corner voxels, byte (dz*4 + dy*2 + dx)
};

template <uint32_t L>
__device__ __forceinline__ VolTap vol_fetch(const MarchParams& P, const uint8_t* __restrict__ vol,
                                            f3 q) {
  VolTap t;
  int ix = axis_floor(q.x, (float)P.W, &t.fx);
  int iy = axis_floor(q.y, (float)P.H, &t.fy);
  int iz = axis_floor(q.z, (float)P.D, &t.fz);
  if constexpr (L == kLayoutCorner8) {
    const uint32_t W1 = P.W + 1u, H1 = P.H + 1u;
    uint32_t cx = (uint32_t)(clampi(ix + 1, (int)P.W));
    uint32_t cy = (uint32_t)(clampi(iy + 1, (int)P.H));
    uint32_t cz = (uint32_t)(clampi(iz + 1, (int)P.D));
    size_t cell = ((size_t)cz * H1 + cy) * W1 + cx;
    uint2 c = reinterpret_cast<const uint2*>(vol)[cell];
    t.lo = c.x;
    t.hi = c.y;
  } else {
    const int wm = (int)P.W - 1, hm = (int)P.H - 1, dm = (int)P.D - 1;
    uint32_t x0 = clampi(ix, wm), x1 = clampi(ix + 1, wm);
    uint32_t y0 = clampi(iy, hm), y1 = clampi(iy + 1, hm);
    uint32_t z0 = clampi(iz, dm), z1 = clampi(iz + 1, dm);
    size_t r00 = ((size_t)z0 * P.H + y0) * P.W, r10 = ((size_t)z0 * P.H + y1) * P.W;
    size_t r01 = ((size_t)z1 * P.H + y0) * P.W, r11 = ((size_t)z1 * P.H + y1) * P.W;
    t.lo = (uint32_t)vol[r00 + x0] | ((uint32_t)vol[r00 + x1] << 8) |
           ((uint32_t)vol[r10 + x0] << 16) | ((uint32_t)vol[r10 + x1] << 24);
    t.hi = (uint32_t)vol[r01 + x0] | ((uint32_t)vol[r01 + x1] << 8) |
           ((uint32_t)vol[r11 + x0] << 16) | ((uint32_t)vol[r11 + x1] << 24);
  }
  return t;
}

__device__ __forceinline__ float vol_filter(const VolTap& t) {
  float c00 = lerp((float)(t.lo & 0xffu), (float)((t.lo >> 8) & 0xffu), t.fx);
  float c10 = lerp((float)((t.lo >> 16) & 0xffu), (float)(t.lo >> 24), t.fx);
  float c01 = lerp((float)(t.hi & 0xffu), (float)((t.hi >> 8) & 0xffu), t.fx);
  float c11 = lerp((float)((t.hi >> 16) & 0xffu), (float)(t.hi >> 24), t.fx);
  float c0 = lerp(c00, c10, t.fy);
  float c1 = lerp(c01, c11, t.fy);
  return lerp(c0, c1, t.fz) * kInv255;
}

template <uint32_t L>
__device__ __forceinline__ float sample_volume(const MarchParams& P, const uint8_t* __restrict__ vol,
                                               f3 q) {
  return vol_filter(vol_fetch<L>(P, vol, q));
}

__device__ __forceinline__ float byte_f(uint32_t v, int sh) { return (float)((v >> sh) & 0xffu); }

// ------------------------------------------------------------- march kernel
// Cost attribution, compiled only into the experiment library
// (-DVPT_EXPERIMENTS): knock-out switches (they change results) and
// s_memtime stamps that accumulate per-segment wave cycles (they do not).
#ifdef VPT_EXPERIMENTS
__constant__ uint32_t g_ko;
__device__ unsigned long long g_stamp[16];
#define KO(bit) ((g_ko >> (bit)) & 1u)
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_DECL unsigned long long _tp = stamp_now(), _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(k)                          \
  do {                                    \
    unsigned long long _tn = stamp_now(); \
    _acc[k] += _tn - _tp;                 \
    _tp = _tn;                            \
  } while (0)
#define STAMP_FLUSH()                                                        \
  do {                                                                       \
    if ((threadIdx.x & 63u) == 0u)                                           \
      for (int _k = 0; _k < 8; _k++) atomicAdd(&g_stamp[_k], _acc[_k]);     \
  } while (0)
#else
#define KO(bit) 0u
#define STAMP_DECL
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP_FLUSH() \
  do {                \
  } while (0)
#endif

template <uint32_t L, bool SPEC>
__global__ __launch_bounds__(kMarchBlock) void k_march(const MarchParams P, float* __restrict__ ph,
                                                       const uint8_t* __restrict__ vol,
                                                       const uint16_t* __restrict__ tf_rg,
                                                       const uint32_t* __restrict__ tf_b4,
                                                       const uint8_t* __restrict__ tf_brow,
                                                       const uint8_t* __restrict__ light,
                                                       uint16_t* __restrict__ rgba) {
  // (albedo, alpha) of the whole TF in LDS: every step's 4 TF taps become
  // ds_read_u16 instead of divergent L2 gathers. When the anisotropy channel
  // does not vary with wavelength (P.b_rows), its 256 row values sit in LDS
  // too and the bilinear b lookup is an exact row lerp; otherwise one
  // 4-corner gather from tf_b4.
  __shared__ uint4 s_tf4[256 * 256 * 2 / 16];
  __shared__ float s_light[256];
  __shared__ float s_brow[256];

  STAMP_DECL
  uint32_t x, y;
  size_t i;
  const bool live = tile_pixel<kMarchBlock>(P, x, y, i);
  const size_t S = P.npad;
  Photon p;
  if (live) load_photon(ph, S, i, p);  // issue the state loads before the LDS fill

  const uint4* src = reinterpret_cast<const uint4*>(tf_rg);
#pragma unroll
  for (uint32_t k = 0; k < 256 * 256 * 2 / 16 / kMarchBlock; k++)
    s_tf4[threadIdx.x + k * kMarchBlock] = src[threadIdx.x + k * kMarchBlock];
  if (threadIdx.x < 256u) {
    s_light[threadIdx.x] = (float)light[threadIdx.x];
    s_brow[threadIdx.x] = (float)tf_brow[threadIdx.x];
  }
  __syncthreads();
  if (!live) return;
  const uint16_t* s_tf = reinterpret_cast<const uint16_t*>(s_tf4);
  STAMP(0);  // prologue: state loads issued, TF/light staged in LDS

  float sx, sy;
  screen_of(P, x, y, sx, sy);
  f3 from{0.0f, 0.0f, 0.0f};
  bool fixed = near_fixed(P, sx, sy, from);
  WaveConst wc = wave_const(p.lambda, s_light);
  uint32_t st = hash3(x, y, P.seed);  // wgsl:122 (state is not carried across passes)

  if constexpr (SPEC) {
    // add_radiance of a termination is deferred into the next step's gather
    // shadow (it only touches the radiance bins, applied in the same order).
    float pend_n = 0.0f, pend_l = 0.0f;
    uint32_t pend_bin = 0u;
    auto apply_pending = [&]() {
      if (pend_n != 0.0f) {
        float inv_n = rcp(pend_n);
#pragma unroll
        for (int b = 0; b < kMaxBins; b++) {  // PhotonSpectral_add_radiance, wgsl:292-302
          if ((uint32_t)b < P.nb) {
            float tgt = ((uint32_t)b == pend_bin) ? pend_l : 0.0f;
            p.rad[b] = p.rad[b] + (tgt - p.rad[b]) * inv_n;
          }
        }
        pend_n = 0.0f;
      }
    };
    for (uint32_t step = 0; step < P.steps; step++) {
      // distance + wheel draws (exponential.wgsl, wgsl:124-125, :141)
      uint32_t s1 = pcg_hash(st);
      float dist = -spec_log((float)s1 * 2.3283064365386963e-10f) * P.rcp_extinction;
      p.pos.x = p.pos.x + dist * p.dir.x;
      p.pos.y = p.pos.y + dist * p.dir.y;
      p.pos.z = p.pos.z + dist * p.dir.z;
      uint32_t sw = pcg_hash(s1);
      float wheel = (float)sw * 2.3283064365386963e-10f;
      bool oob = p.pos.x > 1.0f || p.pos.y > 1.0f || p.pos.z > 1.0f || p.pos.x < 0.0f ||
                 p.pos.y < 0.0f || p.pos.z < 0.0f;
      VolTap vt;
      if (KO(1)) {
        vt.fx = vt.fy = vt.fz = 0.5f;
        vt.lo = vt.hi = 0x80808080u;
      } else {
        vt = vol_fetch<L>(P, vol, p.pos);  // gather in flight from here
      }
      STAMP(1);  // step head: draws, log, advance, gather issue (first step: + state-load wait)
      apply_pending();

      // Speculative candidates, all derived from the state after the wheel
      // draw and independent of the gather: the reset (draws h1..h5) and the
      // g-independent half of the HG scatter (sphere from h1,h2; uniform h3).
      uint32_t h1 = pcg_hash(sw), h2 = pcg_hash(h1), h3 = pcg_hash(h2);
      uint32_t h4 = pcg_hash(h3), h5 = pcg_hash(h4);
      float dx, dy;
      {
        float radius = sqrt_cr((float)h1 * 2.3283064365386963e-10f);
        float angle = kTwoPi * ((float)h2 * 2.3283064365386963e-10f);
        float sn, cs;
        spec_sincos(angle, &sn, &cs);
        dx = radius * cs;
        dy = radius * sn;
      }
      Photon rc;
      WaveConst wcr = wc;
      if (KO(3)) {
        rc.pos = from;
        rc.dir = f3{dx, dy, 1.0f};
        rc.lambda = p.lambda;
        rc.bin = p.bin;
      } else {
        reset_from_draws(P, rc, sx, sy, fixed, from, dx, dy, h3, h4, h5);
        wcr = wave_const(rc.lambda, s_light);
      }
      STAMP(2);  // speculative reset candidate
      float nrm = dx * dx + dy * dy;  // sphere.wgsl
      float srad = 2.0f * sqrt_cr(1.0f - nrm);
      f3 u{srad * dx, srad * dy, 1.0f - 2.0f * nrm};
      float u3 = (float)h3 * 2.3283064365386963e-10f;
      float ud = dot3(u, p.dir);
      f3 circle = KO(4) ? u : norm3(f3{u.x - ud * p.dir.x, u.y - ud * p.dir.y, u.z - ud * p.dir.z});
      STAMP(3);  // speculative scatter half

      // sample_volume_color (wgsl:75-80) -> probabilities (wgsl:132-139)
      float d = vol_filter(vt);
      float fr;
      int ir = axis_floor(d, 256.0f, &fr);
      uint32_t b4 = 0u;
      if (!P.b_rows) b4 = tf_b4[(uint32_t)clampi(ir + 1, 256) * kTfCells + (uint32_t)wc.cc];
      const uint32_t ri0 = (uint32_t)clampi(ir, 255), ri1 = (uint32_t)clampi(ir + 1, 255);
      uint32_t r0 = ri0 * 256u, r1 = ri1 * 256u;
      uint32_t t00, t10, t01, t11;
      if (KO(2)) {
        t00 = t10 = t01 = t11 = 0x8080u + r0;
      } else {
        t00 = s_tf[r0 + wc.c0];
        t10 = s_tf[r0 + wc.c1];
        t01 = s_tf[r1 + wc.c0];
        t11 = s_tf[r1 + wc.c1];
      }
      float albedo = lerp(lerp(byte_f(t00, 0), byte_f(t10, 0), wc.fc),
                          lerp(byte_f(t01, 0), byte_f(t11, 0), wc.fc), fr) * kInv255;
      float alpha = lerp(lerp(byte_f(t00, 8), byte_f(t10, 8), wc.fc),
                         lerp(byte_f(t01, 8), byte_f(t11, 8), wc.fc), fr) * kInv255;
      float pnull = 1.0f - alpha;
      float pscat = (p.bounces >= P.max_bounces) ? 0.0f : alpha * albedo;
      float pabs = (1.0f - pnull) - pscat;
      STAMP(4);  // gather wait + trilinear filter + TF (LDS) + probabilities

      if (oob || wheel < pabs) {
        // exit (wgsl:142-150) or absorption (wgsl:151-155): adopt the candidate
        float rad = 0.0f;
        if (oob) {
          rad = wc.intensity;
          if (!P.light_iso) {
            float cosl = (p.dir.x * P.light_dir[0] + p.dir.y * P.light_dir[1]) + p.dir.z * P.light_dir[2];
            rad = smax(cosl * wc.intensity, 0.0f);
          }
        }
        p.samples++;
        pend_n = (float)p.samples;
        pend_l = rad;
        pend_bin = p.bin;
        p.pos = rc.pos;
        p.dir = rc.dir;
        p.bounces = 0u;
        p.lambda = rc.lambda;
        p.bin = rc.bin;
        wc = wcr;
        st = h5;
      } else if (wheel < pabs + pscat) {
        // HG scatter (wgsl:82-97, :156-160) with g from the TF blue channel
        float bch = P.b_rows ? lerp(s_brow[ri0], s_brow[ri1], fr) * kInv255
                             : lerp(lerp(byte_f(b4, 0), byte_f(b4, 8), wc.fc),
                                    lerp(byte_f(b4, 16), byte_f(b4, 24), wc.fc), fr) * kInv255;
        float g = bch * 2.0f - 1.0f;
        if (__builtin_fabsf(g) < kEps) {
          p.dir = u;
          st = h2;
        } else {
          float g2 = g * g;
          float c = (1.0f - g2) * rcp((1.0f - g) + (2.0f * g) * u3);
          float hgcos = ((1.0f + g2) - c * c) * rcp(2.0f * g);
          float sn = sqrt_cr(1.0f - hgcos * hgcos);
          p.dir = f3{sn * circle.x + hgcos * p.dir.x, sn * circle.y + hgcos * p.dir.y,
                     sn * circle.z + hgcos * p.dir.z};
          st = h3;
        }
        p.bounces++;
      } else {
        st = sw;  // null collision
      }
      STAMP(5);  // decision + adopt / HG finish
    }
    apply_pending();
  } else {
    for (uint32_t step = 0; step < P.steps; step++) {
      float dist = -spec_log(rnd_uniform(st)) * P.rcp_extinction;  // exponential.wgsl
      p.pos.x = p.pos.x + dist * p.dir.x;
      p.pos.y = p.pos.y + dist * p.dir.y;
      p.pos.z = p.pos.z + dist * p.dir.z;
      float wheel = rnd_uniform(st);  // wgsl:141 (drawn before the branch either way)
      bool oob = p.pos.x > 1.0f || p.pos.y > 1.0f || p.pos.z > 1.0f || p.pos.x < 0.0f ||
                 p.pos.y < 0.0f || p.pos.z < 0.0f;

      // sample_volume_color (wgsl:75-80); its value is unused when out of bounds.
      float pabs = 0.0f, pscat = 0.0f, fr = 0.0f;
      int ir = 0;
      if (!oob) {
        float d = sample_volume<L>(P, vol, p.pos);
        ir = axis_floor(d, 256.0f, &fr);
        uint32_t r0 = (uint32_t)clampi(ir, 255) * 256u, r1 = (uint32_t)clampi(ir + 1, 255) * 256u;
        uint32_t t00 = s_tf[r0 + wc.c0], t10 = s_tf[r0 + wc.c1];
        uint32_t t01 = s_tf[r1 + wc.c0], t11 = s_tf[r1 + wc.c1];
        float albedo = lerp(lerp(byte_f(t00, 0), byte_f(t10, 0), wc.fc),
                            lerp(byte_f(t01, 0), byte_f(t11, 0), wc.fc), fr) * kInv255;
        float alpha = lerp(lerp(byte_f(t00, 8), byte_f(t10, 8), wc.fc),
                           lerp(byte_f(t01, 8), byte_f(t11, 8), wc.fc), fr) * kInv255;
        float pnull = 1.0f - alpha;
        pscat = (p.bounces >= P.max_bounces) ? 0.0f : alpha * albedo;
        pabs = (1.0f - pnull) - pscat;
      }

      if (oob || wheel < pabs) {
        // exit (wgsl:142-150) or absorption (wgsl:151-155)
        float rad = 0.0f;
        if (oob) {  // sample_light, wgsl:62-73
          rad = wc.intensity;
          if (!P.light_iso) {
            float cosl = (p.dir.x * P.light_dir[0] + p.dir.y * P.light_dir[1]) + p.dir.z * P.light_dir[2];
            rad = smax(cosl * wc.intensity, 0.0f);
          }
        }
        p.samples++;
        float inv_n = rcp((float)p.samples);
  #pragma unroll
        for (int b = 0; b < kMaxBins; b++) {  // PhotonSpectral_add_radiance, wgsl:292-302
          if ((uint32_t)b < P.nb) {
            float tgt = ((uint32_t)b == p.bin) ? rad : 0.0f;
            p.rad[b] = p.rad[b] + (tgt - p.rad[b]) * inv_n;
          }
        }
        photon_reset(P, p, sx, sy, fixed, from, st);
        wc = wave_const(p.lambda, s_light);
      } else if (wheel < pabs + pscat) {
        // TF blue channel (wgsl:130) only where it is used
        float bch;
        if (P.b_rows) {
          bch = lerp(s_brow[clampi(ir, 255)], s_brow[clampi(ir + 1, 255)], fr) * kInv255;
        } else {
          uint32_t b4 = tf_b4[(uint32_t)clampi(ir + 1, 256) * kTfCells + (uint32_t)wc.cc];
          bch = lerp(lerp(byte_f(b4, 0), byte_f(b4, 8), wc.fc),
                     lerp(byte_f(b4, 16), byte_f(b4, 24), wc.fc), fr) * kInv255;
        }
        p.dir = sample_hg(st, bch * 2.0f - 1.0f, p.dir);  // wgsl:156-160
        p.bounces++;
      }
    }
  }

  store_state(ph, S, i, p);
#pragma unroll
  for (int b = 0; b < kMaxBins; b++) ph[(kRad0 + b) * S + i] = p.rad[b];

  // PhotonSpectral_radiance_to_rgb (wgsl:304-326) + textureStore (wgsl:168)
  float X = 0.0f, Y = 0.0f, Z = 0.0f;
#pragma unroll
  for (int b = 0; b < kMaxBins; b++) {
    if ((uint32_t)b < P.nb) {
      X = X + p.rad[b] * P.xb[b];
      Y = Y + p.rad[b] * P.yb[b];
      Z = Z + p.rad[b] * P.zb[b];
    }
  }
  float r = (3.240479f * X - 1.537150f * Y) - 0.498536f * Z;
  float g = (-0.969255f * X + 1.875990f * Y) + 0.041556f * Z;
  float bl = (0.055647f * X - 0.204041f * Y) + 1.057311f * Z;
  uint2 px;
  px.x = (uint32_t)f2h(r) | ((uint32_t)f2h(g) << 16);
  px.y = (uint32_t)f2h(bl) | (0x3c00u << 16);
  reinterpret_cast<uint2*>(rgba)[(size_t)y * P.R + x] = px;
  STAMP(6);  // epilogue: state + image stores issued
  STAMP_FLUSH();
}



// --------------------------------------------------------- volume relayout
// cell (cx,cy,cz) in [0,W]x[0,H]x[0,D] holds voxels clamp(c-1), clamp(c) per axis;
// byte (dz*4 + dy*2 + dx) of the u64 = voxel (x0+dx, y0+dy, z0+dz).
__global__ __launch_bounds__(256) void k_corner8(const uint8_t* __restrict__ lin, uint32_t W,
                                                 uint32_t H, uint32_t D, uint2* __restrict__ out) {
  const uint32_t W1 = W + 1u, H1 = H + 1u;
  const size_t ncell = (size_t)W1 * H1 * (D + 1u);
  for (size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncell;
       c += (size_t)gridDim.x * blockDim.x) {
    uint32_t cx = (uint32_t)(c % W1);
    size_t rest = c / W1;
    uint32_t cy = (uint32_t)(rest % H1);
    uint32_t cz = (uint32_t)(rest / H1);
    uint32_t x0 = clampi((int)cx - 1, (int)W - 1), x1 = clampi((int)cx, (int)W - 1);
    uint32_t y0 = clampi((int)cy - 1, (int)H - 1), y1 = clampi((int)cy, (int)H - 1);
    uint32_t z0 = clampi((int)cz - 1, (int)D - 1), z1 = clampi((int)cz, (int)D - 1);
    size_t r00 = ((size_t)z0 * H + y0) * W, r10 = ((size_t)z0 * H + y1) * W;
    size_t r01 = ((size_t)z1 * H + y0) * W, r11 = ((size_t)z1 * H + y1) * W;
    uint2 v;
    v.x = (uint32_t)lin[r00 + x0] | ((uint32_t)lin[r00 + x1] << 8) |
          ((uint32_t)lin[r10 + x0] << 16) | ((uint32_t)lin[r10 + x1] << 24);
    v.y = (uint32_t)lin[r01 + x0] | ((uint32_t)lin[r01 + x1] << 8) |
          ((uint32_t)lin[r11 + x0] << 16) | ((uint32_t)lin[r11 + x1] << 24);
    out[c] = v;
  }
}

// ----------------------------------------------------- multi-GPU composite
// (rgb * n, n) per pixel from the rgba16f target and the photon sample count.
__global__ __launch_bounds__(256) void k_pack(const MarchParams P, const float* __restrict__ ph,
                                              const uint16_t* __restrict__ rgba,
                                              float4* __restrict__ out) {
  uint32_t x, y;
  size_t i;
  if (!tile_pixel(P, x, y, i)) return;
  size_t pix = (size_t)y * P.R + x;
  uint2 px = reinterpret_cast<const uint2*>(rgba)[pix];
  float n = (float)as_u(ph[kSamples * (size_t)P.npad + i]);
  float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(px.x & 0xffffu));
  float g = (float)__builtin_bit_cast(_Float16, (uint16_t)(px.x >> 16));
  float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(px.y & 0xffffu));
  out[pix] = make_float4(r * n, g * n, b * n, n);
}

// ----------------------------------------------------------- diagnostics
__global__ void k_debug_eval(int fn, const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                             uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t v = in[i];
  float s, c;
  switch (fn) {
    case 0: out[i] = as_u(spec_log(as_f(v))); break;
    case 1: spec_sincos(as_f(v), &s, &c); out[i] = as_u(s); break;
    case 2: spec_sincos(as_f(v), &s, &c); out[i] = as_u(c); break;
    case 3: out[i] = pcg_hash(v); break;
    case 4: out[i] = f2h(as_f(v)); break;
    default: out[i] = 0u;
  }
}

}  // namespace vpt

// ------------------------------------------------------------ launchers
namespace vpt {

hipError_t launch_reset(const MarchParams& P, float* ph, hipStream_t s) {
  hipLaunchKernelGGL(k_reset, dim3(march_blocks(P)), dim3(kBlock), 0, s, P, ph);
  return hipGetLastError();
}

hipError_t launch_march(uint32_t layout, uint32_t variant, const MarchParams& P, float* ph,
                        const uint8_t* vol, const uint16_t* tf_rg, const uint32_t* tf_b4,
                        const uint8_t* tf_brow, const uint8_t* light, uint16_t* rgba,
                        hipStream_t s) {
  dim3 grid(tile_blocks(P, kMarchBlock));
#ifdef VPT_EXPERIMENTS
  {
    static uint32_t last = 0xffffffffu;
    uint32_t ko = variant & ~1u;
    if (ko != last) {
      hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_ko), &ko, sizeof ko);
      if (e != hipSuccess) return e;
      last = ko;
    }
  }
#endif
  const bool spec = (variant & 1u) == 0u;  // variant bit 0: plain (non-speculative) step
#define VPT_LAUNCH(LAY, SP)                                                                     \
  hipLaunchKernelGGL((k_march<LAY, SP>), grid, dim3(kMarchBlock), 0, s, P, ph, vol, tf_rg, tf_b4, \
                     tf_brow, light, rgba)
  if (layout == kLayoutCorner8) {
    if (spec) VPT_LAUNCH(kLayoutCorner8, true); else VPT_LAUNCH(kLayoutCorner8, false);
  } else {
    if (spec) VPT_LAUNCH(kLayoutLinear, true); else VPT_LAUNCH(kLayoutLinear, false);
  }
#undef VPT_LAUNCH
  return hipGetLastError();
}

hipError_t launch_corner8(const uint8_t* lin, uint32_t W, uint32_t H, uint32_t D, void* out,
                          hipStream_t s) {
  size_t ncell = (size_t)(W + 1) * (H + 1) * (D + 1);
  size_t blocks = (ncell + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_corner8, dim3((uint32_t)blocks), dim3(256), 0, s, lin, W, H, D,
                     reinterpret_cast<uint2*>(out));
  return hipGetLastError();
}

hipError_t launch_pack(const MarchParams& P, const float* ph, const uint16_t* rgba, float4* out,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_pack, dim3(march_blocks(P)), dim3(kBlock), 0, s, P, ph, rgba, out);
  return hipGetLastError();
}

hipError_t launch_debug_eval(int fn, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_debug_eval, dim3((n + 255) / 256), dim3(256), 0, s, fn, in, out, n);
  return hipGetLastError();
}

}  // namespace vpt

// ------------------------------------------------ exhaustive fast-math proof
// Compares a fast candidate sequence against the correctly rounded reference
// for every u32 input pattern in [lo, lo + n): the fast paths are used by the
// march only where this check finds zero mismatches (tests/test_gpu_fastmath.py).
namespace vpt {

__device__ __forceinline__ bool same_bits(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__device__ __forceinline__ float cand_eval(int fn, float x, float* ref) {
  switch (fn) {
    case 0: {  // raw v_rcp_f32 vs RN(1/x)
      *ref = 1.0f / x;
      return __builtin_amdgcn_rcpf(x);
    }
    case 1: {  // v_rcp_f32 + one FMA Newton step
      *ref = 1.0f / x;
      float y = __builtin_amdgcn_rcpf(x);
      float e = __builtin_fmaf(-x, y, 1.0f);
      return __builtin_fmaf(e, y, y);
    }
    case 2: {  // raw v_sqrt_f32 vs RN(sqrt x)
      *ref = __builtin_sqrtf(x);
      return __builtin_amdgcn_sqrtf(x);
    }
    case 3: {  // log's s = f / (2 + f) for f = x - 1: fast rcp + one residual step
      float f = x - 1.0f;
      float d = 2.0f + f;
      *ref = f / d;
      float y = __builtin_amdgcn_rcpf(d);
      float e = __builtin_fmaf(-d, y, 1.0f);
      y = __builtin_fmaf(e, y, y);
      float q = f * y;
      float r = __builtin_fmaf(-q, d, f);
      return __builtin_fmaf(r, y, q);
    }
    case 4: {  // v_sqrt_f32 + Tuckerman neighbour select (no denormal scaling)
      *ref = __builtin_sqrtf(x);
      float s0 = __builtin_amdgcn_sqrtf(x);
      float sdn = __uint_as_float(__float_as_uint(s0) - 1u);
      float sup = __uint_as_float(__float_as_uint(s0) + 1u);
      float rdn = __builtin_fmaf(-sdn, s0, x);
      float rup = __builtin_fmaf(-sup, s0, x);
      float r = s0;
      r = (rdn <= 0.0f) ? sdn : r;
      r = (rup > 0.0f) ? sup : r;
      return r;
    }
    case 6: {  // the march's RN(1/x)
      *ref = 1.0f / x;
      return rcp_cr(x);
    }
    case 7: {  // the march's RN(sqrt x)
      *ref = __builtin_sqrtf(x);
      return sqrt_cr(x);
    }
    case 8: {  // spec_log's division on its domain (x = m)
      float f = x - 1.0f;
      *ref = f / (2.0f + f);
      return log_div(f);
    }
    case 5: {  // v_sqrt_f32 + one Newton correction using the rsq estimate
      *ref = __builtin_sqrtf(x);
      float s0 = __builtin_amdgcn_sqrtf(x);
      float e = __builtin_fmaf(-s0, s0, x);
      float h = 0.5f * __builtin_amdgcn_rsqf(x);
      return __builtin_fmaf(e, h, s0);
    }
    default:
      *ref = 0.0f;
      return 0.0f;
  }
}

__global__ void k_verify(int fn, uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first,
                         uint32_t nfirst) {
  uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    float x = __uint_as_float(lo + k), ref;
    float got = cand_eval(fn, x, &ref);
    if (!same_bits(got, ref)) {
      unsigned long long idx = atomicAdd(bad, 1ull);
      if (idx < nfirst) first[idx] = lo + k;
    }
  }
}

hipError_t read_stamps(unsigned long long* out8) {
#ifdef VPT_EXPERIMENTS
  hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stamp), 8 * sizeof(unsigned long long));
  unsigned long long z[16] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof z);
  return e;
#else
  for (int k = 0; k < 8; k++) out8[k] = 0;
  return hipSuccess;
#endif
}

hipError_t launch_verify(int fn, uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first,
                         uint32_t nfirst, hipStream_t s) {
  hipLaunchKernelGGL(k_verify, dim3(8192), dim3(256), 0, s, fn, lo, n, bad, first, nfirst);
  return hipGetLastError();
}

}  // namespace vpt
