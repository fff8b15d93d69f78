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

__device__ __forceinline__ bool tile_pixel(const MarchParams& P, uint32_t& x, uint32_t& y,
                                           size_t& idx) {
  uint32_t b = xcd_swizzle(blockIdx.x, gridDim.x);
  uint32_t tile = b * (kBlock / 64) + (threadIdx.x >> 6);
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
template <uint32_t L>
__device__ __forceinline__ float sample_volume(const MarchParams& P, const uint8_t* __restrict__ vol,
                                               f3 q) {
  float fx, fy, fz;
  int ix = axis_floor(q.x, (float)P.W, &fx);
  int iy = axis_floor(q.y, (float)P.H, &fy);
  int iz = axis_floor(q.z, (float)P.D, &fz);
  float v000, v100, v010, v110, v001, v101, v011, v111;
  if constexpr (L == kLayoutCorner8) {
    const uint32_t W1 = P.W + 1u, H1 = P.H + 1u;
    uint32_t cx = (uint32_t)(clampi(ix + 1, (int)P.W));
    uint32_t cy = (uint32_t)(clampi(iy + 1, (int)P.H));
    uint32_t cz = (uint32_t)(clampi(iz + 1, (int)P.D));
    size_t cell = ((size_t)cz * H1 + cy) * W1 + cx;
    uint2 c = reinterpret_cast<const uint2*>(vol)[cell];
    v000 = (float)(c.x & 0xffu);
    v100 = (float)((c.x >> 8) & 0xffu);
    v010 = (float)((c.x >> 16) & 0xffu);
    v110 = (float)(c.x >> 24);
    v001 = (float)(c.y & 0xffu);
    v101 = (float)((c.y >> 8) & 0xffu);
    v011 = (float)((c.y >> 16) & 0xffu);
    v111 = (float)(c.y >> 24);
  } else {
    const int wm = (int)P.W - 1, hm = (int)P.H - 1, dm = (int)P.D - 1;
    uint32_t x0 = clampi(ix, wm), x1 = clampi(ix + 1, wm);
    uint32_t y0 = clampi(iy, hm), y1 = clampi(iy + 1, hm);
    uint32_t z0 = clampi(iz, dm), z1 = clampi(iz + 1, dm);
    size_t r00 = ((size_t)z0 * P.H + y0) * P.W, r10 = ((size_t)z0 * P.H + y1) * P.W;
    size_t r01 = ((size_t)z1 * P.H + y0) * P.W, r11 = ((size_t)z1 * P.H + y1) * P.W;
    v000 = (float)vol[r00 + x0];
    v100 = (float)vol[r00 + x1];
    v010 = (float)vol[r10 + x0];
    v110 = (float)vol[r10 + x1];
    v001 = (float)vol[r01 + x0];
    v101 = (float)vol[r01 + x1];
    v011 = (float)vol[r11 + x0];
    v111 = (float)vol[r11 + x1];
  }
  float c00 = lerp(v000, v100, fx);
  float c10 = lerp(v010, v110, fx);
  float c01 = lerp(v001, v101, fx);
  float c11 = lerp(v011, v111, fx);
  float c0 = lerp(c00, c10, fy);
  float c1 = lerp(c01, c11, fy);
  return lerp(c0, c1, fz) * kInv255;
}

__device__ __forceinline__ float tf_chan(uint32_t a, uint32_t b, int sh, float f) {
  return lerp((float)((a >> sh) & 0xffu), (float)((b >> sh) & 0xffu), f);
}

// ------------------------------------------------------------- march kernel
template <uint32_t L>
__global__ __launch_bounds__(kBlock) void k_march(const MarchParams P, float* __restrict__ ph,
                                                  const uint8_t* __restrict__ vol,
                                                  const uint32_t* __restrict__ tf,
                                                  const uint8_t* __restrict__ light,
                                                  uint16_t* __restrict__ rgba) {
  __shared__ float s_light[256];
  for (uint32_t t = threadIdx.x; t < 256u; t += kBlock) s_light[t] = (float)light[t];
  __syncthreads();

  uint32_t x, y;
  size_t i;
  if (!tile_pixel(P, x, y, i)) return;
  const size_t S = P.npad;
  float sx, sy;
  screen_of(P, x, y, sx, sy);

  f3 from{0.0f, 0.0f, 0.0f};
  bool fixed = near_fixed(P, sx, sy, from);
  Photon p;
  load_photon(ph, S, i, p);
  WaveConst wc = wave_const(p.lambda, s_light);
  uint32_t st = hash3(x, y, P.seed);  // wgsl:122 (state is not carried across passes)

  for (uint32_t step = 0; step < P.steps; step++) {
    float dist = -spec_log(rnd_uniform(st)) * P.rcp_extinction;  // exponential.wgsl
    p.pos.x = p.pos.x + dist * p.dir.x;
    p.pos.y = p.pos.y + dist * p.dir.y;
    p.pos.z = p.pos.z + dist * p.dir.z;
    float wheel = rnd_uniform(st);  // wgsl:141 (drawn before the branch either way)
    bool oob = p.pos.x > 1.0f || p.pos.y > 1.0f || p.pos.z > 1.0f || p.pos.x < 0.0f ||
               p.pos.y < 0.0f || p.pos.z < 0.0f;

    // sample_volume_color (wgsl:75-80); its value is unused when out of bounds.
    float pabs = 0.0f, pscat = 0.0f, aniso = 0.0f;
    if (!oob) {
      float d = sample_volume<L>(P, vol, p.pos);
      float fr;
      int ir = axis_floor(d, 256.0f, &fr);
      uint32_t r0 = (uint32_t)clampi(ir, 255) * 256u, r1 = (uint32_t)clampi(ir + 1, 255) * 256u;
      uint32_t t00 = tf[r0 + wc.c0], t10 = tf[r0 + wc.c1];
      uint32_t t01 = tf[r1 + wc.c0], t11 = tf[r1 + wc.c1];
      float albedo = lerp(tf_chan(t00, t10, 0, wc.fc), tf_chan(t01, t11, 0, wc.fc), fr) * kInv255;
      float alpha = lerp(tf_chan(t00, t10, 8, wc.fc), tf_chan(t01, t11, 8, wc.fc), fr) * kInv255;
      float bch = lerp(tf_chan(t00, t10, 16, wc.fc), tf_chan(t01, t11, 16, wc.fc), fr) * kInv255;
      aniso = bch * 2.0f - 1.0f;
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
      p.dir = sample_hg(st, aniso, p.dir);  // wgsl:156-160
      p.bounces++;
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
}

template __global__ void k_march<kLayoutLinear>(const MarchParams, float*, const uint8_t*,
                                                const uint32_t*, const uint8_t*, uint16_t*);
template __global__ void k_march<kLayoutCorner8>(const MarchParams, float*, const uint8_t*,
                                                 const uint32_t*, const uint8_t*, uint16_t*);

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

hipError_t launch_march(uint32_t layout, const MarchParams& P, float* ph, const uint8_t* vol,
                        const uint32_t* tf, const uint8_t* light, uint16_t* rgba, hipStream_t s) {
  if (layout == kLayoutCorner8)
    hipLaunchKernelGGL(k_march<kLayoutCorner8>, dim3(march_blocks(P)), dim3(kBlock), 0, s, P, ph,
                       vol, tf, light, rgba);
  else
    hipLaunchKernelGGL(k_march<kLayoutLinear>, dim3(march_blocks(P)), dim3(kBlock), 0, s, P, ph,
                       vol, tf, light, rgba);
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
