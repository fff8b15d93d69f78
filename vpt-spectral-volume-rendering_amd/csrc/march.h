// march.h — the spectral MCM photon march and photon reset for gfx950.
//
// One lane owns one photon (= one pixel), exactly like the reference's
// compute_main (MCMSpectralComputeRenderer.wgsl:107-179 render, :213-231
// reset). What is MI355X-specific is the data layout, the mapping and the
// instruction diet of the divergent paths:
//   * photon state is stored as SoA planes of 32-bit words in "wave-tile"
//     order — wave w of the grid owns an 8x8 pixel tile and lane
//     l = 8*ly + lx its pixel — so every plane load/store is one fully
//     coalesced 256-B wave access and a wave's rays start in a compact
//     screen-space footprint (volume gathers hit the same cache lines);
//   * the volume is either x-fastest u8 (LINEAR) or CORNER8: one u64 per
//     trilinear cell holding its 8 corner voxels, so the 2x2x2 stencil is a
//     single 8-B load instead of 8 byte gathers;
//   * blocks are remapped so consecutive tiles run on the same XCD;
//   * a wave of 64 photons almost always has some lane exiting/absorbing and
//     some lane scattering in every step, so the wave pays for the reset and
//     scatter paths nearly every step: they are kept short — one correctly
//     rounded reciprocal per divisor (the spec's division), a branchless bin
//     search, the per-pixel near point hoisted out of the loop when blur = 0,
//     and the per-wavelength TF column / light terms cached per photon.
//   All of these are value-preserving: results are bit-identical to the oracle.
#pragma once

#include "mcm_device.h"

namespace vpt {

enum : uint32_t { kLayoutLinear = 0, kLayoutCorner8 = 1, kLayoutBrick8 = 2, kLayoutColumn4 = 3 };
// Kernel template layouts: CORNER8 / BRICK8 / COLUMN4 with 32-bit byte offsets
// (MarchParams::vol32) or with 64-bit ones (cell arrays over 4 GiB, e.g. 1024^3).
enum : uint32_t {
  kTplLinear = 0, kTplCorner8 = 1, kTplCorner8Wide = 2, kTplBrick8 = 3, kTplBrick8Wide = 4,
  kTplColumn4 = 5, kTplColumn4Wide = 6
};
// COLUMN4: per (cx, cy) cell column the D + 2 quads q(k) = the 2x2 corner
// voxels (clamped x cx-1 .. cx, y cy-1 .. cy) at z = clamp(k - 1), as u32 in
// CORNER8's byte order (dy * 2 + dx), z fastest: the CORNER8 cell
// (cx, cy, cz) is q(cz) | q(cz + 1) << 32, the 8 bytes at quad index cz of its
// column — one 4-B-aligned 8-B load per sample from half CORNER8's footprint
// (4 B per cell: 541 MB at 512^3, 4.3 GB at 1024^3).
// BRICK8: the CORNER8 cells grouped into 4x4x4-cell bricks of 512 B (bricks in
// raster order, x fastest); inside a brick the cell index interleaves the
// coordinate bits as (x0 x1 y0 z0 y1 z1), so one 128-B line holds a 4x2x2 cell
// block (5x3x3 voxels) instead of a 16x1x1 row.
constexpr uint32_t kBrickCells = 4;  // cells per brick edge
__host__ __device__ __forceinline__ uint32_t brick_inner(uint32_t cx, uint32_t cy, uint32_t cz) {
  return (cx & 3u) | ((cy & 1u) << 2) | ((cz & 1u) << 3) | ((cy & 2u) << 3) | ((cz & 2u) << 4);
}

// Plane indices of the SoA photon buffer.
enum Plane : uint32_t {
  kPx = 0, kPy, kPz, kDx, kDy, kDz, kBounces, kSamples, kBin, kLambda, kRad0, kNumPlanes = kRad0 + kMaxBins
};
// Planes of the RGB sibling's photon (Photon.wgsl): the first eight coincide.
enum RgbPlane : uint32_t { kTr0 = 8, kRgbRad0 = 11, kRgbPlanes = 14 };
constexpr uint32_t kRgbTfMax = 4096;  // TF texels staged in LDS (row 0, decoded float4)

constexpr int kRbEdges = 8;  // MarchParams::rb_edge (a projected box has at most 6 hull edges)

struct MarchParams {
  float m[16];           // mvpInverse, column-major
  float inv_res[2];      // 1/R as f32 (js:297)
  uint32_t seed;         // bitcast<u32>(randSeed)
  float blur;
  float extinction;
  float rcp_extinction;  // RN(1/extinction): exponential.wgsl's division
  uint32_t max_bounces;
  uint32_t steps;
  uint32_t nb;           // u32(spectrum[0] + 0.5)
  uint32_t bins_sorted;  // lam[1..nb-1] non-decreasing: branchless bin search valid
  // sorted, every boundary and max - min finite: the count runs over 11
  // boundaries unrolled, with lam_pad[i] = +inf for i >= nb (no trip loop)
  uint32_t bins_padded;
  float lam_pad[kMaxBins];
  uint32_t bins_uniform; // lam[i] == fma(f32(i), bin_w, lam[0]) exactly: arithmetic bin
  float bin_w, rcp_bin_w;
  float lam[13];         // spectrum[1 .. 13]: bin boundaries
  float min_lam, max_lam; // spectrum[1], spectrum[nb + 1] (wgsl:262-263)
  float xb[kMaxBins], yb[kMaxBins], zb[kMaxBins];  // CMF bin means (0 past nb)
  float light_dir[3];    // normalize(light_direction) (host-computed, IEEE)
  float anisotropy;      // RGB sibling: the HG g uniform (MCMComputeRenderer.wgsl:140)
  uint32_t tf_w;         // RGB sibling: TF width (texels of row 0 in LDS)
  float env[4];          // RGB sibling: the 1x1 environment texel, unorm -> f32
  uint32_t light_iso;    // length(light_direction) < EPS
  uint32_t b_rows;       // TF blue channel column-invariant: use the LDS row table
  uint32_t sched;        // march tile mapping: 0 scheduled (TileSched flags, slots round-robin over
                         // the XCDs), 1 raster, 2 scheduled XCD by XCD (round 2's order)
  // Robust-miss screen region (NDC, host-derived from the forward matrix):
  // with blur 0, every ray of a pixel whose centre lies outside
  // [rb_x0, rb_x1] x [rb_y0, rb_y1], or beyond one of the rb_edge lines
  // (a * sx + b * sy > c: the edges of the convex hull of the expanded cube's
  // projected corners, padded; unused edges have c = FLT_MAX), misses the unit
  // cube by a margin, so each of its steps is an exit (see k_march's robust
  // path; robust_pixel).
  uint32_t robust;
  float rb_x0, rb_x1, rb_y0, rb_y1;
  float rb_edge[kRbEdges][3];
  uint32_t R, tiles_x, n_tiles, npad;
  uint32_t band_y0, band_y1;  // pixel rows [band_y0, band_y1) this renderer owns (Mode B)
  uint32_t W, H, D;
  // CORNER8 cell byte offsets fit 32 bits ((W+1)(H+1)(D+1) * 8 < 2^32 and
  // (D+1)(H+1) < 2^24): the gather address is u24 multiply-adds on a 32-bit
  // offset from the SGPR base instead of a 64-bit multiply chain
  uint32_t vol32;
  uint32_t BW, BH;  // BRICK8: bricks along x and y (ceil((W+1)/4), ceil((H+1)/4))
  // |w| of every unprojected point < 2^120 (host bound from the matrix, the
  // resolution and blur): a precondition of the FAST march specialisation
  uint32_t w_bounded;
  // Row-deduplicated TF (set by launch_march for non-FAST launches): the LDS TF
  // holds the TF's distinct density rows as u32 texels (albedo | alpha << 8 |
  // anisotropy << 16) and s_rowmap maps a density row to its distinct row, so
  // the anisotropy taps come from LDS with albedo and alpha (no tf_b4 gather).
  uint32_t tf_dedup;
  // The bin as a function of the wavelength draw h5 (lambda_of is monotone in
  // h5 and the bin in lambda, so bin(h5) is a step function): per cell of
  // 2^22 draws the bin at the cell start and the one threshold inside it,
  // host-built and exact (kBinLutCells u32 thresholds, then as many bytes of
  // base | count << 4). Set when no cell holds two distinct thresholds.
  uint32_t bins_lut;
  // Dark background (k_march, FAST geometry): waves whose every sample is
  // provably +0 run the draw chain alone (1, the default); 0 off (VPTMCM_DARK).
  uint32_t dark;
  // Completion signal (TileSched::done_ctr / done_flag): the cumulative wave
  // count after this launch and the value its last wave writes to the flag.
  uint32_t done_target, done_seq;
  // The handle's march launch count including this one, and whether this
  // launch may keep the previous launch's tile deal (TileSched::changed_in):
  // 1 unless the host touched the schedule state since (first launch,
  // VPTMCM_SCHED_CACHE=0).
  uint32_t launch_seq, sched_reuse;
  // Macro-cell alpha bound (k_march's certain null collisions, MODE-independent):
  // texel cells (cx, cy, cz) >> maj_shift index a maj_nx x maj_ny x maj_nz table
  // of 4-bit codes q (two per byte, maj_bytes staged in LDS, a multiple of 16),
  // each with q * 17 >= every alpha byte of every TF texel a sample in those
  // cells can reach; a lane whose wheel draw clears the code's bound takes the
  // null collision without the volume gather (same decision, kernels.hip
  // maj_threshold). maj_on 0: no table.
  uint32_t maj_on, maj_shift, maj_nx, maj_ny, maj_bytes;
};
// Byte capacity of the LDS macro table (nibbles: 40,960 macro cells, e.g. 33^3
// cells of 16^3 texel cells at 512^3)
constexpr uint32_t kMajBytes = 20480;
constexpr uint32_t kBinLutCells = 1024u;
constexpr uint32_t kBinLutShift = 22u;

// ---------------------------------------------------------------- RNG draws
// disk.wgsl from its two hash draws
__device__ __forceinline__ void disk_of(uint32_t h1, uint32_t h2, float& dx, float& dy) {
  float radius = sqrt_z((float)h1 * 2.3283064365386963e-10f);
  float angle = kTwoPi * ((float)h2 * 2.3283064365386963e-10f);
  float s, c;
  spec_sincos(angle, &s, &c);
  dx = radius * c;
  dy = radius * s;
}
__device__ __forceinline__ void rnd_disk(uint32_t& st, float& dx, float& dy) {  // disk.wgsl
  uint32_t h1 = pcg_hash(st);
  st = pcg_hash(h1);
  disk_of(h1, st, dx, dy);
}
__device__ __forceinline__ f3 rnd_sphere(uint32_t& st) {  // sphere.wgsl:4-10
  float dx, dy;
  rnd_disk(st, dx, dy);
  float nrm = fmaf(dy, dy, dx * dx);
  float radius = 2.0f * sqrt_z(1.0f - nrm);
  float z = 1.0f - 2.0f * nrm;
  return f3{radius * dx, radius * dy, z};
}

// sampleHenyeyGreenstein{AngleCosine}, wgsl:82-97
__device__ __forceinline__ f3 sample_hg(uint32_t& st, float g, f3 dir) {
  f3 u = rnd_sphere(st);
  if (__builtin_fabsf(g) < kEps) return u;
  float g2 = g * g;
  float c = (1.0f - g2) * rcp_small(fmaf(2.0f * g, rnd_uniform(st), 1.0f - g));
  float hgcos = fmaf(-c, c, 1.0f + g2) * rcp_small(2.0f * g);
  float ud = dot3(u, dir);
  f3 circle = norm3(f3{fmaf(-ud, dir.x, u.x), fmaf(-ud, dir.y, u.y), fmaf(-ud, dir.z, u.z)});
  float sn = sqrt_z(fmaf(-hgcos, hgcos, 1.0f));
  return f3{fmaf(sn, circle.x, hgcos * dir.x), fmaf(sn, circle.y, hgcos * dir.y),
            fmaf(sn, circle.z, hgcos * dir.z)};
}

// Per-photon wavelength constants: TF column taps + weight, and the light
// intensity textureSampleLevel(uLightSpectrum, (t, .5)).r * 5 (wgsl:64-65).
struct WaveConst {
  int c0, c1;     // clamped column taps
  int cc;         // column cell of the 4-corner b table: clamp(ic, -1, 255) + 1
  float fc;
  float intensity;
};
__device__ __forceinline__ WaveConst wave_const(float lambda, const float* s_light) {
  float t = (lambda - 400.0f) * rcp(700.0f - 400.0f);  // wgsl:64 == wgsl:77
  WaveConst w;
  int ic = axis_floor(t, 256.0f, &w.fc);
  w.c0 = clampi(ic, 255);
  w.c1 = clampi(ic + 1, 255);
  w.cc = clampi(ic + 1, 256);
  w.intensity = lerp(s_light[w.c0], s_light[w.c1], w.fc) * kInv255 * 5.0f;
  return w;
}

// PhotonSpectral_set_wavelength, wgsl:276-290. For non-decreasing boundaries
// the first i with lambda < lam[i] is 1 + #{i : !(lambda < lam[i])}, so the
// search is a branchless count; otherwise the sequential first-match search.
// UNI: the launch's host check guarantees bins_uniform, nb >= 1, w_bounded,
// blur == 0 and an even R (the FAST march specialisation), so the arithmetic
// path is taken without the branches.
template <bool UNI = false>
__device__ __forceinline__ uint32_t bin_of(const MarchParams& P, float lambda) {
  if (!UNI && P.nb == 0u) return 0xffffffffu;  // nb - 1 wraps (first-reset quirk)
  uint32_t bin;
  if (UNI || P.bins_uniform) {
    // Host-verified: lam[i] == fma(f32(i), w, lam0) for i <= nb, lam0 > 0,
    // lam[nb] <= 2 lam0 (so lambda - lam0 is exact). The candidate
    // floor((lambda - lam0) * RN(1/w)) is within one bin of the count, and
    // two exact comparisons against the boundaries fix it.
    float q = (lambda - P.lam[0]) * P.rcp_bin_w;
    int k = (int)__builtin_floorf(q);
    k = k < 0 ? 0 : (k > (int)P.nb - 1 ? (int)P.nb - 1 : k);
    float kf = (float)k;
    float lo = fmaf(kf, P.bin_w, P.lam[0]);
    float hi = fmaf(kf + 1.0f, P.bin_w, P.lam[0]);
    // (lambda < lo) ? k - 1 : (!(lambda < hi) && k + 1 < nb) ? k + 1 : k,
    // as arithmetic on the compare bits (the ternary chain compiles to
    // exec-mask branches)
    const bool dn = lambda < lo;
    const bool up = !(lambda < hi) & (k + 1 < (int)P.nb) & !dn;
    return (uint32_t)(k - (int)dn + (int)up);
  }
  if (P.bins_sorted && P.bins_padded) {
    // every lambda is finite here, so !(lambda < +inf) adds nothing past nb - 1
    bin = 0u;
#pragma unroll
    for (int i = 1; i < kMaxBins; i++) bin += !(lambda < P.lam_pad[i]) ? 1u : 0u;
  } else if (P.bins_sorted) {
    // uniform trip count (nb - 1): no per-bin masks held live across the
    // march (they used to spill 22 SGPRs into VGPR lanes)
    bin = 0u;
    const uint32_t nb = __builtin_amdgcn_readfirstlane(P.nb);
    for (uint32_t i = 1u; i < nb; i++) bin += !(lambda < P.lam[i]) ? 1u : 0u;
  } else {
    bin = P.nb - 1u;
    for (uint32_t i = 1u; i < P.nb; i++) {
      if (lambda < P.lam[i]) {
        bin = i - 1u;
        break;
      }
    }
  }
  return bin;
}

struct Photon {
  f3 pos, dir;
  uint32_t bounces, samples, bin;
  float lambda;
  float rad[kMaxBins];
};

// near point of the camera ray: M * (screen + disk*blur, -1, 1), divided by w.
// WB: the host has bounded |w| < 2^120 for every (a, b) the launch can produce
// (MarchParams::w_bounded), so rcp_small's one-compare guard suffices.
template <bool WB = false>
__device__ __forceinline__ f3 unproject(const float* m, float a, float b, float z) {
  float d[4];
#pragma unroll
  for (int r = 0; r < 4; r++) d[r] = fmaf(m[12 + r], 1.0f, fmaf(m[8 + r], z, fmaf(m[4 + r], b, m[r] * a)));
  float iw = WB ? rcp_small(d[3]) : rcp(d[3]);
  return f3{d[0] * iw, d[1] * iw, d[2] * iw};
}

// PhotonSpectral_reset, wgsl:249-266 (+ unprojectRand.wgsl, intersectCube.wgsl).
// fixed_from: blur == 0 and the screen position has no zero coordinate, so
// screen + disk*0 == screen exactly and the near point is the per-pixel
// constant `from`; the two disk draws are still consumed.
__device__ __forceinline__ void photon_reset(const MarchParams& P, Photon& p, float sx, float sy,
                                             bool fixed_from, f3 from, uint32_t& st) {
  if (fixed_from) {
    st = pcg_hash(pcg_hash(st));
  } else {
    float dx, dy;
    rnd_disk(st, dx, dy);
    from = unproject(P.m, fmaf(dx, P.blur, sx), fmaf(dy, P.blur, sy), -1.0f);
  }
  float q0 = rnd_uniform(st);
  float q1 = rnd_uniform(st);
  f3 to = unproject(P.m, fmaf(fmaf(q0, 2.0f, -1.0f), P.inv_res[0], sx),
                    fmaf(fmaf(q1, 2.0f, -1.0f), P.inv_res[1], sy), 1.0f);
  f3 dir = norm3(f3{to.x - from.x, to.y - from.y, to.z - from.z});
  p.dir = dir;
  p.bounces = 0u;
  float rx = rcp_small(dir.x), ry = rcp_small(dir.y), rz = rcp_small(dir.z);
  float t1x = smin((0.0f - from.x) * rx, (1.0f - from.x) * rx);
  float t1y = smin((0.0f - from.y) * ry, (1.0f - from.y) * ry);
  float t1z = smin((0.0f - from.z) * rz, (1.0f - from.z) * rz);
  float tn = smax(smax(smax(t1x, t1y), t1z), 0.0f);
  p.pos = f3{fmaf(tn, dir.x, from.x), fmaf(tn, dir.y, from.y), fmaf(tn, dir.z, from.z)};
  float lambda = fmaf(rnd_uniform(st), P.max_lam - P.min_lam, P.min_lam);
  p.lambda = lambda;
  p.bin = bin_of(P, lambda);
}

// The pieces of PhotonSpectral_reset (wgsl:249-266) from pre-drawn hashes:
// h1,h2 are the disk draws (already turned into dx, dy), h3,h4 the square,
// h5 the wavelength.
// Direction of the new camera ray: normalize(far - near) (unprojectRand.wgsl).
template <bool WB = false>
__device__ __forceinline__ f3 ray_dir_from_draws(const MarchParams& P, float sx, float sy, f3 from,
                                                 uint32_t h3, uint32_t h4) {
  float q0 = (float)h3 * 2.3283064365386963e-10f;
  float q1 = (float)h4 * 2.3283064365386963e-10f;
  f3 to = unproject<WB>(P.m, fmaf(fmaf(q0, 2.0f, -1.0f), P.inv_res[0], sx),
                    fmaf(fmaf(q1, 2.0f, -1.0f), P.inv_res[1], sy), 1.0f);
  return norm3(f3{to.x - from.x, to.y - from.y, to.z - from.z});
}
// Start point on the ray with hardware min/max3: valid when no slab distance
// is zero, i.e. no coordinate of `from` is exactly 0 or 1 (then every
// (c - from)*RN(1/d) is a non-zero number, an infinity or a quiet NaN, and
// v_min/v_max/v_max3 return what smin/smax do; see hw_min).
// omf = 1 - from (a per-pixel constant the caller keeps in registers); with
// from != 0, 0 - from is exactly -from (a free negation modifier).
__device__ __forceinline__ f3 ray_start_hw(f3 from, f3 omf, f3 dir) {
  // the three reciprocals share one wave-uniform range guard (rcp_small's)
  float rx = rcp_in_range(dir.x), ry = rcp_in_range(dir.y), rz = rcp_in_range(dir.z);
  {
    const bool bx = !(__builtin_fabsf(dir.x) >= 1.17549435e-38f);
    const bool by = !(__builtin_fabsf(dir.y) >= 1.17549435e-38f);
    const bool bz = !(__builtin_fabsf(dir.z) >= 1.17549435e-38f);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bx | by | bz) != 0ull, 0)) {
      rx = bx ? rcp_slow(dir.x) : rx;
      ry = by ? rcp_slow(dir.y) : ry;
      rz = bz ? rcp_slow(dir.z) : rz;
    }
  }
  // (on arithmetic results: plain v_min/v_max/v_max3, no canonicalisation)
  float t1x = hw_min(-from.x * rx, omf.x * rx);
  float t1y = hw_min(-from.y * ry, omf.y * ry);
  float t1z = hw_min(-from.z * rz, omf.z * rz);
  float tn = hw_max(hw_max3(t1x, t1y, t1z), 0.0f);
  return f3{fmaf(tn, dir.x, from.x), fmaf(tn, dir.y, from.y), fmaf(tn, dir.z, from.z)};
}
// A lane whose near point is fixed and has no coordinate equal to 0 or 1.
__device__ __forceinline__ bool slab_generic(bool fixed_from, f3 from) {
  return fixed_from && from.x != 0.0f && from.x != 1.0f && from.y != 0.0f && from.y != 1.0f &&
         from.z != 0.0f && from.z != 1.0f;
}
// Start point on the ray: from + max(tnear, 0) * dir (intersectCube.wgsl, wgsl:254-256).
__device__ __forceinline__ f3 ray_start(f3 from, f3 dir) {
  float rx = rcp_small(dir.x), ry = rcp_small(dir.y), rz = rcp_small(dir.z);
  float t1x = smin((0.0f - from.x) * rx, (1.0f - from.x) * rx);
  float t1y = smin((0.0f - from.y) * ry, (1.0f - from.y) * ry);
  float t1z = smin((0.0f - from.z) * rz, (1.0f - from.z) * rz);
  float tn = smax(smax(smax(t1x, t1y), t1z), 0.0f);
  return f3{fmaf(tn, dir.x, from.x), fmaf(tn, dir.y, from.y), fmaf(tn, dir.z, from.z)};
}
// Wavelength and bin (PhotonSpectral_set_wavelength, wgsl:276-290).
__device__ __forceinline__ float lambda_of(const MarchParams& P, uint32_t h5) {
  return fmaf((float)h5 * 2.3283064365386963e-10f, P.max_lam - P.min_lam, P.min_lam);
}

// bin_of(lambda_of(h5)); LUTB: from the LDS copy of MarchParams::bins_lut's
// table (lut: kBinLutCells thresholds, then the base | count << 4 bytes).
template <bool UNIB = false, bool LUTB = false>
__device__ __forceinline__ uint32_t bin_of_draw(const MarchParams& P, float lambda, uint32_t h5,
                                                const uint32_t* lut) {
  if constexpr (LUTB) {
    const uint32_t c = h5 >> kBinLutShift;
    const uint32_t t = lut[c];
    const uint32_t bk = reinterpret_cast<const uint8_t*>(lut + kBinLutCells)[c];
    return (bk & 15u) + (h5 >= t ? (bk >> 4) : 0u);
  } else {
    return bin_of<UNIB>(P, lambda);
  }
}

// UNI: blur 0, even R and a host-bounded |w| (fixed near points, one-compare
// reciprocal guard); UNIB: equal-width bins (bin_of's arithmetic path).
template <bool UNI = false, bool UNIB = UNI, bool LUTB = false>
__device__ __forceinline__ void reset_from_draws(const MarchParams& P, Photon& p, float sx, float sy,
                                                 bool fixed_from, f3 from, float dx, float dy,
                                                 uint32_t h3, uint32_t h4, uint32_t h5,
                                                 bool slab_hw = false, f3 omf = f3{0.0f, 0.0f, 0.0f},
                                                 const uint32_t* lut = nullptr) {
  // UNI launches have blur == 0 and an even R, so every near point is fixed
  // (screen coordinates of pixel centres are never 0 then)
  if constexpr (!UNI) {
    if (!fixed_from) from = unproject(P.m, fmaf(dx, P.blur, sx), fmaf(dy, P.blur, sy), -1.0f);
  }
  p.dir = ray_dir_from_draws<UNI>(P, sx, sy, from, h3, h4);
  if (slab_hw)  // wave-uniform: every lane's from is slab_generic, omf = 1 - from
    p.pos = ray_start_hw(from, omf, p.dir);
  else
    p.pos = ray_start(from, p.dir);
  p.lambda = lambda_of(P, h5);
  p.bin = bin_of_draw<UNIB, LUTB>(P, p.lambda, h5, lut);
}

__device__ __forceinline__ void screen_of(const MarchParams& P, uint32_t x, uint32_t y, float& sx,
                                          float& sy) {  // wgsl:118
  sx = fmaf((float)x + 0.5f, P.inv_res[0], -0.5f) * 2.0f;
  sy = fmaf((float)y + 0.5f, P.inv_res[1], -0.5f) * -2.0f;
}

// Consecutive logical blocks -> same XCD (blocks are dealt round-robin over 8).
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nblocks) {
  if ((nblocks & 7u) != 0u) return b;
  return (b & 7u) * (nblocks >> 3) + (b >> 3);
}

}  // namespace vpt
