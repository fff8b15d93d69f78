// kernels.h — launch interface of the gfx950 kernels (kernels.hip) used by
// the C-ABI implementation (vptmcm.cpp).
#pragma once

#include <cstddef>

#include <hip/hip_ext.h>

#include "march.h"

namespace vpt {

constexpr uint32_t kBlock = 256;        // reset/pack: 4 waves, each one 8x8 pixel tile
constexpr uint32_t kMarchBlock = 1024;  // march: 16 waves share the LDS copy of the TF

inline uint32_t tile_blocks(const MarchParams& P, uint32_t block) {
  return (P.n_tiles + (block / 64) - 1) / (block / 64);
}
inline uint32_t march_blocks(const MarchParams& P) { return tile_blocks(P, kBlock); }

// TF re-layouts (built on the host by vptmcm_set_material_tf):
//   tf_rg  u16[256*256]: (albedo | alpha << 8) per texel — staged in LDS (128 KB)
//   tf_b4  u32[257*257]: the 4 anisotropy corners of each bilinear cell
//   tf_brow u8[256]: anisotropy per row when it does not vary with wavelength
constexpr uint32_t kTfCells = 257;
constexpr uint32_t kTfRowsMax = 128;  // distinct TF rows the LDS holds as u32 texels (128 KB)

// Per-pass tile schedule of the march (see schedule_tile in kernels.hip): one
// byte per tile, written by the pass ("its wave entered the volume") and read
// by the next pass to deal volume tiles evenly over the SIMDs.
struct TileSched {
  const uint8_t* flags_in;
  uint8_t* flags_out;
  // per wave slot (block * 16 + wave) the packed tile the schedule gave it last
  // launch (tile | flag << 31, 0xffffffff idle): a hot wave starts loading that
  // tile's photon state before its own schedule ends, and reloads on a change
  uint32_t* prev;
  // Completion signal (vptmcm_synchronize): every wave of the launch adds 1 to
  // done_ctr (device memory, cumulative over launches) once its stores have
  // landed; the wave that brings it to MarchParams::done_target writes
  // MarchParams::done_seq to done_flag, a word of fine-grained host memory the
  // host polls. Null: no signal.
  uint32_t* done_ctr;
  uint32_t* done_flag;
  // (rgb * n, n) per pixel of the launch's last pass (k_pack's values, written
  // with the image; the cross-rank composite's buffer), or null
  float4* pack;
  // Deal reuse: a wave whose tile's flag changed writes the launch's
  // MarchParams::launch_seq to changed_out; the next launch reads it as
  // changed_in (the two words alternate like the flag rows). A launch whose
  // predecessor changed no flag deals exactly what that launch dealt (the
  // deal is a function of the flags alone), so it takes each slot's tile from
  // prev instead of running the schedule.
  const uint32_t* changed_in;
  uint32_t* changed_out;
};
// Flag byte of a tile (written by each launch for the next one's schedule):
// bit 0 its wave entered the volume.
constexpr uint32_t kFlagVolume = 1u;
constexpr uint32_t kSchedChunk = 4 * kMarchBlock;  // tiles scanned per block-wide round
constexpr uint32_t kSchedMaxTiles = 16384;         // larger frames use the raster mapping
// Seeds of the passes one march launch runs back to back (render_passes): the
// photon state stays in registers between them; every pass reseeds the RNG
// from its own seed (wgsl:122). A launch runs n <= kMaxFusedPasses passes.
constexpr uint32_t kMaxFusedPasses = 32;
struct PassSeeds {
  uint32_t n;
  uint32_t pad;
  uint32_t seed[kMaxFusedPasses];
};
static_assert(offsetof(PassSeeds, seed) == 8, "pass_seed() reads seed[] at kernarg byte 8");
// k_march(PassSeeds, MarchParams, ...): MarchParams starts right after PassSeeds
static_assert(sizeof(PassSeeds) % alignof(MarchParams) == 0, "MarchParams kernarg offset");
static_assert(offsetof(MarchParams, yb) == offsetof(MarchParams, xb) + 4 * kMaxBins &&
                  offsetof(MarchParams, zb) == offsetof(MarchParams, yb) + 4 * kMaxBins,
              "cmf_table() reads xb, yb, zb contiguously");
inline uint32_t sched_flag_bytes(uint32_t n_tiles) {
  return (n_tiles + kSchedChunk - 1) / kSchedChunk * kSchedChunk;
}
inline uint32_t sched_slot_words(uint32_t n_tiles) {  // TileSched::prev: 16 wave slots per block
  return (n_tiles + 15u) / 16u * 16u;
}

hipError_t launch_reset(const MarchParams& P, float* ph, hipStream_t s);
// What one march launch ran (vptmcm_debug_last_launch): the MODE
// specialisation, the layout template (kTpl*), the step loop (bit 0: 1
// speculative, 0 plain; bit 1: the macro-cell bound) and the number of fused passes.
struct MarchLaunchInfo {
  uint32_t mode, tpl, spec, passes;
};
// variant: tuning bits (bit 0 = plain step loop instead of the speculative one)
hipError_t launch_march(uint32_t layout, uint32_t variant, const MarchParams& P, const PassSeeds& PS,
                        const TileSched& T, float* ph,
                        const uint8_t* vol, const uint16_t* tf_rg, const uint32_t* tf_b4,
                        const uint8_t* tf_brow, const uint8_t* light, uint16_t* rgba, float* rgb32,
                        hipStream_t s, hipEvent_t ev_beg = nullptr, hipEvent_t ev_end = nullptr,
                        const uint32_t* tf_rows = nullptr, const uint8_t* tf_rowmap = nullptr,
                        const uint32_t* bin_lut = nullptr, MarchLaunchInfo* info = nullptr,
                        const uint8_t* maj = nullptr);
// Macro-cell alpha bound (MarchParams::maj_*): the density range of the macro
// cells of the box [m0, m0 + mn) from the linear staging volume, and the
// 4-bit alpha codes of all n cells from those ranges and the TF's per-row
// maximum alpha byte
hipError_t launch_macro_minmax(const uint8_t* lin, uint32_t W, uint32_t H, uint32_t D, uint32_t shift,
                               uint32_t nx, uint32_t ny, const uint32_t m0[3], const uint32_t mn[3],
                               uint16_t* mm, hipStream_t s);
hipError_t launch_macro_alpha(const uint16_t* mm, uint32_t n, const uint8_t* rowmax, uint8_t* q,
                              uint32_t bytes, hipStream_t s);
// Artistic tone mapper uniforms, derived on the host from (low, mid, high,
// saturation, gamma) (WebGPUArtisticToneMapper.js:81-88, ArtisticToneMapper.wgsl:40-46).
struct ToneParams {
  float low, inv_range, saturation, exponent;  // exponent = -log2((mid-low)/(high-low)) / gamma
};
hipError_t launch_tonemap_artistic(const uint16_t* rgba16, uint32_t n, const ToneParams& T,
                                   uint32_t* out, hipStream_t s);
// RGB sibling renderer (MCMComputeRenderer.wgsl): reset / march kernels.
hipError_t launch_reset_rgb(const MarchParams& P, float* ph, hipStream_t s);
hipError_t launch_march_rgb(uint32_t layout, const MarchParams& P, const PassSeeds& PS,
                            const TileSched& T, float* ph, const uint8_t* vol, const float4* tf,
                            uint16_t* rgba, float* rgb32, hipStream_t s,
                            hipEvent_t ev_beg = nullptr, hipEvent_t ev_end = nullptr,
                            MarchLaunchInfo* info = nullptr, const uint8_t* maj = nullptr);
// LINEAR -> CORNER8 / BRICK8 relayout of the cell box [c0, c0 + n) (default:
// every cell of the (W+1)(H+1)(D+1) grid)
hipError_t launch_corner8(const uint8_t* lin, uint32_t W, uint32_t H, uint32_t D, uint32_t BW,
                          uint32_t BH, void* out, hipStream_t s, const uint32_t c0[3] = nullptr,
                          const uint32_t n[3] = nullptr);
// LINEAR -> COLUMN4 quads of the box [c0, c0 + n) over (cx, cy, k) (default:
// every quad of the (W+1)(H+1)(D+2) grid)
hipError_t launch_column4(const uint8_t* lin, uint32_t W, uint32_t H, uint32_t D, void* out,
                          hipStream_t s, const uint32_t c0[3] = nullptr, const uint32_t n[3] = nullptr);
hipError_t launch_pack(const MarchParams& P, const float* ph, const float* rgb32, float4* out,
                       hipStream_t s);
// Multi-replica composite (k_composite): the n source buffers of npx (rgb*n, n)
// float4 summed in source order, / sum(n) -> fp32 rgb and rgba16float (either
// output and counts may be null). Sources and outputs may point into a shard
// of the frame; coherent: system-scope loads / stores, for sources and outputs
// in other devices' memory (the sharded device-list composite).
constexpr uint32_t kMaxReplicas = 8;
struct CompositeSrc {
  const float4* p[kMaxReplicas];
  uint32_t n;
};
hipError_t launch_composite(const CompositeSrc& S, uint32_t npx, float* rgb32, uint16_t* rgba,
                            float* counts, hipStream_t s, bool coherent = false);
// Guard build (VPT_GUARD): the layouts whose volume gathers left the volume
// allocation since the last call (bit = kTpl*), cleared by the call (0 in the product).
hipError_t guard_take_oob(uint32_t* out);
// fn 13 checks bin_of's arithmetic path against the count on the spectrum in P
hipError_t launch_verify(int fn, const MarchParams& P, uint32_t lo, uint32_t n,
                         unsigned long long* bad, uint32_t* first, uint32_t nfirst, hipStream_t s);
hipError_t launch_debug_eval(int fn, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s);

}  // namespace vpt
