// kernels.h — launch interface of the gfx950 kernels (kernels.hip) used by
// the C-ABI implementation (vptmcm.cpp).
#pragma once

#include "march.h"

namespace vpt {

constexpr uint32_t kBlock = 256;  // 4 waves, each one 8x8 pixel tile

inline uint32_t march_blocks(const MarchParams& P) {
  return (P.n_tiles + (kBlock / 64) - 1) / (kBlock / 64);
}

hipError_t launch_reset(const MarchParams& P, float* ph, hipStream_t s);
hipError_t launch_march(uint32_t layout, const MarchParams& P, float* ph, const uint8_t* vol,
                        const uint32_t* tf, const uint8_t* light, uint16_t* rgba, hipStream_t s);
hipError_t launch_corner8(const uint8_t* lin, uint32_t W, uint32_t H, uint32_t D, void* out,
                          hipStream_t s);
hipError_t launch_pack(const MarchParams& P, const float* ph, const uint16_t* rgba, float4* out,
                       hipStream_t s);
hipError_t launch_debug_eval(int fn, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s);

}  // namespace vpt
