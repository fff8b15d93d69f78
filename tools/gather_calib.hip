// gather_calib.hip — known-bytes calibration of the memory-side counters for
// the march's access pattern (measurement aid, not product): scattered 8-B
// loads (one u64 per lane, the CORNER8 cell gather) from a table of T bytes.
//
// Every lane issues N independent gathers at PCG-hashed cell indices, so the
// gather count is known exactly (grid * N) and the bytes the program asks for
// are 8 per gather. Run once plainly (rate: gathers/s and the implied bytes per
// gather for 64-B and 128-B fills against the HBM peak) and under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE
// (FETCH_SIZE per gather = the counter's tally for one scattered 8-B load).
//   hipcc -O3 --offload-arch=gfx950 tools/gather_calib.hip -o tools/gather_calib
//   tools/gather_calib <table MiB> [gathers per lane] [blocks] [load flavour 0-4]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint32_t pcg(uint32_t v) {
  uint32_t s = v * 747796405u + 2891336453u;
  uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
  return (w >> 22u) ^ w;
}

// Eight 8-B gathers with the cache-policy bits of load flavour V: 0 plain, 1
// nontemporal (nt), 2 sc1, 3 sc0 sc1, 4 nt sc1. The asm flavours issue all
// eight loads and their vmcnt(0) in ONE asm statement with early-clobber
// outputs: the results exist only after the wait, and no output register may
// share a VGPR with an address still to be issued.
#define VPT_G8(POL)                                                                      \
  asm volatile("global_load_dwordx2 %0, %8, off " POL "\n"                              \
               "global_load_dwordx2 %1, %9, off " POL "\n"                              \
               "global_load_dwordx2 %2, %10, off " POL "\n"                             \
               "global_load_dwordx2 %3, %11, off " POL "\n"                             \
               "global_load_dwordx2 %4, %12, off " POL "\n"                             \
               "global_load_dwordx2 %5, %13, off " POL "\n"                             \
               "global_load_dwordx2 %6, %14, off " POL "\n"                             \
               "global_load_dwordx2 %7, %15, off " POL "\n"                             \
               "s_waitcnt vmcnt(0)"                                                      \
               : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]),       \
                 "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])                                  \
               : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]),      \
                 "v"(p[6]), "v"(p[7])                                                   \
               : "memory")

template <int V>
__device__ __forceinline__ void gload8(const uint2* const p[8], uint2 v[8]) {
  if constexpr (V == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = *p[k];
  } else if constexpr (V == 1) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint64_t u = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p[k]));
      v[k] = make_uint2((uint32_t)u, (uint32_t)(u >> 32));
    }
  } else if constexpr (V == 2) {
    VPT_G8("sc1");
  } else if constexpr (V == 3) {
    VPT_G8("sc0 sc1");
  } else {
    VPT_G8("nt sc1");
  }
}

// 8 gathers in flight per lane per round; `mask` = cells - 1 (power of two)
template <int V>
__global__ __launch_bounds__(256) void k_gather(const uint2* __restrict__ tab, uint32_t mask,
                                                uint32_t rounds, uint32_t* __restrict__ out) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint32_t h = pcg(gid * 2654435761u + 12345u), acc = 0u;
  for (uint32_t r = 0; r < rounds; r++) {
    const uint2* p[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      h = pcg(h);
      p[k] = tab + (h & mask);
    }
    uint2 v[8];
    gload8<V>(p, v);
#pragma unroll
    for (int k = 0; k < 8; k++) acc += v[k].x ^ v[k].y;
  }
  out[gid] = acc;
}

template <int V>
void launch(uint32_t blocks, const uint2* tab, uint32_t mask, uint32_t rounds, uint32_t* out) {
  k_gather<V><<<blocks, 256>>>(tab, mask, rounds, out);
}
using Launch = void (*)(uint32_t, const uint2*, uint32_t, uint32_t, uint32_t*);
static const Launch kLaunch[5] = {launch<0>, launch<1>, launch<2>, launch<3>, launch<4>};

__global__ void k_fill(uint2* tab, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) tab[i] = make_uint2((uint32_t)i, (uint32_t)(i >> 7));
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 1024;
  const uint32_t per_lane = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
  const uint32_t blocks = argc > 3 ? (uint32_t)atoi(argv[3]) : 4096;
  const int flavour = argc > 4 ? atoi(argv[4]) : 0;  // gload<V>
  if (flavour < 0 || flavour > 4) {
    fprintf(stderr, "load flavour must be 0-4\n");
    return 2;
  }
  size_t cells = mib * 1024 * 1024 / 8;
  if (cells & (cells - 1)) {
    fprintf(stderr, "table size must be a power of two MiB\n");
    return 2;
  }
  if (cells > (1ull << 32)) {
    fprintf(stderr, "table too large for 32-bit cell indices\n");
    return 2;
  }
  uint2* tab;
  uint32_t* out;
  CK(hipMalloc(&tab, cells * 8));
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  k_fill<<<4096, 256>>>(tab, cells);
  CK(hipDeviceSynchronize());
  const uint32_t rounds = per_lane / 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  kLaunch[flavour](blocks, tab, (uint32_t)(cells - 1), rounds, out);  // warm-up
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) kLaunch[flavour](blocks, tab, (uint32_t)(cells - 1), rounds, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double g = (double)blocks * 256 * rounds * 8;  // gathers per launch
  const double s = ms * 1e-3 / reps;
  printf("{\"flavour\": %d, \"table_bytes\": %zu, \"gathers_per_launch\": %.0f, \"launch_us\": %.2f, "
         "\"ggathers_per_s\": %.2f, \"tbps_if_64B\": %.2f, \"tbps_if_128B\": %.2f}\n",
         flavour, cells * 8, g, s * 1e6, g / s * 1e-9, g * 64 / s * 1e-12, g * 128 / s * 1e-12);
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
