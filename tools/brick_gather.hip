// brick_gather.hip — would an Infinity-Cache-resident u8 brick layout beat
// COLUMN4 in the volume-filling regime? (measurement aid, not product;
// VERDICT r05 next 2). Random trilinear samples, 8 in flight per lane:
//   mode 0  one 8-B load per sample (COLUMN4's gather) from a table of T bytes
//   mode 1  four 2-B loads per sample at o, o+9, o+81, o+90 of a random 9^3-B
//           brick (8^3 cells + a 1-voxel apron, u8: 729 B per 512 cells; a
//           512^3 volume is 262,144 bricks = 191 MB, Infinity-Cache sized)
//   hipcc -O3 --offload-arch=gfx950 tools/brick_gather.hip -o tools/brick_gather
//   tools/brick_gather <mode> <table MiB> [samples per lane] [blocks]
// One JSON line: samples/s for the table.
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

__device__ __forceinline__ uint32_t ld2(const uint8_t* p) {
  uint16_t v;
  __builtin_memcpy(&v, p, 2);  // one (possibly unaligned) 2-B load
  return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_sample(const uint8_t* __restrict__ tab, uint32_t units,
                                                uint32_t rounds, uint32_t* __restrict__ out) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  uint32_t h = pcg(gid * 2654435761u + 777u), acc = 0u;
  for (uint32_t r = 0; r < rounds; r++) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      h = pcg(h);
      const uint32_t u = __umulhi(h, units);  // uniform over [0, units)
      if constexpr (MODE == 0) {
        const uint2 q = reinterpret_cast<const uint2*>(tab)[u];
        v[k] = q.x ^ q.y;
      } else {
        const uint32_t c = pcg(h ^ 0x9e3779b9u);
        const uint8_t* b = tab + (size_t)u * 729u + (c & 7u) + ((c >> 3) & 7u) * 9u + ((c >> 6) & 7u) * 81u;
        v[k] = ld2(b) ^ (ld2(b + 9) << 3) ^ (ld2(b + 81) << 7) ^ (ld2(b + 90) << 11);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc += v[k];
  }
  out[gid] = acc;
}

__global__ void k_fill(uint8_t* tab, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    tab[i] = (uint8_t)(i * 131u >> 3);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const size_t mib = argc > 2 ? strtoull(argv[2], 0, 10) : 512;
  const uint32_t per_lane = argc > 3 ? (uint32_t)atoi(argv[3]) : 256;
  const uint32_t blocks = argc > 4 ? (uint32_t)atoi(argv[4]) : 4096;
  if (mode < 0 || mode > 1 || mib == 0 || mib > 4096) {
    fprintf(stderr, "usage: brick_gather <0|1> <MiB <= 4096> [samples per lane] [blocks]\n");
    return 2;
  }
  const size_t bytes = mib << 20;
  const uint32_t units = (uint32_t)(mode == 0 ? bytes / 8 : bytes / 729);
  uint8_t* tab;
  uint32_t* out;
  CK(hipMalloc(&tab, bytes + 64));
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  k_fill<<<4096, 256>>>(tab, bytes + 64);
  CK(hipDeviceSynchronize());
  const uint32_t rounds = per_lane / 8;
  auto launch = [&]() {
    if (mode == 0) k_sample<0><<<blocks, 256>>>(tab, units, rounds, out);
    else k_sample<1><<<blocks, 256>>>(tab, units, rounds, out);
  };
  launch();  // warm-up (and Infinity-Cache fill)
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double n = (double)blocks * 256 * rounds * 8, s = ms * 1e-3 / reps;
  printf("{\"mode\": %d, \"table_bytes\": %zu, \"samples_per_launch\": %.0f, \"launch_us\": %.2f, "
         "\"gsamples_per_s\": %.2f}\n", mode, bytes, n, s * 1e6, n / s * 1e-9);
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
