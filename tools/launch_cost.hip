// Floor of a one-pass march launch on gfx950 (tuning aid, not part of the
// product): the march's grid (256 blocks x 1024 threads, R = 512) running
// only the pieces of its fixed per-launch work, to attribute the ~16 us that a
// one-pass launch costs beyond a fused pass:
//   empty    the dispatch and drain of the grid alone
//   state    + every lane loads and stores its 22 photon-state words (SoA planes)
//   lds      + the 128 KiB TF copied into LDS by every block
//   image    + the fp32 (12 B) and rgba16f (8 B) image stores of every pixel
// Each variant: 200 back-to-back launches between two events (average per
// launch) after 50 warm-up launches.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_cost.hip -o tools/launch_cost && tools/launch_cost
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kPlanes = 22;
constexpr uint32_t kPhotons = 512 * 512;
constexpr uint32_t kTfWords = 128 * 1024 / 4;

template <int V>
__global__ __launch_bounds__(1024) void k_cost(float* __restrict__ ph, const uint32_t* __restrict__ tf,
                                               float* __restrict__ rgb32, uint2* __restrict__ rgba,
                                               uint32_t salt) {
  __shared__ uint32_t s_tf[V >= 2 ? kTfWords : 1];
  const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
  float acc = 0.0f;
  if (V >= 2) {
    for (uint32_t k = threadIdx.x; k < kTfWords; k += 1024u) s_tf[k] = tf[k];
    __syncthreads();
    acc += __uint_as_float(s_tf[(i * 97u + salt) & (kTfWords - 1u)] & 0x3fffffffu);
  }
  if (V >= 1) {
    float w[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; p++) w[p] = ph[(size_t)p * kPhotons + i];
#pragma unroll
    for (int p = 0; p < kPlanes; p++) ph[(size_t)p * kPhotons + i] = w[p] + acc;
    acc += w[0];
  }
  if (V >= 3) {
    rgb32[i * 3u + 0u] = acc;
    rgb32[i * 3u + 1u] = acc + 1.0f;
    rgb32[i * 3u + 2u] = acc + 2.0f;
    rgba[i] = make_uint2(__float_as_uint(acc), salt);
  }
}

template <int V>
float time_variant(float* ph, const uint32_t* tf, float* rgb32, uint2* rgba) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int k = 0; k < 50; k++) hipLaunchKernelGGL(k_cost<V>, dim3(256), dim3(1024), 0, 0, ph, tf, rgb32, rgba, k);
  (void)hipEventRecord(a, 0);
  const int n = 200;
  for (int k = 0; k < n; k++) hipLaunchKernelGGL(k_cost<V>, dim3(256), dim3(1024), 0, 0, ph, tf, rgb32, rgba, k);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1e3f / n;
}

int main() {
  float *ph = nullptr, *rgb32 = nullptr;
  uint32_t* tf = nullptr;
  uint2* rgba = nullptr;
  if (hipMalloc(&ph, (size_t)kPlanes * kPhotons * 4) != hipSuccess ||
      hipMalloc(&tf, kTfWords * 4) != hipSuccess || hipMalloc(&rgb32, (size_t)kPhotons * 12) != hipSuccess ||
      hipMalloc(&rgba, (size_t)kPhotons * 8) != hipSuccess) {
    fprintf(stderr, "allocation failed\n");
    return 1;
  }
  (void)hipMemset(ph, 0, (size_t)kPlanes * kPhotons * 4);
  (void)hipMemset(tf, 0, kTfWords * 4);
  const float e = time_variant<0>(ph, tf, rgb32, rgba);
  const float s = time_variant<1>(ph, tf, rgb32, rgba);
  const float l = time_variant<2>(ph, tf, rgb32, rgba);
  const float m = time_variant<3>(ph, tf, rgb32, rgba);
  printf("{\"grid\": \"256 x 1024\", \"us_per_launch\": {\"empty\": %.2f, \"state\": %.2f, \"lds\": %.2f, "
         "\"image\": %.2f}}\n", e, s, l, m);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
