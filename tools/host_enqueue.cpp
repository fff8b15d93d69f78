// Host-side cost of a march launch through the C-ABI (tuning aid, not part of
// the product): per timed region of one F-pass launch, the time spent inside
// vptmcm_render_passes (make_params + the launch API), inside
// vptmcm_synchronize, and the wall time, with and without the region's HIP
// events; beside it the enqueue cost of an empty kernel launched with
// hipLaunchKernelGGL and with hipExtLaunchKernelGGL, for the HIP floor.
// Medians over N regions, after warm-up.
//   hipcc -O2 --offload-arch=gfx950 -Iinclude tools/host_enqueue.cpp \
//     -Lvpt-spectral-volume-rendering_amd/lib -lvptmcm \
//     -Wl,-rpath,$PWD/vpt-spectral-volume-rendering_amd/lib -o tools/host_enqueue
//   tools/host_enqueue [F=20] [N=200]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "vptmcm.h"

__global__ void k_empty(uint32_t* p) {
  if (p && threadIdx.x == 1023u && blockIdx.x == 100000u) p[0] = 1u;
}
struct Big {  // a kernarg block the size of the march's (PassSeeds + MarchParams + pointers)
  uint32_t w[240];
};
__global__ void k_empty_big(Big b, uint32_t* p) {
  if (p && threadIdx.x == 1023u && blockIdx.x == 100000u) p[0] = b.w[7];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? NAN : v[v.size() / 2];
}
#define CK(x)                                                              \
  do {                                                                     \
    int rc_ = (x);                                                         \
    if (rc_) {                                                             \
      fprintf(stderr, "%s failed: %d %s\n", #x, rc_, vptmcm_last_error(h)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 20u;
  const int N = argc > 2 ? atoi(argv[2]) : 200;
  const uint32_t R = 512, V = 128;
  vptmcm* h = nullptr;
  vptmcm_config cfg{R, VPTMCM_MAX_BINS, 0, VPTMCM_LAYOUT_CORNER8, 0};
  CK(vptmcm_create(&cfg, &h));
  std::vector<uint8_t> vol((size_t)V * V * V);
  for (uint32_t z = 0; z < V; z++)  // a soft sphere
    for (uint32_t y = 0; y < V; y++)
      for (uint32_t x = 0; x < V; x++) {
        const float dx = x - V / 2.0f, dy = y - V / 2.0f, dz = z - V / 2.0f;
        const float r = std::sqrt(dx * dx + dy * dy + dz * dz) / (V / 2.0f);
        vol[((size_t)z * V + y) * V + x] = (uint8_t)(r < 1.0f ? 255.0f * (1.0f - r) : 0.0f);
      }
  CK(vptmcm_set_volume(h, vol.data(), V, V, V));
  std::vector<uint8_t> tf(VPTMCM_TF_BYTES);
  for (size_t k = 0; k < tf.size(); k++) tf[k] = (uint8_t)((k * 37u) >> 3);
  CK(vptmcm_set_material_tf(h, tf.data()));
  std::vector<uint8_t> spd(256, 100);
  const float dir[3] = {1.0f, 0.0f, 0.0f};
  CK(vptmcm_set_light(h, spd.data(), dir));
  float spec[64] = {12.0f};
  for (int i = 0; i <= 12; i++) spec[1 + i] = 400.0f + 25.0f * i;
  CK(vptmcm_set_spectrum(h, spec));
  vptmcm_params P{32.0f, 0.0f, 8u, 8u, 0.0f};
  CK(vptmcm_set_params(h, &P));
  const float mvp[16] = {1.2f, 0, 0, 0, 0, 1.2f, 0, 0, 0, 0, 0, -4.5f, 0, 0, -1.0f, 5.0f};
  CK(vptmcm_reset(h, mvp, 1u));
  std::vector<uint32_t> seeds(F);
  for (uint32_t k = 0; k < F; k++) seeds[k] = 0x9e3779b9u * (k + 1u);
  for (int k = 0; k < 300; k++) CK(vptmcm_render_passes(h, mvp, seeds.data(), F));
  CK(vptmcm_synchronize(h));

  printf("{\"passes\": %u, \"regions\": %d", F, N);
  for (int timing = 0; timing < 2; timing++) {
    std::vector<double> enq, syn, wall, kern;
    for (int k = 0; k < N; k++) {
      CK(vptmcm_enable_kernel_timing(h, timing));
      const double t0 = now_us();
      CK(vptmcm_render_passes(h, mvp, seeds.data(), F));
      const double t1 = now_us();
      CK(vptmcm_synchronize(h));
      const double t2 = now_us();
      enq.push_back(t1 - t0);
      syn.push_back(t2 - t1);
      wall.push_back(t2 - t0);
      if (timing) {
        double ms = 0.0;
        uint64_t n = 0;
        CK(vptmcm_kernel_time(h, &ms, &n));
        kern.push_back(ms * 1e3);
        CK(vptmcm_enable_kernel_timing(h, 0));
      }
    }
    printf(", \"%s\": {\"enqueue_us\": %.2f, \"sync_us\": %.2f, \"wall_us\": %.2f, \"kernel_us\": %.2f}",
           timing ? "timed" : "untimed", med(enq), med(syn), med(wall), med(kern));
  }
  vptmcm_destroy(h);

  // the HIP floor: enqueue of an empty 256 x 1024 launch
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return 1;
  std::vector<double> plain, ext, ext_ev, ext_b, ext_e, big, marker_enq, marker_wall, stamp_wall;
  Big bg{};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int k = 0; k < N + 50; k++) {
    double t0 = now_us();
    hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, nullptr);
    double t1 = now_us();
    (void)hipStreamSynchronize(s);
    double t2 = now_us();
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, nullptr, nullptr, 0, nullptr);
    double t3 = now_us();
    (void)hipStreamSynchronize(s);
    double t4 = now_us();
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, e0, e1, 0, nullptr);
    double t5 = now_us();
    (void)hipStreamSynchronize(s);
    double t6 = now_us();
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, e0, nullptr, 0, nullptr);
    double t7 = now_us();
    (void)hipStreamSynchronize(s);
    double t8 = now_us();
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, nullptr, e1, 0, nullptr);
    double t9 = now_us();
    (void)hipStreamSynchronize(s);
    // an explicit begin marker + an end stamp from the dispatch, against the
    // begin stamp from the dispatch (t5 - t4 / t7 - t6): enqueue and wall
    const double m0 = now_us();
    (void)hipEventRecord(e0, s);
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, nullptr, e1, 0, nullptr);
    const double m1 = now_us();
    (void)hipStreamSynchronize(s);
    const double m2 = now_us();
    hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, e0, e1, 0, nullptr);
    const double m3 = now_us();
    (void)hipStreamSynchronize(s);
    const double m4 = now_us();
    if (k >= 50) {
      marker_enq.push_back(m1 - m0);
      marker_wall.push_back(m2 - m0);
      stamp_wall.push_back(m4 - m2);
    }
    bg.w[7] = (uint32_t)k;
    double t10 = now_us();
    hipLaunchKernelGGL(k_empty_big, dim3(256), dim3(1024), 0, s, bg, nullptr);
    double t11 = now_us();
    (void)hipStreamSynchronize(s);
    if (k >= 50) {
      plain.push_back(t1 - t0);
      ext.push_back(t3 - t2);
      ext_ev.push_back(t5 - t4);
      ext_b.push_back(t7 - t6);
      ext_e.push_back(t9 - t8);
      big.push_back(t11 - t10);
    }
  }
  printf(", \"region_begin\": {\"marker_then_launch_enqueue_us\": %.2f, \"marker_then_launch_wall_us\": %.2f, "
         "\"dispatch_stamped_wall_us\": %.2f}", med(marker_enq), med(marker_wall), med(stamp_wall));
  std::vector<double> setdev, lasterr, getdev;
  for (int k = 0; k < 2000; k++) {
    const double a = now_us();
    (void)hipSetDevice(0);
    const double b = now_us();
    (void)hipGetLastError();
    const double c = now_us();
    int d = -1;
    (void)hipGetDevice(&d);
    const double e = now_us();
    setdev.push_back(b - a);
    lasterr.push_back(c - b);
    getdev.push_back(e - c);
  }
  printf(", \"api_us\": {\"hipSetDevice\": %.3f, \"hipGetLastError\": %.3f, \"hipGetDevice\": %.3f}",
         med(setdev), med(lasterr), med(getdev));
  printf(", \"empty_kernel_enqueue_us\": {\"hipLaunchKernelGGL\": %.2f, \"hipExtLaunchKernelGGL\": %.2f, "
         "\"begin_and_end_events\": %.2f, \"begin_event\": %.2f, \"end_event\": %.2f, "
         "\"hipLaunchKernelGGL_960B_kernarg\": %.2f}}\n",
         med(plain), med(ext), med(ext_ev), med(ext_b), med(ext_e), med(big));
  return hipStreamDestroy(s) == hipSuccess ? 0 : 1;
}
