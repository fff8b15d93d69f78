// vptmcm.cpp — implementation of the C-ABI declared in include/vptmcm.h.
//
// Host-side orchestration of one renderer instance on one MI355X:
// resource ownership (photon planes, render target, volume, TF, light,
// spectrum), per-pass uniform preparation, kernel launches on an in-order
// HIP stream, HIP-event kernel timing, and the RCCL photon-parallel
// composite. Each entry point cites the reference code it replaces.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/vptmcm.h"
#include "kernels.h"

#ifndef VPT_STAMP
#define VPT_STAMP 0  // measurement builds (csrc/stamp.h) set it for both sources
#endif
// Guard build (-DVPT_GUARD=1 for both sources, kernels.hip): every device
// allocation is filled with the poison byte VPT_POISON (so a read of memory
// the library never wrote breaks bit-exactness) and bracketed by guard zones
// of poison that are checked, with the kernels' volume-gather bounds flags,
// after every launch; a hit fails the call with VPTMCM_EHIP naming it.
#ifndef VPT_GUARD
#define VPT_GUARD 0
#endif
#ifndef VPT_POISON
#define VPT_POISON 0xA5u
#endif

using namespace vpt;

namespace {

thread_local std::string g_create_error;

// ---- device allocations (guard zones in the guard build)
constexpr size_t kGuardBytes = VPT_GUARD ? 65536 : 0;
struct GuardAlloc {
  void* base;
  size_t bytes;
};
std::mutex g_guard_mu;
std::map<uintptr_t, GuardAlloc>& guard_live() {
  static std::map<uintptr_t, GuardAlloc> m;
  return m;
}

hipError_t dev_alloc_raw(void** p, size_t bytes) {
  if (!VPT_GUARD) return hipMalloc(p, bytes);
  void* base = nullptr;
  hipError_t e = hipMalloc(&base, bytes + 2 * kGuardBytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return e;
  }
  e = hipMemset(base, (int)VPT_POISON, bytes + 2 * kGuardBytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();  // before any stream of the library touches it
  if (e != hipSuccess) {
    (void)hipFree(base);
    *p = nullptr;
    return e;
  }
  *p = static_cast<char*>(base) + kGuardBytes;
  std::lock_guard<std::mutex> lk(g_guard_mu);
  guard_live()[(uintptr_t)*p] = GuardAlloc{base, bytes};
  return hipSuccess;
}

template <class T>
hipError_t dev_alloc(T** p, size_t bytes) {
  void* v = nullptr;
  const hipError_t e = dev_alloc_raw(&v, bytes);
  *p = static_cast<T*>(v);
  return e;
}

// The guard zones of one allocation hold nothing but poison (guard build).
bool guard_intact(uintptr_t user, const GuardAlloc& a) {
  std::vector<uint8_t> g(kGuardBytes);
  for (int side = 0; side < 2; side++) {
    const char* z = side ? reinterpret_cast<const char*>(user) + a.bytes : static_cast<const char*>(a.base);
    if (hipMemcpy(g.data(), z, kGuardBytes, hipMemcpyDeviceToHost) != hipSuccess) return false;
    for (uint8_t b : g)
      if (b != (uint8_t)VPT_POISON) return false;
  }
  return true;
}

// Every live allocation's guard zones: "" when intact, else which one broke.
std::string guard_scan() {
  if (!VPT_GUARD) return std::string();
  std::lock_guard<std::mutex> lk(g_guard_mu);
  for (const auto& kv : guard_live())
    if (!guard_intact(kv.first, kv.second)) {
      char b[128];
      snprintf(b, sizeof b, "guard zone of the %zu-byte allocation at %p overwritten", kv.second.bytes,
               (void*)kv.first);
      return b;
    }
  return std::string();
}

hipError_t dev_free(void* p) {
  if (!VPT_GUARD || !p) return hipFree(p);
  GuardAlloc a{nullptr, 0};
  {
    std::lock_guard<std::mutex> lk(g_guard_mu);
    auto it = guard_live().find((uintptr_t)p);
    if (it == guard_live().end()) return hipFree(p);  // not ours
    a = it->second;
    if (!guard_intact(it->first, a))
      fprintf(stderr, "vptmcm guard: guard zone of the %zu-byte allocation at %p overwritten (at free)\n",
              a.bytes, p);
    guard_live().erase(it);
  }
  return hipFree(a.base);
}

struct EventPair {
  hipEvent_t beg = nullptr, end = nullptr;
};

// One forwarded operation of a device-list handle, type-erased for a worker.
struct ReplicaJob {
  int (*call)(const void*, vptmcm*) = nullptr;
  const void* f = nullptr;
};

// The worker thread of one peer replica of a device-list handle: every
// forwarded operation (ingest, render_passes, reset, the composite's pack and
// push, synchronize) runs on all replicas at once, each replica's host work
// and enqueue on its own thread, instead of one replica after another from the
// caller's thread. Posting is a counter bump; an idle worker spins for up to
// 200 us (the handle's sync_spin_us if shorter) and then sleeps on the
// condition variable.
struct ReplicaWorker {
  vptmcm* c = nullptr;
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  std::atomic<uint64_t> posted{0}, finished{0};
  std::atomic<bool> quit{false};
  ReplicaJob job;
  int rc = 0;
  int64_t spin_us = 0;
};

}  // namespace

struct vptmcm {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t R = 0, tiles_x = 0, n_tiles = 0, npad = 0;
  uint32_t layout = kLayoutLinear;
  uint32_t kind = VPTMCM_RENDERER_SPECTRAL;
  uint32_t variant = 0;  // tuning knob (VPTMCM_MARCH_VARIANT), results identical
  uint32_t band_y0 = 0, band_y1 = 0;  // vptmcm_set_band (band_y1 = R after create)

  float* photons = nullptr;    // kNumPlanes * npad words
  uint16_t* rgba = nullptr;    // R*R*4 halfs
  float* rgb32 = nullptr;      // R*R*3 floats: the last launch's image before the f16 store
  uint32_t* ldr = nullptr;     // R*R rgba8 of the tone mapper (lazily allocated)
  uint8_t* vol_lin = nullptr;  // W*H*D (staging for CORNER8; the volume for LINEAR)
  void* vol_c8 = nullptr;      // (W+1)(H+1)(D+1) u64
  uint32_t W = 0, H = 0, D = 0;
  bool volume_ready = false;   // renderable: from volume_begin on (unwritten blocks read zero)
  bool vol_done = false;       // LINEAR after volume_end (its staging copy is the volume)
  // CORNER8 / BRICK8 cells [vol_c0, vol_c1) whose blocks arrived since the last
  // relayout: re-laid out in one launch before the next march reads the cells
  // (or at volume_end), so a slice-by-slice ingest relays each cell once
  bool vol_dirty = false;
  uint32_t vol_c0[3] = {0, 0, 0}, vol_c1[3] = {0, 0, 0};
  uint16_t* tf_rg = nullptr;   // 65536 (albedo | alpha << 8) texels
  uint32_t* tf_b4 = nullptr;   // 257*257 anisotropy corner cells
  uint8_t* tf_brow = nullptr;  // 256 anisotropy rows (valid when b_rows)
  uint32_t* tf_rows = nullptr;   // kTfRowsMax distinct TF rows, u32 texels (valid when tf_dedup)
  uint8_t* tf_rowmap = nullptr;  // density row -> distinct row
  uint32_t* bin_lut = nullptr;   // MarchParams::bins_lut table (device)
  // Macro-cell alpha bound (MarchParams::maj_*): per macro cell the volume's
  // byte range (maj_mm, kept current by every relayout) and the 4-bit alpha
  // codes the march stages in LDS (maj_q, rebuilt before a march whenever the
  // volume or the TF changed: maj_valid); tf_rowmax = max alpha byte per TF row
  uint16_t* maj_mm = nullptr;
  uint8_t* maj_q = nullptr;
  uint8_t* tf_rowmax = nullptr;
  uint32_t maj_shift = 0, maj_nx = 0, maj_ny = 0, maj_nz = 0, maj_n = 0, maj_bytes = 0;
  bool maj_ok = false, maj_valid = false;
  bool bin_lut_ok = false;
  uint32_t bin_lut_host[kBinLutCells + kBinLutCells / 4] = {};
  uint32_t tf_dedup = 0;
  uint32_t b_rows = 1;         // zero TF: column-invariant
  uint8_t* light = nullptr;    // 256 bytes
  float4* tf_rgb = nullptr;    // RGB sibling: decoded TF row 0 (kRgbTfMax texels)
  uint32_t tf_rgb_w = 0;
  float env[4] = {1.0f, 1.0f, 1.0f, 1.0f};  // RGB sibling: 1x1 white (WebGPURenderingContext.js:97-108)
  uint8_t* sched = nullptr;    // tile schedule flags: [2][sched_flag_bytes(n_tiles)]
  uint32_t* sched_prev = nullptr;  // each wave slot's last scheduled tile (TileSched::prev)
  uint32_t sched_cur = 0;      // which flag row the next march reads
  uint32_t* sched_changed = nullptr;  // [2] TileSched::changed_in / changed_out, alternating
  bool sched_cache = true;     // VPTMCM_SCHED_CACHE=0: every launch runs the schedule
  uint32_t dark = 1;           // MarchParams::dark: 1 the dark-background chain, 0 off (VPTMCM_DARK)

  float spectrum[VPTMCM_SPECTRUM_FLOATS] = {};
  uint8_t light_host[256];
  float light_dir[3] = {1.0f, 0.0f, 0.0f};
  vptmcm_params params{1.0f, 0.0f, 8u, 8u, 0.0f};  // property defaults, js:19-48

  // timing
  // Region timing: the first march launch after enable stamps `region.beg`
  // from its own dispatch packet and every timed launch stamps `region.end`
  // at its completion, so the last one closes the region (an end marker
  // enqueued behind it cost 9-11 us of wall time per region). Per-launch
  // event pairs were measured to cost 1.6 us per fused pass (the markers'
  // cache maintenance between back-to-back launches), so only the region is
  // bracketed.
  bool timing = false;
  bool time_stop = true;  // the last launch stamps region.end itself (VPTMCM_TIME_STOP=0: a marker)
  // VPTMCM_TIME_BEGIN=marker: region.beg is a marker recorded just before the
  // region's first launch instead of a stamp from that launch's dispatch packet
  bool time_begin_marker = false;
  bool region_closed = false;
  EventPair region;
  uint64_t launches = 0;
  uint64_t march_launches = 0;  // every march launch since create (vptmcm_debug_last_launch)
  // vptmcm_synchronize / kernel_time poll the stream for up to this long before
  // blocking (VPTMCM_SYNC_SPIN_US, 0 = block at once): a blocking wait wakes
  // through an interrupt, whose latency on a busy host adds tens of
  // microseconds to every short region
  int64_t sync_spin_us = 2000;
  // Completion signal of the spectral march (TileSched::done_ctr/done_flag):
  // the last wave of a launch writes its sequence number to a word of
  // fine-grained host memory once every wave's stores have landed, so
  // vptmcm_synchronize sees a march-terminated stream finish without the
  // end-of-kernel packet's cache write-back and completion signal (~9 us on
  // the driver's one-launch region). VPTMCM_DONE_FLAG=0 turns it off.
  bool done_on = true;
  uint32_t* done_ctr = nullptr;        // device: cumulative wave count
  uint32_t* done_host = nullptr;       // host (fine-grained): the last signalled sequence number
  uint32_t* done_dev = nullptr;        // its device address
  uint32_t done_total = 0, done_seq = 0;
  bool done_pending = false;           // the stream's last enqueued work is march done_seq
  // With a communicator, every spectral march over the whole frame also writes
  // (rgb * n, n) into comp[comp_next] (TileSched::pack, k_pack's values): when
  // it is the stream's last work, vptmcm_comm_allreduce_radiance reduces that
  // buffer without a k_pack launch.
  bool pack_fresh = false;
  // Device-list (PEER) replicas: the march packs (rgb * n, n) into grp_pack[b]
  // for the next composite (b = that composite's buffer), so a composite that
  // follows a march launches no k_pack: pack_buf is the buffer the stream's
  // last march packed (valid with pack_fresh), grp_owner the handle holding
  // the composite's bookkeeping (replica 0; itself for replica 0).
  int pack_buf = -1;
  struct vptmcm* grp_owner = nullptr;
  MarchLaunchInfo last_launch{};
  // Whether the march skips certain null collisions' gathers (MarchParams::
  // maj_on; same results either way) is measured, not guessed: it pays where
  // the march waits on volume line fills (a volume filling the frame, +35 %
  // per pass at 512^3; 1024^3, +5 %) and costs where it does not (the
  // default camera, -6 %; a cache-resident 256^3 volume). VPTMCM_MAJ=auto
  // (default): launches outside timed regions are timed now and then with
  // their own events, in pairs of adjacent launches (one with the skip, one
  // without), and the averaged ratio picks the faster; on / off pin it. Off
  // runs k_march<..., MAJ = false>, the step loop without the test. Pairs
  // are read back without blocking, up to kPairs of them in flight, so a
  // caller that enqueues many launches ahead of the GPU still gets its
  // measurements.
  static constexpr int kPairs = 8;
  static constexpr int kQuads = 2;
  struct MajTuner {
    int mode = 2;                 // 0 off, 1 on, 2 auto
    int choice = 0;               // the last pick measured, for sizes with none yet
    // per launch size n (passes): the time with the skip over without it,
    // from pairs of adjacent launches of that size, one each way. A pair's
    // two launches do not run alike (one-pass launches: the first of a pair
    // runs ~7 % slower whichever it is), so a pair counts only with the next
    // pair of the other order: the geometric mean of their ratios, averaged
    // over such pairs of pairs (-1: none measured yet). Sizes differ: at the
    // default camera a 32-pass launch is issue-bound (the skip costs 6 %)
    // while a one-pass launch ends with its slowest in-volume waves (the skip
    // saves 1.6 %).
    float ratio[kMaxFusedPasses + 1];
    float half[kMaxFusedPasses + 1];         // a pair's ratio awaiting the other order (-1: none)
    // pairs of pairs folded into ratio[n] since the last reset or camera
    // change: it decides from kQuads on (until then every launch of size n
    // outside a timed region is a probe, and a ratio from the previous camera,
    // if any, still picks)
    uint8_t quads[kMaxFusedPasses + 1];
    uint32_t cam_launches = 0;    // launches since the camera last changed (pairs start only from 1 on)
    uint32_t launches[kMaxFusedPasses + 1];  // launches of size n since its last pair
    uint8_t first[kMaxFusedPasses + 1];      // the first choice of size n's next pair
    uint8_t half_first[kMaxFusedPasses + 1]; // the first choice of the pair held in half
    float mvp[16] = {};           // the camera of the launches measured (another one: measure again)
    uint32_t epoch = 0;           // bumped by a reset or a new camera: pairs of an older epoch are dropped
    struct Pair {
      hipEvent_t b[2] = {nullptr, nullptr}, e[2] = {nullptr, nullptr};
      int first = 0;              // the choice of the pair's first launch (the second: the other)
      uint32_t n = 0, epoch = 0;
      int stage = 0;              // launches enqueued (2: complete, waiting to be read)
    } pairs[kPairs];              // a ring: head the oldest, count in flight
    int head = 0, count = 0;
  } maj_tune;
  // The camera's robust-miss region (robust_region: a double-precision matrix
  // inverse and the projected hull) for the last matrix seen: a progressive
  // renderer re-sends one camera every pass, so launches reuse it instead of
  // recomputing it (keyed on the matrix bits and 1/R, the only inputs).
  struct RobustCache {
    bool valid = false, ok = false;
    float m[16];
    float ir = 0.0f;
    float rb[4];
    float edge[kRbEdges][3];
  } robust_cache;

  // multi-GPU
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // Bound on any wait for the communicator (init, an enqueue still in progress,
  // a stream holding RCCL work): VPTMCM_COMM_TIMEOUT_MS, default 120 s. On
  // expiry or an asynchronous RCCL error the communicator is aborted and the
  // call returns VPTMCM_ECOMM, so a dead or hung peer ends the job instead of
  // hanging every rank.
  int64_t comm_timeout_ms = 120000;
  bool comm_failed = false;  // the communicator was aborted (comm_fail): waits stay bounded
  uint32_t* band_cover = nullptr;  // Mode B: one counter per 8-row tile, all-reduced
  hipStream_t comm_stream = nullptr;
  float4* comp[2] = {nullptr, nullptr};
  hipEvent_t comp_ready[2] = {nullptr, nullptr};
  hipEvent_t comp_done[2] = {nullptr, nullptr};
  int comp_next = 0, comp_last = -1;
  bool comp_sharded[2] = {false, false};  // comp[k] holds only this rank's reduce-scattered shard
  // Lazily fused render() calls: consecutive passes with one matrix are queued
  // and launched as one multi-pass march when anything observes or changes
  // the renderer (every other entry point flushes first), or at 32 passes.
  uint32_t pend_n = 0;
  uint32_t pend_seeds[kMaxFusedPasses];
  float pend_mvp[16];
  double* host_scratch = nullptr;
  // Mode A composite target: k_composite over comp[comp_last] (vptmcm_read_composite)
  float* comp_rgb32 = nullptr;
  uint16_t* comp_rgba = nullptr;
  float* comp_counts = nullptr;

  // Multi-device handle (vptmcm_config::n_devices): replica 0 is this handle,
  // replicas 1..N-1 are full single-device handles of their own; every input
  // and every pass is forwarded to them (their seed stream: replica_seed), and
  // the render target is the composite of all replicas, made on this device.
  std::vector<vptmcm*> peers;
  uint32_t replica = 0;            // the replica index (seed stream) of this handle
  bool grouped = false;            // created from a device list (even of one device)
  uint32_t group_transport = VPTMCM_GROUP_PEER;
  bool grp_dirty = true;           // a march / reset since the last composite
  // this replica's (rgb*n, n) on its device; PEER double-buffers it (composite
  // j packs into [j & 1]), so a pack never waits for the composite before it
  float4* grp_pack[2] = {nullptr, nullptr};
  float4* grp_gather = nullptr;    // replica 0, RCCL: the reduced sum
  // The composite image: PEER, this replica's pixel shard [grp_p0, grp_p1) of
  // it, on its own device (the composite is never gathered on one device: the
  // readers copy every shard to the host at once); RCCL, replica 0: all of it
  float* grp_rgb32 = nullptr;      // fp32
  uint16_t* grp_rgba = nullptr;    // rgba16float
  float* grp_counts = nullptr;     // PEER: sum(n)
  uint32_t* grp_ldr = nullptr;     // PEER: the tone mapper's rgba8 of the shard (lazily)
  size_t grp_p0 = 0, grp_p1 = 0;
  hipEvent_t grp_packed = nullptr; // this replica's pack of the current composite is complete
  // PEER (sharded): replica k composites pixel shard k of every replica's pack
  // on its own device, on a stream of its own (its next march does not wait
  // for the other replicas), writing that slice of the image into devices[0]
  hipStream_t grp_stream = nullptr;
  // this replica's shard of composite j is written (and, so, its reads of
  // every replica's buffer j & 1 are done): [j & 1]
  hipEvent_t grp_shard[2] = {nullptr, nullptr};
  // replica 0, RCCL: the composite (reduce + k_composite) is complete; the
  // readers and the next pack wait for it ([0]; PEER uses grp_shard instead)
  hipEvent_t grp_done[2] = {nullptr, nullptr};
  uint32_t grp_seq = 0;            // replica 0: composites issued
  // replica 0, PEER: the composite (1-based seq) that last used buffer b, and
  // the highest composite known complete on the host (synchronize / reads):
  // a buffer whose last composite is known complete needs no fence wait
  uint32_t grp_use_seq[2] = {0u, 0u};
  uint32_t grp_synced_seq = 0;
  int grp_last = -1;               // replica 0: the buffer of the last composite
  std::vector<ncclComm_t> grp_comms;  // RCCL transport: one communicator per replica (InitAll)
  // replica 0: one worker thread per peer (VPTMCM_GROUP_THREADS=0: none, the
  // operations run serially on the caller's thread)
  std::vector<std::unique_ptr<ReplicaWorker>> workers;

  std::string err;
};

#define FAIL(h, code, ...)                                              \
  do {                                                                  \
    char _b[512];                                                       \
    snprintf(_b, sizeof _b, __VA_ARGS__);                               \
    (h)->err = _b;                                                      \
    return (code);                                                      \
  } while (0)

#define HIPCHK(h, expr)                                                        \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess)                                                      \
      FAIL(h, VPTMCM_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
           __FILE__, __LINE__);                                                \
  } while (0)

namespace {

const float kNoMatrix[16] = {};  // for launches that only read the non-camera fields

// rgba8unorm-srgb decode (the sampler converts before filtering), in double,
// rounded to f32; identical to the oracle's orc_srgb_to_linear
float srgb_to_linear(uint8_t b) {
  double v = b / 255.0;
  return (float)(v <= 0.04045 ? v / 12.92 : std::pow((v + 0.055) / 1.055, 2.4));
}

// Robust-miss region of the march (MarchParams::robust, k_march's robust
// path). In exact arithmetic a camera ray of pixel (sx, sy) runs from the
// near point NDC (sx, sy, -1) to the far point (sx', sy', 1) with
// |sx' - sx|, |sy' - sy| <= invRes, and every point of it beyond the far
// point has NDC z > 1. So if (a) the projective map is regular on the NDC
// box (world w > 0 at its 8 corners), (b) the unit cube, expanded by a
// world-space margin delta that dominates the f32 rounding of the ray, lies
// in front of the camera with NDC z in (-1, 1), and (c) the pixel's jitter
// footprint misses the NDC bounding box of that expanded cube, then every
// computed photon position on the ray is outside [0,1]^3: each step is an
// exit. Computed in double from the f32 matrix; returns the screen bounds
// outside of which pixel centres qualify, or false (no robust pixels).
// edge[kRbEdges][3] receives the hull lines of the same expanded corners'
// projections (counter-clockwise, outward normal (a, b) with |a| + |b| = 1):
// a * sx + b * sy > c qualifies a pixel centre too, c padded like the box.
bool robust_region(const float* m32, float ir, float rb[4], float (*edge)[3]) {
  double M[16], F[16];
  for (int i = 0; i < 16; i++) M[i] = m32[i];  // column-major: M[col * 4 + row]
  auto mul = [](const double* A, double x, double y, double z, double o[4]) {
    for (int r = 0; r < 4; r++) o[r] = A[r] * x + A[4 + r] * y + A[8 + r] * z + A[12 + r];
  };
  double maxnear = 0.0, maxfar = 0.0, o[4];
  for (int c = 0; c < 8; c++) {
    mul(M, (c & 1) ? 1.0 : -1.0, (c & 2) ? 1.0 : -1.0, (c & 4) ? 1.0 : -1.0, o);
    if (!(o[3] > 0.0)) return false;
    for (int k = 0; k < 3; k++) {
      double v = std::fabs(o[k] / o[3]);
      if (!std::isfinite(v)) return false;
      double& mx = (c & 4) ? maxfar : maxnear;
      mx = v > mx ? v : mx;
    }
  }
  // F = M^-1 by Gauss-Jordan with partial pivoting (row-major work copy)
  double A[4][8];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      A[r][c] = M[c * 4 + r];
      A[r][4 + c] = (r == c) ? 1.0 : 0.0;
    }
  for (int c = 0; c < 4; c++) {
    int piv = c;
    for (int r = c + 1; r < 4; r++)
      if (std::fabs(A[r][c]) > std::fabs(A[piv][c])) piv = r;
    if (!(std::fabs(A[piv][c]) > 1e-300)) return false;
    for (int k = 0; k < 8; k++) std::swap(A[c][k], A[piv][k]);
    double d = A[c][c];
    for (int k = 0; k < 8; k++) A[c][k] /= d;
    for (int r = 0; r < 4; r++) {
      if (r == c) continue;
      double f = A[r][c];
      for (int k = 0; k < 8; k++) A[r][k] -= f * A[c][k];
    }
  }
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) F[c * 4 + r] = A[r][4 + c];
  const double delta = 1e-3 * (1.0 + maxnear) + 1e-6 * maxfar;
  double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300, px[8], py[8];
  for (int c = 0; c < 8; c++) {
    mul(F, (c & 1) ? 1.0 + delta : -delta, (c & 2) ? 1.0 + delta : -delta,
        (c & 4) ? 1.0 + delta : -delta, o);
    if (!(o[3] > 0.0)) return false;
    double nx = o[0] / o[3], ny = o[1] / o[3], nz = o[2] / o[3];
    if (!(nz > -1.0 + 1e-6 && nz < 1.0 - 1e-6) || !std::isfinite(nx) || !std::isfinite(ny)) return false;
    x0 = nx < x0 ? nx : x0;
    x1 = nx > x1 ? nx : x1;
    y0 = ny < y0 ? ny : y0;
    y1 = ny > y1 ? ny : y1;
    px[c] = nx;
    py[c] = ny;
  }
  const double pad = (double)ir + 1e-4;
  rb[0] = std::nextafter((float)(x0 - pad), -INFINITY);
  rb[1] = std::nextafter((float)(x1 + pad), INFINITY);
  rb[2] = std::nextafter((float)(y0 - pad), -INFINITY);
  rb[3] = std::nextafter((float)(y1 + pad), INFINITY);
  for (int e = 0; e < kRbEdges; e++) edge[e][0] = edge[e][1] = 0.0f, edge[e][2] = FLT_MAX;
  // convex hull of the eight projections (monotone chain, counter-clockwise)
  int idx[8], hull[16], nh = 0;
  for (int k = 0; k < 8; k++) idx[k] = k;
  std::sort(idx, idx + 8, [&](int a, int b) { return px[a] < px[b] || (px[a] == px[b] && py[a] < py[b]); });
  auto cross = [&](int o_, int a, int b) {
    return (px[a] - px[o_]) * (py[b] - py[o_]) - (py[a] - py[o_]) * (px[b] - px[o_]);
  };
  for (int k = 0; k < 8; k++) {  // lower chain
    while (nh >= 2 && cross(hull[nh - 2], hull[nh - 1], idx[k]) <= 0.0) nh--;
    hull[nh++] = idx[k];
  }
  for (int k = 6, lo = nh + 1; k >= 0; k--) {  // upper chain
    while (nh >= lo && cross(hull[nh - 2], hull[nh - 1], idx[k]) <= 0.0) nh--;
    hull[nh++] = idx[k];
  }
  nh--;  // the last point repeats the first
  if (nh < 3 || nh > kRbEdges) return true;  // degenerate: the box alone
  for (int e = 0; e < nh; e++) {
    const int a = hull[e], b = hull[(e + 1) % nh];
    double nx = py[b] - py[a], ny = px[a] - px[b];  // outward for a counter-clockwise hull
    const double l1 = std::fabs(nx) + std::fabs(ny);
    if (!(l1 > 0.0)) return true;
    nx /= l1;
    ny /= l1;
    double cmax = -1e300;  // the support of every corner (rounding of the hull)
    for (int k = 0; k < 8; k++) cmax = std::max(cmax, nx * px[k] + ny * py[k]);
    // the kernel's f32 evaluation of a * sx + b * sy (|sx|, |sy| <= 1, a and b
    // rounded to f32) errs by < 1e-6: far inside the 1e-4 of the pad
    edge[e][0] = (float)nx;
    edge[e][1] = (float)ny;
    edge[e][2] = std::nextafter((float)(cmax + pad), INFINITY);
  }
  return true;
}

// Uniform preparation shared by render and reset (wgsl:8-18, js:295-312).
// Everything derived here is computed in IEEE f32 exactly as the kernel
// would compute it per lane (host SSE arithmetic, no contraction).
// robust_region of (mvp, ir) through the handle's one-entry cache.
bool robust_cached(vptmcm* h, const float* mvp, float ir, float rb[4], float (*edge)[3]) {
  if (mvp == kNoMatrix) return robust_region(mvp, ir, rb, edge);  // the packs' launches: keep the camera's entry
  auto& c = h->robust_cache;
  if (!c.valid || memcmp(c.m, mvp, sizeof c.m) != 0 || memcmp(&c.ir, &ir, sizeof ir) != 0) {
    c.valid = false;
    c.ok = robust_region(mvp, ir, c.rb, c.edge);
    memcpy(c.m, mvp, sizeof c.m);
    c.ir = ir;
    c.valid = true;
  }
  memcpy(rb, c.rb, sizeof c.rb);
  memcpy(edge, c.edge, sizeof c.edge);
  return c.ok;
}

MarchParams make_params(vptmcm* h, const float* mvp, uint32_t seed) {
  MarchParams P;
  memset(&P, 0, sizeof P);
  memcpy(P.m, mvp, sizeof P.m);
  P.inv_res[0] = (float)(1.0 / (double)h->R);  // Float32Array([1 / R]), js:297
  P.inv_res[1] = P.inv_res[0];
  P.seed = seed;
  P.blur = h->params.blur;
  P.extinction = h->params.extinction;
  P.rcp_extinction = 1.0f / h->params.extinction;  // RN(1/x), the spec's division
  P.max_bounces = h->params.max_bounces;
  P.steps = h->params.steps;
  const float* s = h->spectrum;
  float nbf = s[0] + 0.5f;  // u32(spectrum[0] + 0.5)
  uint32_t nb = (nbf > 0.0f) ? (uint32_t)nbf : 0u;
  P.nb = nb;
  for (int i = 0; i < 13; i++) P.lam[i] = s[1 + i];
  P.bins_sorted = 1u;
  for (uint32_t i = 1; i + 1 < nb; i++)
    if (!(s[1 + i] <= s[2 + i])) P.bins_sorted = 0u;  // lam[i] <= lam[i+1], NaN-safe
  P.min_lam = s[1];
  P.max_lam = s[nb + 1];
  P.bins_padded = 0u;
  if (P.bins_sorted && nb >= 1u && nb <= (uint32_t)kMaxBins) {
    bool fin = std::isfinite(P.max_lam - P.min_lam);
    for (uint32_t i = 0; i <= nb; i++) fin = fin && std::isfinite(s[1 + i]);
    if (fin) {
      P.bins_padded = 1u;
      for (uint32_t i = 0; i < (uint32_t)kMaxBins; i++)
        P.lam_pad[i] = (i >= 1u && i < nb) ? s[1 + i] : INFINITY;
    }
  }
  // Equal-width bins (the reference default, 12 x 25 nm from 400 nm) take the
  // arithmetic bin search of bin_of(); see its comment for the conditions.
  P.bins_uniform = 0u;
  if (nb >= 1u && nb <= (uint32_t)kMaxBins && P.bins_sorted) {
    const float l0 = s[1], w = s[2] - s[1];
    bool ok = std::isfinite(l0) && std::isfinite(w) && l0 > 0.0f && w > 0.0f &&
              std::isfinite(s[nb + 1]) && s[nb + 1] <= 2.0f * l0;
    for (uint32_t i = 0; ok && i <= nb; i++) {
      if (!(s[1 + i] == std::fmaf((float)i, w, l0))) ok = false;  // bin_of's boundary formula
    }
    if (ok) {
      P.bins_uniform = 1u;
      P.bin_w = w;
      P.rcp_bin_w = 1.0f / w;
    }
  }
  for (uint32_t i = 0; i < nb && i < (uint32_t)kMaxBins; i++) {
    P.xb[i] = s[2 + nb + i];
    P.yb[i] = s[2 + 2 * nb + i];
    P.zb[i] = s[2 + 3 * nb + i];
  }
  const float* ld = h->light_dir;
  float dd = std::fmaf(ld[2], ld[2], std::fmaf(ld[1], ld[1], ld[0] * ld[0]));
  float len = sqrtf(dd);
  P.light_iso = len < kEps ? 1u : 0u;
  if (!P.light_iso) {  // normalize = v * RN(1/length)
    float il = 1.0f / len;
    P.light_dir[0] = ld[0] * il;
    P.light_dir[1] = ld[1] * il;
    P.light_dir[2] = ld[2] * il;
  }
  P.b_rows = h->b_rows;
  P.tf_dedup = h->tf_dedup;
  P.bins_lut = h->bin_lut_ok ? 1u : 0u;
  {  // |w| bound for unproject<true>: |a|, |b| <= 1 + max(2/R, |blur|) + 1 (slop)
    const double A = 2.0 + std::max(2.0 / h->R, std::fabs((double)P.blur));
    bool fin = true;
    for (int k = 0; k < 16; k++) fin = fin && std::isfinite(mvp[k]);
    const double wb = (std::fabs((double)mvp[3]) + std::fabs((double)mvp[7])) * A +
                      std::fabs((double)mvp[11]) + std::fabs((double)mvp[15]);
    P.w_bounded = (fin && wb < std::ldexp(1.0, 120)) ? 1u : 0u;
  }
  P.anisotropy = h->params.anisotropy;
  P.tf_w = h->tf_rgb_w;
  for (int k = 0; k < 4; k++) P.env[k] = h->env[k];
  float rb[4];
  P.robust = (P.blur == 0.0f && P.rcp_extinction > 0.0f && std::isfinite(P.rcp_extinction) &&
              robust_cached(h, mvp, P.inv_res[0], rb, P.rb_edge)) ? 1u : 0u;
  if (!P.robust)
    for (int e = 0; e < kRbEdges; e++) P.rb_edge[e][0] = P.rb_edge[e][1] = 0.0f, P.rb_edge[e][2] = FLT_MAX;
  if (P.robust) {
    P.rb_x0 = rb[0];
    P.rb_x1 = rb[1];
    P.rb_y0 = rb[2];
    P.rb_y1 = rb[3];
  }
  P.R = h->R;
  P.band_y0 = h->band_y0;
  P.band_y1 = h->band_y1;
  P.tiles_x = h->tiles_x;
  P.n_tiles = h->n_tiles;
  P.npad = h->npad;
  P.W = h->W;
  P.H = h->H;
  P.D = h->D;
  {
    const uint64_t w1 = h->W + 1ull, h1 = h->H + 1ull, d1 = h->D + 1ull;
    const uint64_t bw = (w1 + kBrickCells - 1) / kBrickCells, bh = (h1 + kBrickCells - 1) / kBrickCells,
                   bd = (d1 + kBrickCells - 1) / kBrickCells;
    P.BW = (uint32_t)bw;
    P.BH = (uint32_t)bh;
    if (h->layout == kLayoutBrick8)
      P.vol32 = (bw * bh * bd * 512ull < (1ull << 32) && bd * bh < (1ull << 24)) ? 1u : 0u;
    else if (h->layout == kLayoutColumn4)  // u24 products: (H+1)(W+1) and D+2 below 2^24
      P.vol32 = (w1 * h1 * (d1 + 1ull) * 4ull < (1ull << 32) && w1 * h1 < (1ull << 24)) ? 1u : 0u;
    else
      P.vol32 = (w1 * h1 * d1 * 8ull < (1ull << 32) && d1 * h1 < (1ull << 24) && w1 < (1ull << 24))
                    ? 1u : 0u;
    if (h->variant & 8u) P.vol32 = 0u;  // variant bit 3: force the 64-bit gather (tests)
  }
  return P;
}

int check_handle(vptmcm* h) { return h ? VPTMCM_OK : VPTMCM_EINVAL; }

// Guard build: after the handle's queued work has finished, no volume gather
// left the volume allocation and every guard zone still holds poison; the
// product (VPT_GUARD 0) checks nothing.
int guard_check(vptmcm* h, const char* where) {
  if (!VPT_GUARD) return VPTMCM_OK;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->grp_stream) HIPCHK(h, hipStreamSynchronize(h->grp_stream));
  uint32_t oob = 0u;
  HIPCHK(h, guard_take_oob(&oob));
  if (oob) FAIL(h, VPTMCM_EHIP, "guard: %s: a volume gather left the volume allocation (templates 0x%x)", where, oob);
  const std::string g = guard_scan();
  if (!g.empty()) FAIL(h, VPTMCM_EHIP, "guard: %s: %s", where, g.c_str());
  return VPTMCM_OK;
}

// Work other than a march is enqueued on the handle's stream: the stream no
// longer ends with a signalling march (vptmcm::done_pending) or with one that
// packed the composite buffer (vptmcm::pack_fresh).
void stream_op(vptmcm* h) {
  h->done_pending = false;
  h->pack_fresh = false;
}

// The handle's stream for enqueueing anything but the march itself: every
// such enqueue names the stream through this helper, so the completion flag
// and the packed composite buffer can only stand while a march really is the
// stream's last work (the march launch in do_march is the one raw use).
hipStream_t enq(vptmcm* h) {
  stream_op(h);
  return h->stream;
}

// MarchParams::bins_lut (march MODE 6 / 7): the wavelength bin as a step
// function of the draw h5. lambda_of(h5) = fma(f32(h5) * 2^-32, max - min,
// min) is monotone in h5 when max >= min (every operation rounds
// monotonically) and bin_of counts the padded boundaries b_i with
// !(lambda < b_i), so bin(h5) = #{i : h5 >= T_i}, T_i the first h5 whose
// lambda reaches b_i, found by bisection on the f32 expression the kernel
// evaluates. Per cell of 2^22 draws the table holds the bin at the cell start
// and the one threshold inside the cell; boundaries closer than about
// (max - min) / 1024 (two distinct thresholds in one cell) keep the
// comparison search. The table is checked against bin_of's rule at every
// threshold and its neighbours and on a 2^16-point grid before it is enabled.
int build_bin_lut(vptmcm* h) {
  h->bin_lut_ok = false;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));  // no launch still reads the table
  const float ident[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  const MarchParams Q = make_params(h, ident, 0u);
  if (!Q.bins_sorted || !Q.bins_padded || !(Q.max_lam >= Q.min_lam)) return VPTMCM_OK;
  const float d = Q.max_lam - Q.min_lam, mn = Q.min_lam;
  auto lam = [&](uint64_t v) { return std::fmaf((float)(uint32_t)v * 2.3283064365386963e-10f, d, mn); };
  auto bin_rule = [&](uint64_t v) {  // bin_of's padded search
    const float l = lam(v);
    uint32_t b = 0u;
    for (int i = 1; i < kMaxBins; i++) b += !(l < Q.lam_pad[i]) ? 1u : 0u;
    return b;
  };
  uint64_t T[kMaxBins];
  int nt = 0;
  for (int i = 1; i < kMaxBins; i++) {
    const float b = Q.lam_pad[i];
    if (!std::isfinite(b)) continue;  // the +inf padding never counts
    uint64_t lo = 0, hi = 1ull << 32;  // first v in [0, 2^32) with !(lam(v) < b), else 2^32
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (!(lam(mid) < b)) hi = mid; else lo = mid + 1;
    }
    T[nt++] = lo;
  }
  uint32_t* thr = h->bin_lut_host;
  uint8_t* bk = reinterpret_cast<uint8_t*>(h->bin_lut_host + kBinLutCells);
  for (uint32_t c = 0; c < kBinLutCells; c++) {
    const uint64_t c0 = (uint64_t)c << kBinLutShift, c1 = c0 + (1ull << kBinLutShift);
    uint32_t base = 0u, k = 0u;
    uint64_t t = 0;
    for (int j = 0; j < nt; j++) {
      if (T[j] <= c0) {
        base++;
      } else if (T[j] < c1) {
        if (k && T[j] != t) return VPTMCM_OK;  // two distinct thresholds in one cell
        t = T[j];
        k++;
      }
    }
    thr[c] = k ? (uint32_t)t : 0u;
    bk[c] = (uint8_t)(base | (k << 4));
  }
  auto lut_bin = [&](uint64_t v) {
    const uint32_t c = (uint32_t)(v >> kBinLutShift);
    return (bk[c] & 15u) + ((uint32_t)v >= thr[c] ? (bk[c] >> 4) : 0u);
  };
  for (int j = 0; j < nt; j++)
    for (int64_t e = -2; e <= 2; e++) {
      const int64_t v = (int64_t)T[j] + e;
      if (v >= 0 && v < (1ll << 32) && lut_bin((uint64_t)v) != bin_rule((uint64_t)v)) return VPTMCM_OK;
    }
  for (uint64_t v = 0; v < (1ull << 32); v += 0x10001ull)
    if (lut_bin(v) != bin_rule(v)) return VPTMCM_OK;
  HIPCHK(h, hipMemcpyAsync(h->bin_lut, h->bin_lut_host, sizeof h->bin_lut_host,
                           hipMemcpyHostToDevice, enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->bin_lut_ok = true;
  return VPTMCM_OK;
}

// The start event of the next march launch: the region's begin event for the
// first timed launch (stamped by the dispatch packet itself), else none.
int time_slot(vptmcm* h, hipEvent_t* beg) {
  *beg = nullptr;
  if (!h->timing) return VPTMCM_OK;
  if (!h->region.beg) {
    HIPCHK(h, hipEventCreateWithFlags(&h->region.beg, hipEventDisableSystemFence));
    HIPCHK(h, hipEventCreateWithFlags(&h->region.end, hipEventDisableSystemFence));
  }
  if (h->launches++ == 0) {
    if (h->time_begin_marker) HIPCHK(h, hipEventRecord(h->region.beg, enq(h)));
    else *beg = h->region.beg;
  }
  h->region_closed = false;
  return VPTMCM_OK;
}

// Enqueue the region's end event behind the last timed launch (once).
int time_close(vptmcm* h) {
  if (!h->timing || h->launches == 0 || h->region_closed) return VPTMCM_OK;
  if (h->time_stop) {
    h->region_closed = true;
    return VPTMCM_OK;
  }
  HIPCHK(h, hipEventRecord(h->region.end, enq(h)));
  h->region_closed = true;
  stream_op(h);  // work behind the signalling march
  return VPTMCM_OK;
}

// The macro-cell tuner (vptmcm::maj_tune): forget the ratio (the volume, the
// TF, the camera or the march parameters changed: the trade-off moved). A pair
// in flight is abandoned (its events are simply recorded again later).
void maj_tune_reset(vptmcm* h) {
  for (uint32_t n = 0; n <= kMaxFusedPasses; n++) {
    h->maj_tune.ratio[n] = h->maj_tune.half[n] = -1.0f;
    h->maj_tune.quads[n] = 0;
    h->maj_tune.launches[n] = 0;
    h->maj_tune.first[n] = 0;
  }
  h->maj_tune.epoch++;
}

// A new camera: measure again, but keep each size's ratio as the pick until
// the new one decides (a camera that moves every launch — an interactive
// rotation — never gets a pair, and keeps the last decision).
void maj_tune_camera(vptmcm* h) {
  for (uint32_t n = 0; n <= kMaxFusedPasses; n++) {
    h->maj_tune.half[n] = -1.0f;
    h->maj_tune.quads[n] = 0;
  }
  h->maj_tune.cam_launches = 0;
  h->maj_tune.epoch++;
}

// Re-lay out the cells of the blocks that arrived since the last relayout
// (vptmcm::vol_dirty) from the staging copy, on the handle's stream.
int flush_relayout(vptmcm* h) {
  if (!h->vol_dirty) return VPTMCM_OK;
  h->vol_dirty = false;
  const bool brick = h->layout == kLayoutBrick8;
  const uint32_t n[3] = {h->vol_c1[0] - h->vol_c0[0], h->vol_c1[1] - h->vol_c0[1], h->vol_c1[2] - h->vol_c0[2]};
  if (h->layout == kLayoutColumn4) {
    // quad k holds voxel slice clamp(k - 1): the cells' z range [z0, z1) needs
    // quads [z0, z1 + 1), clipped to the column's D + 2
    const uint32_t z1 = std::min(h->vol_c1[2] + 1u, h->D + 2u);
    const uint32_t nq[3] = {n[0], n[1], z1 - h->vol_c0[2]};
    HIPCHK(h, launch_column4(h->vol_lin, h->W, h->H, h->D, h->vol_c8, enq(h), h->vol_c0, nq));
  } else {
    HIPCHK(h, launch_corner8(h->vol_lin, h->W, h->H, h->D, brick ? (h->W + kBrickCells) / kBrickCells : 0u,
                             brick ? (h->H + kBrickCells) / kBrickCells : 0u, h->vol_c8, enq(h),
                             h->vol_c0, n));
  }
  if (h->maj_ok) {  // the macro cells the re-laid-out cells fall in
    uint32_t m0[3], mn[3];
    const uint32_t lim[3] = {h->maj_nx, h->maj_ny, h->maj_nz};
    for (int k = 0; k < 3; k++) {
      m0[k] = h->vol_c0[k] >> h->maj_shift;
      const uint32_t m1 = std::min((h->vol_c1[k] + (1u << h->maj_shift) - 1u) >> h->maj_shift, lim[k]);
      mn[k] = m1 > m0[k] ? m1 - m0[k] : 0u;
    }
    HIPCHK(h, launch_macro_minmax(h->vol_lin, h->W, h->H, h->D, h->maj_shift, h->maj_nx, h->maj_ny, m0, mn,
                                  h->maj_mm, enq(h)));
    h->maj_valid = false;
    maj_tune_reset(h);
  }
  return guard_check(h, "relayout");
}

// A device-list handle whose composite is sharded over its replicas (PEER).
bool sharded(const vptmcm* h) { return !h->peers.empty() && h->group_transport == VPTMCM_GROUP_PEER; }

// Replica k of a device-list handle (0: the handle itself).
vptmcm* replica_of(vptmcm* h, uint32_t k) { return k ? h->peers[k - 1] : h; }

// Before replica c writes its PEER pack buffer b (owner o = replica 0): every
// shard kernel that read buffer b in the last composite using it has finished
// (its replicas' grp_shard[b]); nothing to wait for when the host already
// knows that composite complete.
int fence_pack_buffer(vptmcm* o, vptmcm* c, uint32_t b) {
  if (o->grp_use_seq[b] <= o->grp_synced_seq) return VPTMCM_OK;
  const uint32_t n = 1u + (uint32_t)o->peers.size();
  for (uint32_t k = 0; k < n; k++) HIPCHK(c, hipStreamWaitEvent(enq(c), replica_of(o, k)->grp_shard[b], 0));
  return VPTMCM_OK;
}

// Fold the finished pairs into the ratios, oldest first (non-blocking: stops
// at the first pair the GPU has not finished).
void maj_tune_harvest(vptmcm* h) {
  auto& t = h->maj_tune;
  while (t.count > 0) {
    auto& pr = t.pairs[t.head];
    if (pr.stage == 1) return;  // the open pair: its second launch is not enqueued yet
    if (pr.stage == 2 && (hipEventQuery(pr.e[0]) != hipSuccess || hipEventQuery(pr.e[1]) != hipSuccess)) {
      (void)hipGetLastError();  // a not-ready query is not an error
      return;
    }
    t.head = (t.head + 1) % vptmcm::kPairs;
    t.count--;
    if (pr.stage != 2 || pr.epoch != t.epoch) continue;  // abandoned, or from before a reset
    float ms[2] = {0.0f, 0.0f};
    bool ok = true;
    for (int k = 0; k < 2; k++)
      ok = ok && hipEventElapsedTime(&ms[k], pr.b[k], pr.e[k]) == hipSuccess && ms[k] > 0.0f;
    if (!ok) {
      (void)hipGetLastError();
      continue;
    }
    const float on = pr.first ? ms[0] : ms[1], off = pr.first ? ms[1] : ms[0];
    const float r = on / off;
    const uint32_t n = pr.n;
    if (t.half[n] < 0.0f || t.half_first[n] == pr.first) {  // wait for a pair of the other order
      t.half[n] = r;
      t.half_first[n] = (uint8_t)pr.first;
      continue;
    }
    const float rr = sqrtf(t.half[n] * r);
    t.half[n] = -1.0f;
    float& q = t.ratio[n];
    q = (q < 0.0f || t.quads[n] == 0) ? rr : 0.5f * q + 0.5f * rr;  // (a previous camera's ratio is replaced)
    if (t.quads[n] < 255) t.quads[n]++;
    if (t.quads[n] >= vptmcm::kQuads) t.choice = q < 1.0f ? 1 : 0;
    if (const char* v = getenv("VPTMCM_MAJ_TRACE"))
      if (v[0] == '1')
        fprintf(stderr, "maj_tune: pairs n=%u on %.3f off %.3f us/pass, ratio %.4f (both orders %.4f) -> %.4f, "
                "choice %d\n", n, (double)(on * 1e3f / n), (double)(off * 1e3f / n), (double)r, (double)rr,
                (double)q, t.choice);
  }
}

// The skip for the next launch of n passes, and the probe events to time it
// with (none unless it is one of a pair; never while the caller times a
// region, whose launches stay untouched).
int maj_tune_pick(vptmcm* h, const float* mvp, uint32_t n, hipEvent_t* pb, hipEvent_t* pe) {
  auto& t = h->maj_tune;
  *pb = *pe = nullptr;
  if (t.mode != 2) return t.mode;
  if (!h->timing) maj_tune_harvest(h);  // (no event queries inside the caller's timed regions)
  if (memcmp(t.mvp, mvp, sizeof t.mvp) != 0) {  // the volume's screen coverage moved
    memcpy(t.mvp, mvp, sizeof t.mvp);
    maj_tune_camera(h);
  } else if (t.cam_launches < 0xffffffffu) {
    t.cam_launches++;
  }
  const bool decided = t.quads[n] >= vptmcm::kQuads;
  const int pick = t.ratio[n] < 0.0f ? t.choice : t.ratio[n] < 1.0f ? 1 : 0;
  auto* open = t.count > 0 ? &t.pairs[(t.head + t.count - 1) % vptmcm::kPairs] : nullptr;
  if (open && open->stage != 1) open = nullptr;
  if (open && (h->timing || open->n != n || open->epoch != t.epoch)) {
    open->stage = 0;  // its second launch would not be adjacent or alike: abandoned
    open = nullptr;
  }
  if (h->timing) return pick;
  if (open) {  // the pair's second launch, the other way
    open->stage = 2;
    *pb = open->b[1];
    *pe = open->e[1];
    return open->first ^ 1;
  }
  // a pair starts once the camera held for a launch (its second launch is then
  // likely to share it), at once while undecided, else every 16 launches
  if (t.count == vptmcm::kPairs || t.cam_launches == 0 || !(!decided || ++t.launches[n] >= 16)) return pick;
  auto& pr = t.pairs[(t.head + t.count) % vptmcm::kPairs];
  for (int k = 0; k < 2; k++)
    if ((!pr.b[k] && hipEventCreate(&pr.b[k]) != hipSuccess) || (!pr.e[k] && hipEventCreate(&pr.e[k]) != hipSuccess)) {
      (void)hipGetLastError();
      return pick;
    }
  t.count++;
  pr.first = t.first[n];
  pr.n = n;
  pr.epoch = t.epoch;
  pr.stage = 1;
  t.first[n] ^= 1;
  t.launches[n] = 0;
  *pb = pr.b[0];
  *pe = pr.e[0];
  return pr.first;
}

// One march launch of n <= kMaxFusedPasses passes (seeds) with matrix mvp.
int do_march(vptmcm* h, const float* mvp, const uint32_t* seeds, uint32_t n) {
  if (!h->volume_ready) FAIL(h, VPTMCM_ESTATE, "render: no volume set (setVolume first)");
  if (n == 0) return VPTMCM_OK;
  if (n > kMaxFusedPasses) FAIL(h, VPTMCM_EINVAL, "internal: %u passes in one launch", n);
  if (int rc = flush_relayout(h)) return rc;
  if (h->maj_ok && !h->maj_valid) {  // the volume or the TF changed since the codes were built
    HIPCHK(h, launch_macro_alpha(h->maj_mm, h->maj_n, h->tf_rowmax, h->maj_q, h->maj_bytes, enq(h)));
    h->maj_valid = true;
  }
  MarchParams P = make_params(h, mvp, seeds[0]);
  hipEvent_t tb = nullptr, te = nullptr;  // a tuner probe's events
  if (h->maj_ok && maj_tune_pick(h, mvp, n, &tb, &te) == 1) {
    P.maj_on = 1u;
    P.maj_shift = h->maj_shift;
    P.maj_nx = h->maj_nx;
    P.maj_ny = h->maj_ny;
    P.maj_bytes = h->maj_bytes;
  }
  PassSeeds PS;
  memset(&PS, 0, sizeof PS);
  PS.n = n;
  for (uint32_t k = 0; k < n; k++) PS.seed[k] = seeds[k];
  P.dark = h->dark;
  hipEvent_t eb = nullptr, ee = nullptr;
  int rc = time_slot(h, &eb);
  if (rc) return rc;
  if (h->timing && h->time_stop) ee = h->region.end;
  if (tb) {  // a tuner probe (never inside a timed region)
    eb = tb;
    ee = te;
  }
  const uint8_t* vol = h->layout != kLayoutLinear ? (const uint8_t*)h->vol_c8 : h->vol_lin;
  const uint32_t c = h->sched_cur, nf = sched_flag_bytes(h->n_tiles);
  TileSched T{h->sched + c * nf, h->sched + (c ^ 1u) * nf, h->sched_prev, nullptr, nullptr, nullptr,
              h->sched_changed + c, h->sched_changed + (c ^ 1u)};
  // the previous launch's deal may stand unless this is the handle's first
  // launch (only launches touch the schedule state)
  P.launch_seq = (uint32_t)(h->march_launches + 1u);
  P.sched_reuse = (h->sched_cache && h->march_launches > 0u) ? 1u : 0u;
  const bool signal = h->done_on && h->kind == VPTMCM_RENDERER_SPECTRAL;
  // (measurement builds, VPT_STAMP != 0, store neither rgb32 nor the pack: the
  // all-reduce then runs k_pack, whose inputs are as invalid as those builds' results)
  const bool packable = !VPT_STAMP && h->kind == VPTMCM_RENDERER_SPECTRAL && h->band_y0 == 0 &&
                        h->band_y1 == h->R;
  const bool pack = packable && (h->comm || (h->grp_owner && sharded(h->grp_owner)));
  int pack_buf = -1;
  if (pack && h->comm) {  // the buffer is free once the all-reduce issued two composites ago is done
    HIPCHK(h, hipStreamWaitEvent(enq(h), h->comp_done[h->comp_next], 0));
    T.pack = h->comp[h->comp_next];
  } else if (pack) {  // the next composite's buffer, free once composite j - 2's shards have read it
    vptmcm* o = h->grp_owner;
    pack_buf = (int)(o->grp_seq & 1u);
    if (int rc = fence_pack_buffer(o, h, (uint32_t)pack_buf)) return rc;
    T.pack = h->grp_pack[pack_buf];
  }
  if (signal) {  // every block of the grid counts once (committed below, once launched)
    P.done_target = h->done_total + tile_blocks(P, kMarchBlock);
    P.done_seq = h->done_seq + 1u;
    T.done_ctr = h->done_ctr;
    T.done_flag = h->done_dev;
  }
  // variant bit 1: raster mapping; bit 7: round 2's XCD-by-XCD slot order
  P.sched = (h->n_tiles > kSchedMaxTiles || (h->variant & 2u)) ? 1u : (h->variant & 128u) ? 2u : 0u;
  if (h->kind == VPTMCM_RENDERER_RGB)
    HIPCHK(h, launch_march_rgb(h->layout, P, PS, T, h->photons, vol, h->tf_rgb, h->rgba, h->rgb32,
                               h->stream, eb, ee, &h->last_launch,
                               (h->variant & 256u) ? nullptr : h->maj_q));  // variant bit 8: no bound
  else
    HIPCHK(h, launch_march(h->layout, h->variant, P, PS, T, h->photons, vol, h->tf_rg, h->tf_b4,
                           h->tf_brow, h->light, h->rgba, h->rgb32, h->stream, eb, ee, h->tf_rows,
                           h->tf_rowmap, h->bin_lut, &h->last_launch, h->maj_q));
  h->march_launches++;
  h->sched_cur = c ^ 1u;
  h->grp_dirty = true;
  if (signal) {
    h->done_total = P.done_target;
    h->done_seq = P.done_seq;
  }
  h->done_pending = signal;
  h->pack_fresh = pack;
  h->pack_buf = pack_buf;
  return guard_check(h, "march");
}

// Launch the queued render() passes (see vptmcm::pend_n) as one march.
int flush_renders(vptmcm* h) {
  if (h->pend_n == 0) return VPTMCM_OK;
  HIPCHK(h, hipSetDevice(h->device));
  const uint32_t n = h->pend_n;
  h->pend_n = 0;
  return do_march(h, h->pend_mvp, h->pend_seeds, n);
}

// ---- communicator waits (see vptmcm::comm_timeout_ms)

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// VPTMCM_COMM_TRACE=1: timestamped lines on stderr at each stage of the
// communicator's setup and failure handling (diagnostics of RCCL hangs).
void comm_trace(const char* fmt, ...) {
  const char* on = getenv("VPTMCM_COMM_TRACE");
  if (!on || on[0] != '1') return;
  char b[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  fprintf(stderr, "[vptmcm comm %lld ms] %s\n", (long long)now_ms(), b);
  fflush(stderr);
}

// Abort the communicator after an error or a timeout: RCCL kernels still
// waiting for a peer observe the abort flag and exit, so the handle's streams
// drain. The communicator exists only once its initialisation has returned
// (vptmcm_comm_init), i.e. past RCCL's bootstrap, so the abort does not wait
// for a peer. Every later communicator call returns VPTMCM_ECOMM, and the
// handle's stream waits stay bounded (vptmcm::comm_failed).
int comm_fail(vptmcm* h, const char* what, const char* why) {
  comm_trace("abort: start (%s)", what);
  if (h->comm) (void)ncclCommAbort(h->comm);
  comm_trace("abort: returned");
  h->comm = nullptr;
  h->comm_failed = true;
  FAIL(h, VPTMCM_ECOMM, "%s: %s (communicator aborted; rank %d of %d)", what, why, h->rank, h->nranks);
}

// The communicator's asynchronous state: OK, 1 (still in progress) or the
// VPTMCM_ECOMM of comm_fail.
int comm_state(vptmcm* h, const char* what) {
  ncclResult_t st = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError(h->comm, &st);
  if (r != ncclSuccess) st = r;
  if (st == ncclSuccess) return VPTMCM_OK;
  if (st == ncclInProgress) return 1;
  return comm_fail(h, what, ncclGetErrorString(st));
}

// Wait until a non-blocking communicator call (init, or an enqueue that
// returned ncclInProgress) has completed.
int comm_settle(vptmcm* h, const char* what) {
  const int64_t t0 = now_ms();
  int64_t last = t0;
  for (uint32_t spin = 0;; spin++) {
    const int rc = comm_state(h, what);
    if (rc <= 0) {
      comm_trace("%s: settled rc=%d after %lld ms", what, rc, (long long)(now_ms() - t0));
      return rc;
    }
    if (now_ms() - last >= 1000) {
      last = now_ms();
      comm_trace("%s: in progress after %lld ms", what, (long long)(last - t0));
    }
    if (now_ms() - t0 > h->comm_timeout_ms) {
      char b[96];
      snprintf(b, sizeof b, "no progress after %lld ms (a peer rank died or hangs?)",
               (long long)h->comm_timeout_ms);
      return comm_fail(h, what, b);
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Check the result of an RCCL call on a non-blocking communicator.
int comm_call(vptmcm* h, ncclResult_t r, const char* what) {
  if (r == ncclInProgress) return comm_settle(h, what);
  if (r != ncclSuccess) return comm_fail(h, what, ncclGetErrorString(r));
  return VPTMCM_OK;
}

// Block until stream s has drained. With a communicator the stream may hold
// RCCL work (or wait on it), so the wait polls the stream and the
// communicator's asynchronous error, spinning first (a composite is a few
// hundred microseconds), and gives up after the communicator timeout.
int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int wait_stream(vptmcm* h, hipStream_t s, const char* what) {
  if (!h->comm && !h->comm_failed) {
    if (h->sync_spin_us > 0) {  // spin, then block
      const int64_t t0 = now_us();
      for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return VPTMCM_OK;
        if (e != hipErrorNotReady) FAIL(h, VPTMCM_EHIP, "%s: %s", what, hipGetErrorString(e));
        if (now_us() - t0 > h->sync_spin_us) break;
      }
    }
    HIPCHK(h, hipStreamSynchronize(s));
    return VPTMCM_OK;
  }
  const int64_t t0 = now_ms();
  for (uint32_t spin = 0;; spin++) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return VPTMCM_OK;
    if (e != hipErrorNotReady) FAIL(h, VPTMCM_EHIP, "%s: %s", what, hipGetErrorString(e));
    if ((spin & 255u) == 0u) {
      const int rc = h->comm ? comm_state(h, what) : VPTMCM_OK;
      if (rc < 0) return rc;
      if (now_ms() - t0 > h->comm_timeout_ms) {
        if (!h->comm)
          FAIL(h, VPTMCM_ECOMM, "%s: stream not drained %lld ms after the communicator's abort", what,
               (long long)h->comm_timeout_ms);
        char b[96];
        snprintf(b, sizeof b, "stream not drained after %lld ms (a peer rank died or hangs?)",
                 (long long)h->comm_timeout_ms);
        return comm_fail(h, what, b);
      }
    }
    if (now_ms() - t0 > 20) std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

// PCG-RXS-M-XS (pcg.wgsl:3-7) on the host, for the replicas' seed streams.
uint32_t pcg_host(uint32_t v) {
  uint32_t x = v * 747796405u + 2891336453u;
  x = ((x >> ((x >> 28u) + 4u)) ^ x) * 277803737u;
  return (x >> 22u) ^ x;
}

// Seed bits of replica k for the pass whose replica-0 seed bits are s: the
// seed stream of rank k of the one-process-per-GPU path (bench.py,
// configs.seed_bits), so N replicas in one process and N processes render the
// same photons.
uint32_t replica_seed(uint32_t s, uint32_t k) { return k ? pcg_host(s ^ (k * 0x9E3779B9u)) : s; }

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

void worker_main(ReplicaWorker* w) {
  uint64_t seen = 0;
  for (;;) {
    const int64_t t0 = now_us();
    uint64_t p;
    while ((p = w->posted.load(std::memory_order_acquire)) == seen) {
      if (w->quit.load(std::memory_order_acquire)) return;
      if (now_us() - t0 > w->spin_us) {
        std::unique_lock<std::mutex> lk(w->m);
        w->cv.wait(lk, [&] {
          return w->posted.load(std::memory_order_acquire) != seen || w->quit.load(std::memory_order_acquire);
        });
      } else {
        cpu_relax();
      }
    }
    seen = p;
    try {
      w->rc = w->job.call(w->job.f, w->c);
    } catch (...) {  // nothing may escape a thread (std::terminate)
      w->c->err = "internal: exception in a replica's worker thread";
      w->rc = VPTMCM_ENOMEM;
    }
    w->finished.store(seen, std::memory_order_release);
  }
}

void post(ReplicaWorker* w, const ReplicaJob& job) {
  w->job = job;
  {
    std::lock_guard<std::mutex> lk(w->m);
    w->posted.store(w->posted.load(std::memory_order_relaxed) + 1, std::memory_order_release);
  }
  w->cv.notify_one();
}

// Wait for the worker's last job: spin, then sleep in short slices (an
// ingest job is milliseconds of host-to-device copy).
int await(ReplicaWorker* w, int64_t spin_us) {
  const uint64_t want = w->posted.load(std::memory_order_relaxed);
  const int64_t t0 = now_us();
  while (w->finished.load(std::memory_order_acquire) != want) {
    if (now_us() - t0 > spin_us)
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    else
      cpu_relax();
  }
  return w->rc;
}

void stop_workers(vptmcm* h);

// Without every worker (thread creation failed) the handle forwards serially.
void start_workers(vptmcm* h) {
  try {
    for (vptmcm* c : h->peers) {
      auto w = std::make_unique<ReplicaWorker>();
      w->c = c;
      // an idle worker spins briefly (back-to-back forwarded calls: render_passes
      // then synchronize) and then sleeps, so a display loop does not keep N
      // cores busy between frames
      w->spin_us = std::min<int64_t>(std::max<int64_t>(h->sync_spin_us, 0), 200);
      w->th = std::thread(worker_main, w.get());
      h->workers.push_back(std::move(w));
    }
  } catch (...) {
    stop_workers(h);
  }
}

void stop_workers(vptmcm* h) {
  for (auto& w : h->workers) {
    {
      std::lock_guard<std::mutex> lk(w->m);
      w->quit.store(true, std::memory_order_release);
    }
    w->cv.notify_one();
  }
  for (auto& w : h->workers)
    if (w->th.joinable()) w->th.join();
  h->workers.clear();
}

// A peer's failure is reported on h, naming the replica.
int peer_failed(vptmcm* h, const vptmcm* c, int rc) {
  try {
    h->err = "replica " + std::to_string(c->replica) + " (device " + std::to_string(c->device) + "): " + c->err;
  } catch (...) {  // out of host memory for the message: the code still says what failed
  }
  return rc;
}

// Run the same single-replica operation on replica 0 (h, when self) and every
// peer of a device-list handle: on the peers' worker threads with h's part on
// the caller's thread, all at once, or one after another without workers. The
// operation must touch only its own replica (and read shared inputs). Every
// replica runs it; the first failure in replica order is the result.
// f runs under a catch-all on every thread: an exception (std::bad_alloc from
// an error message's formatting) becomes an error code instead of unwinding
// the caller's stack while workers still call through &f, or escaping through
// the C ABI; every worker is awaited before this returns.
template <class F>
int guarded(vptmcm* c, const F& f) {
  try {
    return f(c);
  } catch (...) {
    c->err = "internal: exception in a forwarded operation";
    return VPTMCM_ENOMEM;
  }
}

template <class F>
int run_replicas(vptmcm* h, bool self, const F& f) {
  if (h->workers.empty()) {
    if (self)
      if (int rc = guarded(h, f)) return rc;
    for (vptmcm* c : h->peers)
      if (int rc = guarded(c, f)) return peer_failed(h, c, rc);
    return VPTMCM_OK;
  }
  ReplicaJob job;
  job.call = [](const void* p, vptmcm* c) { return (*static_cast<const F*>(p))(c); };
  job.f = &f;
  for (auto& w : h->workers) post(w.get(), job);
  const int rc0 = self ? guarded(h, f) : VPTMCM_OK;
  int first = VPTMCM_OK;
  const vptmcm* bad = nullptr;
  for (auto& w : h->workers) {
    const int rc = await(w.get(), h->sync_spin_us);
    if (rc && !bad) {
      first = rc;
      bad = w->c;
    }
  }
  if (rc0) return rc0;
  return bad ? peer_failed(h, bad, first) : VPTMCM_OK;
}

template <class F>
int for_peers(vptmcm* h, const F& f) { return run_replicas(h, false, f); }

// Replica 0 (h) and its peers.
template <class F>
int for_replicas(vptmcm* h, const F& f) { return run_replicas(h, true, f); }

bool composited(const vptmcm* h) { return !h->peers.empty(); }

void free_volume(vptmcm* h) {
  if (h->vol_lin) (void)dev_free(h->vol_lin);
  if (h->vol_c8) (void)dev_free(h->vol_c8);
  if (h->maj_mm) (void)dev_free(h->maj_mm);
  if (h->maj_q) (void)dev_free(h->maj_q);
  h->vol_lin = nullptr;
  h->vol_c8 = nullptr;
  h->maj_mm = nullptr;
  h->maj_q = nullptr;
  h->maj_ok = h->maj_valid = false;
  h->volume_ready = false;
  h->vol_done = false;
  h->vol_dirty = false;
  h->W = h->H = h->D = 0;
}

}  // namespace

extern "C" {

const char* vptmcm_version(void) { return "vptmcm 0.1.0 (gfx950)"; }

const char* vptmcm_last_error(const vptmcm* h) {
  return h ? h->err.c_str() : g_create_error.c_str();
}

// ---- device-list handles (vptmcm_config::n_devices)

// Pixel shard k of N of the PEER composite: [p0, p1), whole 256-pixel blocks
// of the composite kernel except the last (a shard may be empty for tiny R).
static void shard_range(size_t npx, uint32_t n, uint32_t k, size_t* p0, size_t* p1) {
  const size_t step = ((npx + n - 1) / n + 255) / 256 * 256;
  *p0 = std::min(npx, (size_t)k * step);
  *p1 = std::min(npx, *p0 + step);
}

// The composite's buffers and events. PEER: two pack buffers, a composite
// stream and a shard event per replica; on devices[0] the composite image and
// counts; xGMI peer access between EVERY pair of distinct devices (a shard
// kernel on device k reads every replica's pack and writes devices[0]'s
// image). RCCL: one pack buffer per replica, the reduced sum on devices[0] and
// one communicator per replica by ncclCommInitAll (one process: no bootstrap
// peers that could fail to arrive).
static int group_alloc(vptmcm* h, const int32_t* devs, uint32_t n) {
  const size_t npx = (size_t)h->R * h->R;
  const bool peer = h->group_transport == VPTMCM_GROUP_PEER;
  int rc = for_replicas(h, [&](vptmcm* c) {
    HIPCHK(c, hipSetDevice(c->device));
    for (int k = 0; k < (peer ? 2 : 1); k++) HIPCHK(c, dev_alloc(&c->grp_pack[k], npx * sizeof(float4)));
    HIPCHK(c, hipEventCreateWithFlags(&c->grp_packed, hipEventDisableTiming));
    if (peer) {
      HIPCHK(c, hipStreamCreateWithFlags(&c->grp_stream, hipStreamNonBlocking));
      for (auto& e : c->grp_shard) {
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(e, c->grp_stream));
      }
      shard_range(npx, n, c->replica, &c->grp_p0, &c->grp_p1);
      const size_t m = std::max<size_t>(c->grp_p1 - c->grp_p0, 1);  // (an empty shard keeps a stub)
      HIPCHK(c, dev_alloc(&c->grp_rgb32, m * 3 * sizeof(float)));
      HIPCHK(c, hipMemsetAsync(c->grp_rgb32, 0, m * 3 * sizeof(float), c->grp_stream));
      HIPCHK(c, dev_alloc(&c->grp_rgba, m * 4 * sizeof(uint16_t)));
      HIPCHK(c, hipMemsetAsync(c->grp_rgba, 0, m * 4 * sizeof(uint16_t), c->grp_stream));
      HIPCHK(c, dev_alloc(&c->grp_counts, m * sizeof(float)));
      HIPCHK(c, hipMemsetAsync(c->grp_counts, 0, m * sizeof(float), c->grp_stream));
      HIPCHK(c, hipStreamSynchronize(c->grp_stream));
    }
    return VPTMCM_OK;
  });
  if (rc) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  if (!peer) {
    HIPCHK(h, dev_alloc(&h->grp_gather, npx * sizeof(float4)));
    HIPCHK(h, dev_alloc(&h->grp_rgb32, npx * 3 * sizeof(float)));
    HIPCHK(h, hipMemsetAsync(h->grp_rgb32, 0, npx * 3 * sizeof(float), enq(h)));
    HIPCHK(h, dev_alloc(&h->grp_rgba, npx * 4 * sizeof(uint16_t)));
    HIPCHK(h, hipMemsetAsync(h->grp_rgba, 0, npx * 4 * sizeof(uint16_t), enq(h)));
  }
  for (int k = 0; k < 2; k++) {
    HIPCHK(h, hipEventCreateWithFlags(&h->grp_done[k], hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(h->grp_done[k], enq(h)));
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (peer) {
    // every ordered pair of distinct devices (a shard kernel on `from` reads
    // and writes `to`'s memory); without peer access a kernel cannot reach the
    // other device at all, so the PEER transport is refused (RCCL remains)
    for (uint32_t i = 0; i < n; i++)
      for (uint32_t j = 0; j < n; j++) {
        if (devs[i] == devs[j]) continue;
        int can = 0;
        HIPCHK(h, hipDeviceCanAccessPeer(&can, devs[i], devs[j]));
        if (!can)
          FAIL(h, VPTMCM_EINVAL, "devices %d and %d have no peer access: the PEER group transport needs "
               "it between every pair (use VPTMCM_GROUP_RCCL)", devs[i], devs[j]);
        HIPCHK(h, hipSetDevice(devs[i]));
        const hipError_t e = hipDeviceEnablePeerAccess(devs[j], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
          FAIL(h, VPTMCM_EHIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", devs[i], devs[j], hipGetErrorString(e));
        (void)hipGetLastError();  // clear an already-enabled status
      }
    HIPCHK(h, hipSetDevice(h->device));
  } else {
    h->grp_comms.assign(n, nullptr);
    std::vector<int> dl(devs, devs + n);
    comm_trace("group: ncclCommInitAll n=%u", n);
    const ncclResult_t r = ncclCommInitAll(h->grp_comms.data(), (int)n, dl.data());
    if (r != ncclSuccess) {
      h->grp_comms.clear();
      FAIL(h, VPTMCM_ECOMM, "ncclCommInitAll over %u devices: %s", n, ncclGetErrorString(r));
    }
  }
  return VPTMCM_OK;
}

static int create_group(const vptmcm_config* cfg, vptmcm** out) {
  const uint32_t n = cfg->n_devices;
  if (n > VPTMCM_MAX_DEVICES) {
    g_create_error = "vptmcm_create: at most VPTMCM_MAX_DEVICES (8) devices";
    return VPTMCM_EINVAL;
  }
  if (cfg->group_transport > VPTMCM_GROUP_RCCL) {
    g_create_error = "vptmcm_create: unknown group transport";
    return VPTMCM_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_create_error = "vptmcm_create: no HIP device available";
    return VPTMCM_EHIP;
  }
  for (uint32_t k = 0; k < n; k++) {
    if (cfg->devices[k] < 0 || cfg->devices[k] >= ndev) {
      g_create_error = "vptmcm_create: devices[" + std::to_string(k) + "] = " +
                       std::to_string(cfg->devices[k]) + " is not a device ordinal (" +
                       std::to_string(ndev) + " devices)";
      return VPTMCM_EINVAL;
    }
    for (uint32_t j = 0; j < k && cfg->group_transport == VPTMCM_GROUP_RCCL; j++)
      if (cfg->devices[j] == cfg->devices[k]) {
        g_create_error = "vptmcm_create: the RCCL group transport needs distinct devices (RCCL "
                         "refuses two ranks on one GPU); VPTMCM_GROUP_PEER allows repeats";
        return VPTMCM_EINVAL;
      }
  }
  // The replicas' handles are created at once, the peers on threads of their
  // own (each device's runtime initialisation and allocations overlap), replica
  // 0 on the caller's thread; then checked in replica order.
  struct Made {
    vptmcm* h = nullptr;
    int rc = VPTMCM_OK;
    std::string err;
  };
  std::vector<Made> made(n);
  auto make = [&](uint32_t k) {
    vptmcm_config one = *cfg;
    one.n_devices = 0;
    one.device = cfg->devices[k];
    try {
      made[k].rc = vptmcm_create(&one, &made[k].h);
      if (made[k].rc) made[k].err = g_create_error;  // thread-local: copied out here
    } catch (...) {  // nothing may escape a thread (std::terminate)
      made[k].rc = VPTMCM_ENOMEM;
      made[k].err = "vptmcm_create: out of host memory";
    }
  };
  std::vector<std::thread> makers;
  for (uint32_t k = 1; k < n; k++) {
    try {
      makers.emplace_back(make, k);
    } catch (...) {
      make(k);  // no thread: create it here
    }
  }
  make(0);
  for (auto& t : makers) t.join();
  int rc = VPTMCM_OK;
  std::string msg;
  for (uint32_t k = 0; k < n && !rc; k++)
    if (made[k].rc) {
      rc = made[k].rc;
      msg = k ? "replica " + std::to_string(k) + ": " + made[k].err : made[k].err;
    }
  if (rc) {
    for (auto& m : made) vptmcm_destroy(m.h);
    g_create_error = msg;
    return rc;
  }
  vptmcm* h = made[0].h;
  h->grouped = true;
  h->group_transport = cfg->group_transport;
  auto fail = [&](int code, const std::string& m) {
    vptmcm_destroy(h);
    g_create_error = m;
    return code;
  };
  for (uint32_t k = 1; k < n; k++) {
    made[k].h->replica = k;
    h->peers.push_back(made[k].h);
  }
  if (n > 1 || h->group_transport == VPTMCM_GROUP_RCCL) {
    if ((rc = group_alloc(h, cfg->devices, n))) return fail(rc, "vptmcm_create: " + h->err);
  }
  if (sharded(h))  // the replicas' marches pack for the next composite
    for (uint32_t k = 0; k < n; k++) replica_of(h, k)->grp_owner = h;
  const char* threads = getenv("VPTMCM_GROUP_THREADS");
  if (n > 1 && !(threads && threads[0] == '0')) start_workers(h);
  *out = h;
  return VPTMCM_OK;
}

// The composite of the current frame over every replica. Asynchronous: the
// readers wait for it (composite_ready, read_shards).
//
// PEER (sharded): (1) every replica packs (rgb*n, n) into its buffer j & 1 on
// its own stream, behind its march (that buffer was last read by the shard
// kernels of composite j - 2: every replica's grp_shard[j & 1], long complete
// in steady state); (2) replica k, on its composite stream, waits for
// every replica's pack and composites pixel shard k of all of them — the
// sources summed in replica order, the same f32 sums and division as one
// k_composite over whole buffers — into its own shard of the image: each
// device reads 1/N of every other replica's pack over its own links at once
// and nothing is gathered on one device (readers copy the N shards to the
// host in parallel) and records grp_shard[j & 1]. No step waits on devices[0]
// after the shards: one cross-stream hop (the packs' events) is the whole
// chain. Steps (1) and (2) run on the replicas' worker threads; a step's host enqueue starts once
// every replica has recorded the previous step's event.
//
// RCCL: every replica packs, a grouped ncclReduce sums the packs on
// devices[0], and k_composite divides there, on replica 0's stream.
static int group_composite(vptmcm* h) {
  const uint32_t n = 1u + (uint32_t)h->peers.size();
  const size_t npx = (size_t)h->R * h->R;
  const bool peer = h->group_transport == VPTMCM_GROUP_PEER;
  const uint32_t b = peer ? (h->grp_seq & 1u) : 0u;
  int rc = for_replicas(h, [&](vptmcm* c) {
    if (int r = flush_renders(c)) return r;
    HIPCHK(c, hipSetDevice(c->device));
    // PEER: the stream's last march packed buffer b already (TileSched::pack)
    const bool fresh = peer && c->pack_fresh && c->pack_buf == (int)b;
    if (!fresh) {
      if (peer) {  // buffer b is free once composite j - 2's shard kernels have read it
        if (int r = fence_pack_buffer(h, c, b)) return r;
      } else {  // the last reduce has read it (and its target)
        HIPCHK(c, hipStreamWaitEvent(enq(c), h->grp_done[b], 0));
      }
      const MarchParams P = make_params(c, kNoMatrix, 0);
      HIPCHK(c, launch_pack(P, c->photons, c->rgb32, c->grp_pack[b], enq(c)));
    }
    HIPCHK(c, hipEventRecord(c->grp_packed, enq(c)));
    return VPTMCM_OK;
  });
  if (rc) return rc;
  if (peer) {
    rc = for_replicas(h, [&](vptmcm* c) {
      HIPCHK(c, hipSetDevice(c->device));
      // every pack (this shard's previous readers ran on this stream already)
      for (uint32_t k = 0; k < n; k++) HIPCHK(c, hipStreamWaitEvent(c->grp_stream, replica_of(h, k)->grp_packed, 0));
      size_t p0, p1;
      shard_range(npx, n, c->replica, &p0, &p1);
      if (p1 > p0) {
        CompositeSrc S;
        memset(&S, 0, sizeof S);
        S.n = n;
        for (uint32_t k = 0; k < n; k++) S.p[k] = replica_of(h, k)->grp_pack[b] + p0;
        HIPCHK(c, launch_composite(S, (uint32_t)(p1 - p0), c->grp_rgb32, c->grp_rgba, c->grp_counts,
                                   c->grp_stream, true));
      }
      HIPCHK(c, hipEventRecord(c->grp_shard[b], c->grp_stream));
      return VPTMCM_OK;
    });
    if (rc) return rc;
  } else {
    if (ncclGroupStart() != ncclSuccess) FAIL(h, VPTMCM_ECOMM, "composite: ncclGroupStart failed");
    ncclResult_t r = ncclSuccess;
    for (uint32_t k = 0; k < n && r == ncclSuccess; k++) {
      vptmcm* c = replica_of(h, k);
      r = ncclReduce(c->grp_pack[0], k ? c->grp_pack[0] : h->grp_gather, npx * 4, ncclFloat32, ncclSum, 0,
                     h->grp_comms[k], enq(c));
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r != ncclSuccess || re != ncclSuccess)
      FAIL(h, VPTMCM_ECOMM, "composite: ncclReduce: %s", ncclGetErrorString(r != ncclSuccess ? r : re));
    HIPCHK(h, hipSetDevice(h->device));
    CompositeSrc S;
    memset(&S, 0, sizeof S);
    S.n = 1;
    S.p[0] = h->grp_gather;
    HIPCHK(h, launch_composite(S, (uint32_t)npx, h->grp_rgb32, h->grp_rgba, nullptr, enq(h)));
    HIPCHK(h, hipEventRecord(h->grp_done[b], enq(h)));
  }
  h->grp_seq++;
  h->grp_use_seq[b] = h->grp_seq;
  h->grp_last = (int)b;
  h->grp_dirty = false;
  if (VPT_GUARD) return for_replicas(h, [&](vptmcm* c) { return guard_check(c, "composite"); });
  return VPTMCM_OK;
}

// Before a read of the composite on replica 0's stream: make it if a march or
// reset ran since the last one, and order the stream behind it.
static int composite_ready(vptmcm* h) {
  if (h->grp_dirty || h->grp_last < 0)
    if (int rc = group_composite(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamWaitEvent(enq(h), h->grp_done[h->grp_last], 0));
  return VPTMCM_OK;
}

enum ShardPlane { kShardRgba, kShardRgb, kShardCounts };

// PEER readers: every replica's shard of the composite (made first if a march
// or reset ran since the last one) copied to its place in the host buffer, all
// replicas at once, each on its composite stream, behind its shard kernel.
static int read_shards(vptmcm* h, ShardPlane which, void* out) {
  if (h->grp_dirty || h->grp_last < 0)
    if (int rc = group_composite(h)) return rc;
  const size_t bpp = which == kShardRgba ? 8 : which == kShardRgb ? 12 : 4;
  const int rc = for_replicas(h, [&](vptmcm* c) {
    const size_t m = c->grp_p1 - c->grp_p0;
    if (m == 0) return VPTMCM_OK;
    const void* src = which == kShardRgba ? (const void*)c->grp_rgba
                      : which == kShardRgb ? (const void*)c->grp_rgb32 : (const void*)c->grp_counts;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(static_cast<char*>(out) + c->grp_p0 * bpp, src, m * bpp, hipMemcpyDeviceToHost,
                             c->grp_stream));
    HIPCHK(c, hipStreamSynchronize(c->grp_stream));
    return VPTMCM_OK;
  });
  if (rc == VPTMCM_OK) h->grp_synced_seq = h->grp_seq;  // the shards of the last composite are done
  return rc;
}

int vptmcm_create(const vptmcm_config* cfg, vptmcm** out) {
  g_create_error.clear();
  if (!cfg || !out) {
    g_create_error = "vptmcm_create: null argument";
    return VPTMCM_EINVAL;
  }
  *out = nullptr;
  if (cfg->resolution == 0 || cfg->resolution > 16384) {
    g_create_error = "vptmcm_create: resolution must be in [1, 16384]";
    return VPTMCM_EINVAL;
  }
  if (cfg->max_bins != VPTMCM_MAX_BINS) {
    g_create_error = "vptmcm_create: max_bins must be 12 (MAX_N_BINS)";
    return VPTMCM_EINVAL;
  }
  if (cfg->renderer > VPTMCM_RENDERER_RGB) {
    g_create_error = "vptmcm_create: unknown renderer kind";
    return VPTMCM_EINVAL;
  }
  if (cfg->volume_layout > VPTMCM_LAYOUT_COLUMN4) {
    g_create_error = "vptmcm_create: unknown volume layout";
    return VPTMCM_EINVAL;
  }
  if (cfg->n_devices > 0) return create_group(cfg, out);
  vptmcm* h = new vptmcm();
  auto fail = [&](int code) {
    g_create_error = h->err;
    vptmcm_destroy(h);
    return code;
  };
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    h->err = "vptmcm_create: no HIP device available";
    return fail(VPTMCM_EHIP);
  }
  if (cfg->device >= 0) {
    if (cfg->device >= ndev) {
      h->err = "vptmcm_create: device ordinal out of range";
      return fail(VPTMCM_EINVAL);
    }
    h->device = cfg->device;
    if (hipSetDevice(h->device) != hipSuccess) {
      h->err = "vptmcm_create: hipSetDevice failed";
      return fail(VPTMCM_EHIP);
    }
    // VPTMCM_SYNC_SPIN=1 (analysis): host waits on this device spin instead of
    // yielding (the flags of the calling thread's current device: set after it)
    if (const char* v = getenv("VPTMCM_SYNC_SPIN"))
      if (v[0] == '1') (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  } else {
    (void)hipGetDevice(&h->device);
  }
  if (const char* v = getenv("VPTMCM_TIME_STOP")) h->time_stop = v[0] != '0';
  if (const char* v = getenv("VPTMCM_TIME_BEGIN")) h->time_begin_marker = strcmp(v, "marker") == 0;
  if (const char* v = getenv("VPTMCM_SYNC_SPIN_US")) h->sync_spin_us = strtoll(v, nullptr, 10);
  h->layout = cfg->volume_layout;
  h->kind = cfg->renderer;
  if (const char* v = getenv("VPTMCM_MARCH_VARIANT")) h->variant = (uint32_t)strtoul(v, nullptr, 0);
  h->R = cfg->resolution;
  h->band_y0 = 0;
  h->band_y1 = h->R;
  h->tiles_x = (h->R + 7) / 8;
  h->n_tiles = h->tiles_x * h->tiles_x;
  h->npad = h->n_tiles * 64;
  memset(h->light_host, 0, sizeof h->light_host);
#define CK(expr)                                                     \
  do {                                                               \
    hipError_t _e = (expr);                                          \
    if (_e != hipSuccess) {                                          \
      h->err = std::string(#expr ": ") + hipGetErrorString(_e);      \
      return fail(VPTMCM_ENOMEM);                                    \
    }                                                                \
  } while (0)
  CK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  CK(dev_alloc(&h->photons, (size_t)kNumPlanes * h->npad * sizeof(float)));
  CK(hipMemsetAsync(h->photons, 0, (size_t)kNumPlanes * h->npad * sizeof(float), enq(h)));
  CK(dev_alloc(&h->rgba, (size_t)h->R * h->R * 4 * sizeof(uint16_t)));
  CK(hipMemsetAsync(h->rgba, 0, (size_t)h->R * h->R * 4 * sizeof(uint16_t), enq(h)));
  CK(dev_alloc(&h->rgb32, (size_t)h->R * h->R * 3 * sizeof(float)));
  CK(hipMemsetAsync(h->rgb32, 0, (size_t)h->R * h->R * 3 * sizeof(float), enq(h)));
  CK(dev_alloc(&h->tf_rg, 65536 * sizeof(uint16_t)));
  CK(hipMemsetAsync(h->tf_rg, 0, 65536 * sizeof(uint16_t), enq(h)));  // zero texture, js:85
  CK(dev_alloc(&h->tf_b4, kTfCells * kTfCells * sizeof(uint32_t)));
  CK(hipMemsetAsync(h->tf_b4, 0, kTfCells * kTfCells * sizeof(uint32_t), enq(h)));
  CK(dev_alloc(&h->tf_brow, 256));
  CK(hipMemsetAsync(h->tf_brow, 0, 256, enq(h)));
  CK(dev_alloc(&h->tf_rows, kTfRowsMax * 256 * sizeof(uint32_t)));
  CK(hipMemsetAsync(h->tf_rows, 0, kTfRowsMax * 256 * sizeof(uint32_t), enq(h)));
  CK(dev_alloc(&h->bin_lut, sizeof h->bin_lut_host));
  CK(hipMemsetAsync(h->bin_lut, 0, sizeof h->bin_lut_host, enq(h)));
  CK(dev_alloc(&h->tf_rowmax, 256));
  CK(hipMemsetAsync(h->tf_rowmax, 0, 256, enq(h)));  // the zero texture: alpha 0 in every row
  CK(dev_alloc(&h->tf_rowmap, 256));
  CK(hipMemsetAsync(h->tf_rowmap, 0, 256, enq(h)));
  CK(dev_alloc(&h->light, 256));
  CK(hipMemsetAsync(h->light, 0, 256, enq(h)));
  CK(dev_alloc(&h->tf_rgb, kRgbTfMax * sizeof(float4)));
  CK(dev_alloc(&h->sched, 2 * (size_t)sched_flag_bytes(h->n_tiles)));
  CK(hipMemsetAsync(h->sched, 0, 2 * (size_t)sched_flag_bytes(h->n_tiles), enq(h)));
  CK(dev_alloc(&h->sched_prev, sched_slot_words(h->n_tiles) * sizeof(uint32_t)));
  CK(hipMemsetAsync(h->sched_prev, 0xff, sched_slot_words(h->n_tiles) * sizeof(uint32_t), enq(h)));
  CK(dev_alloc(&h->sched_changed, 2 * sizeof(uint32_t)));
  CK(hipMemsetAsync(h->sched_changed, 0, 2 * sizeof(uint32_t), enq(h)));
  if (const char* v = getenv("VPTMCM_DARK")) h->dark = v[0] == '0' ? 0u : 1u;
  if (const char* v = getenv("VPTMCM_DONE_FLAG")) h->done_on = v[0] != '0';
  if (const char* v = getenv("VPTMCM_SCHED_CACHE")) h->sched_cache = v[0] != '0';
  if (const char* v = getenv("VPTMCM_MAJ"))
    h->maj_tune.mode = strcmp(v, "off") == 0 ? 0 : strcmp(v, "on") == 0 ? 1 : 2;
  maj_tune_reset(h);  // no size measured yet
  CK(dev_alloc(&h->done_ctr, sizeof(uint32_t)));
  CK(hipMemsetAsync(h->done_ctr, 0, sizeof(uint32_t), enq(h)));
  // the flag word in fine-grained host memory; without it, synchronize waits
  // for the stream (the signal is an optimisation, never a requirement)
  if (hipHostMalloc(&h->done_host, sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped) ==
          hipSuccess &&
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->done_dev), h->done_host, 0) == hipSuccess) {
    *h->done_host = 0u;
  } else {
    (void)hipGetLastError();
    h->done_on = false;
  }
  if (h->kind == VPTMCM_RENDERER_RGB) {  // WebGPUAbstractComputeRenderer.js:23-28
    static const uint8_t kDefaultTf[8] = {255, 0, 0, 0, 255, 0, 0, 255};
    if (vptmcm_set_transfer_function(h, kDefaultTf, 2, 1)) return fail(VPTMCM_EHIP);
  }
  CK(hipStreamSynchronize(h->stream));
#undef CK
  *out = h;
  return VPTMCM_OK;
}

void vptmcm_destroy(vptmcm* h) {
  if (!h) return;
  stop_workers(h);
  // Replicas first: their streams may feed this one's composite (they hold no
  // communicator, so their waits are plain stream waits).
  for (vptmcm* c : h->peers) {
    if (c->stream) (void)wait_stream(c, c->stream, "destroy");
    if (c->grp_stream) (void)wait_stream(c, c->grp_stream, "destroy");
  }
  // Bounded waits while a communicator exists or after its abort; streams that
  // did not drain may still touch the handle's buffers (a composite kernel and
  // its copies queued behind an RCCL call that never completed), which are
  // then left allocated (a deliberate leak) rather than freed under running
  // work: every device free below comes after this check.
  bool drained = true;
  if (h->comm_stream) drained = wait_stream(h, h->comm_stream, "destroy") == VPTMCM_OK && drained;
  if (h->stream) drained = wait_stream(h, h->stream, "destroy") == VPTMCM_OK && drained;
  if (h->grp_stream) drained = wait_stream(h, h->grp_stream, "destroy") == VPTMCM_OK && drained;
  for (ncclComm_t c : h->grp_comms)
    if (c) (void)ncclCommDestroy(c);
  h->grp_comms.clear();
  if (h->comm && comm_call(h, ncclCommFinalize(h->comm), "destroy: ncclCommFinalize") == VPTMCM_OK)
    (void)ncclCommDestroy(h->comm);
  for (vptmcm* c : h->peers) {
    if (drained) {  // a peer's pack may be read by this handle's (undrained) composite
      (void)hipSetDevice(c->device);
      for (auto& p : c->grp_pack) {
        if (p) (void)dev_free(p);
        p = nullptr;
      }
      if (c->grp_packed) (void)hipEventDestroy(c->grp_packed);
      for (auto& e : c->grp_shard) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
      }
      if (c->grp_stream) (void)hipStreamDestroy(c->grp_stream);
      c->grp_packed = nullptr;
      c->grp_stream = nullptr;
    }
    vptmcm_destroy(c);
  }
  h->peers.clear();
  if (!drained) {
    comm_trace("destroy: streams not drained; device buffers left allocated");
    delete h;
    return;
  }
  (void)hipSetDevice(h->device);
  for (auto p : h->grp_pack)
    if (p) (void)dev_free(p);
  if (h->grp_packed) (void)hipEventDestroy(h->grp_packed);
  for (auto e : h->grp_shard)
    if (e) (void)hipEventDestroy(e);
  if (h->grp_gather) (void)dev_free(h->grp_gather);
  if (h->grp_rgb32) (void)dev_free(h->grp_rgb32);
  if (h->grp_rgba) (void)dev_free(h->grp_rgba);
  if (h->grp_counts) (void)dev_free(h->grp_counts);
  if (h->grp_ldr) (void)dev_free(h->grp_ldr);
  for (auto e : h->grp_done)
    if (e) (void)hipEventDestroy(e);
  if (h->comp_rgb32) (void)dev_free(h->comp_rgb32);
  if (h->comp_rgba) (void)dev_free(h->comp_rgba);
  if (h->comp_counts) (void)dev_free(h->comp_counts);
  if (h->band_cover) (void)dev_free(h->band_cover);
  for (int k = 0; k < 2; k++) {
    if (h->comp[k]) (void)dev_free(h->comp[k]);
    if (h->comp_ready[k]) (void)hipEventDestroy(h->comp_ready[k]);
    if (h->comp_done[k]) (void)hipEventDestroy(h->comp_done[k]);
  }
  if (h->host_scratch) (void)dev_free(h->host_scratch);
  for (auto& pr : h->maj_tune.pairs)
    for (int k = 0; k < 2; k++) {
      if (pr.b[k]) (void)hipEventDestroy(pr.b[k]);
      if (pr.e[k]) (void)hipEventDestroy(pr.e[k]);
    }
  if (h->region.beg) (void)hipEventDestroy(h->region.beg);
  if (h->region.end) (void)hipEventDestroy(h->region.end);
  free_volume(h);
  if (h->photons) (void)dev_free(h->photons);
  if (h->rgba) (void)dev_free(h->rgba);
  if (h->rgb32) (void)dev_free(h->rgb32);
  if (h->ldr) (void)dev_free(h->ldr);
  if (h->tf_rgb) (void)dev_free(h->tf_rgb);
  if (h->tf_rg) (void)dev_free(h->tf_rg);
  if (h->tf_b4) (void)dev_free(h->tf_b4);
  if (h->tf_brow) (void)dev_free(h->tf_brow);
  if (h->tf_rows) (void)dev_free(h->tf_rows);
  if (h->tf_rowmap) (void)dev_free(h->tf_rowmap);
  if (h->tf_rowmax) (void)dev_free(h->tf_rowmax);
  if (h->bin_lut) (void)dev_free(h->bin_lut);
  if (h->light) (void)dev_free(h->light);
  if (h->sched) (void)dev_free(h->sched);
  if (h->sched_prev) (void)dev_free(h->sched_prev);
  if (h->sched_changed) (void)dev_free(h->sched_changed);
  if (h->done_ctr) (void)dev_free(h->done_ctr);
  if (h->done_host) (void)hipHostFree(h->done_host);
  if (h->comm_stream) (void)hipStreamDestroy(h->comm_stream);
  if (h->grp_stream) (void)hipStreamDestroy(h->grp_stream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

// ------------------------------------------------------------------- inputs

// Block-wise ingest. begin allocates the staging copy (x-fastest u8, zero like
// a fresh texture) and, for CORNER8 / BRICK8, the cell array (zero cells = a
// zero volume); every block is copied into the staging copy and the cells it
// touches join a box that is re-laid out in one launch before the next march
// reads the cells or at end (consecutive placements are batched: a
// slice-by-slice ingest relays each cell once, not twice), so the volume is
// renderable throughout (blocks not yet written read as zero density); end
// frees the staging copy.
static int volume_begin_one(vptmcm* h, uint32_t width, uint32_t height, uint32_t depth) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!width || !height || !depth || width > 8192 || height > 8192 || depth > 8192)
    FAIL(h, VPTMCM_EINVAL, "volume dimensions must be in [1, 8192]");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  free_volume(h);
  size_t n = (size_t)width * height * depth;
  if (dev_alloc(&h->vol_lin, n) != hipSuccess) {
    h->vol_lin = nullptr;
    FAIL(h, VPTMCM_ENOMEM, "volume allocation of %zu bytes failed", n);
  }
  // a fresh texture is zero; the block copies below run on the same stream, after it
  HIPCHK(h, hipMemsetAsync(h->vol_lin, 0, n, enq(h)));
  if (h->layout != kLayoutLinear) {
    // CORNER8: (W+1)(H+1)(D+1) cells in raster order; BRICK8: the same cells
    // in 4x4x4-cell bricks (the brick grid rounds each edge up to whole bricks)
    const bool brick = h->layout == kLayoutBrick8, col = h->layout == kLayoutColumn4;
    const size_t bw = (width + kBrickCells) / kBrickCells, bh = (height + kBrickCells) / kBrickCells,
                 bd = (depth + kBrickCells) / kBrickCells;
    // COLUMN4: (W+1)(H+1)(D+2) quads of 4 B = half as many 8-B units
    const size_t ncell = brick ? bw * bh * bd * 64
                         : col ? ((size_t)(width + 1) * (height + 1) * (depth + 2) + 1) / 2
                               : (size_t)(width + 1) * (height + 1) * (depth + 1);
    // (Round 3's VPTMCM_VOL_ALLOC=contig knob, hipExtMallocWithFlags(...,
    // hipDeviceMallocContiguous), bought nothing and is gone: in round 5 the
    // knob test found that once such an allocation had been freed, later
    // handles in the process rendered wrong bits)
    if (dev_alloc(&h->vol_c8, ncell * 8) != hipSuccess) {
      h->vol_c8 = nullptr;
      free_volume(h);
      FAIL(h, VPTMCM_ENOMEM, "%s volume allocation of %zu bytes failed",
           brick ? "brick8" : col ? "column4" : "corner8",
           ncell * 8);
    }
    HIPCHK(h, hipMemsetAsync(h->vol_c8, 0, ncell * 8, enq(h)));
  }
  h->W = width;
  h->H = height;
  h->D = depth;
  // the macro-cell table: the finest power-of-two macro (>= 8 texel cells)
  // whose codes fit the march's LDS table (re-laid-out layouts)
  if (h->layout != kLayoutLinear) {
    for (uint32_t sh = 3; sh < 14 && !h->maj_ok; sh++) {
      const uint64_t nx = ((uint64_t)width + (1u << sh)) >> sh, ny = ((uint64_t)height + (1u << sh)) >> sh,
                     nz = ((uint64_t)depth + (1u << sh)) >> sh;  // ceil((W + 1) / M)
      const uint64_t n = nx * ny * nz, bytes = ((n + 1) / 2 + 15) / 16 * 16;
      if (bytes > kMajBytes) continue;
      h->maj_shift = sh;
      h->maj_nx = (uint32_t)nx;
      h->maj_ny = (uint32_t)ny;
      h->maj_nz = (uint32_t)nz;
      h->maj_n = (uint32_t)n;
      h->maj_bytes = (uint32_t)bytes;
      h->maj_ok = true;
    }
    if (h->maj_ok) {
      // a fresh volume reads zero: every macro cell's range is [0, 0]
      if (dev_alloc(&h->maj_mm, (size_t)h->maj_n * sizeof(uint16_t)) != hipSuccess ||
          dev_alloc(&h->maj_q, h->maj_bytes) != hipSuccess) {
        free_volume(h);
        FAIL(h, VPTMCM_ENOMEM, "macro-cell table allocation failed");
      }
      HIPCHK(h, hipMemsetAsync(h->maj_mm, 0, (size_t)h->maj_n * sizeof(uint16_t), enq(h)));
      HIPCHK(h, hipMemsetAsync(h->maj_q, 0, h->maj_bytes, enq(h)));
      h->maj_valid = false;
    }
  }
  h->volume_ready = true;
  return VPTMCM_OK;
}

static int volume_write_block_one(vptmcm* h, const uint8_t* data, uint32_t x, uint32_t y, uint32_t z,
                              uint32_t bw, uint32_t bh, uint32_t bd) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!h->vol_lin || h->vol_done)
    FAIL(h, VPTMCM_ESTATE, "volume_write_block outside volume_begin .. volume_end");
  if (!data) FAIL(h, VPTMCM_EINVAL, "null block data");
  if ((uint64_t)x + bw > h->W || (uint64_t)y + bh > h->H || (uint64_t)z + bd > h->D)
    FAIL(h, VPTMCM_EINVAL, "block [%u,%u,%u]+[%u,%u,%u] exceeds volume %ux%ux%u", x, y, z, bw, bh,
         bd, h->W, h->H, h->D);
  if (!bw || !bh || !bd) return VPTMCM_OK;
  HIPCHK(h, hipSetDevice(h->device));
  // Every copy is ordered behind volume_begin's zero-fill (and the renders
  // queued before this call) on the handle's stream and completes before
  // returning (the caller keeps the block buffer).
  if (bw == h->W && bh == h->H && x == 0 && y == 0) {  // whole slices: one contiguous copy
    HIPCHK(h, hipMemcpyAsync(h->vol_lin + (size_t)z * h->W * h->H, data, (size_t)bw * bh * bd,
                             hipMemcpyHostToDevice, enq(h)));
  } else {
    hipMemcpy3DParms p;
    memset(&p, 0, sizeof p);
    p.srcPtr = make_hipPitchedPtr((void*)data, bw, bw, bh);
    p.dstPtr = make_hipPitchedPtr(h->vol_lin, h->W, h->W, h->H);
    p.dstPos = make_hipPos(x, y, z);
    p.extent = make_hipExtent(bw, bh, bd);
    p.kind = hipMemcpyHostToDevice;
    HIPCHK(h, hipMemcpy3DAsync(&p, enq(h)));
  }
  if (h->layout != kLayoutLinear) {
    // the cells whose 8 corners include a voxel of the block, x .. x + bw per
    // axis, join the box re-laid out before the next march (flush_relayout)
    const uint32_t c0[3] = {x, y, z}, c1[3] = {x + bw + 1u, y + bh + 1u, z + bd + 1u};
    for (int k = 0; k < 3; k++) {
      h->vol_c0[k] = h->vol_dirty ? std::min(h->vol_c0[k], c0[k]) : c0[k];
      h->vol_c1[k] = h->vol_dirty ? std::max(h->vol_c1[k], c1[k]) : c1[k];
    }
    h->vol_dirty = true;
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));  // the caller keeps the block buffer
  return VPTMCM_OK;
}

static int volume_end_one(vptmcm* h) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!h->vol_lin || h->vol_done) FAIL(h, VPTMCM_ESTATE, "volume_end without volume_begin");
  HIPCHK(h, hipSetDevice(h->device));
  if (int rc = flush_relayout(h)) return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->layout != kLayoutLinear) {  // every cell is current: the staging copy goes
    HIPCHK(h, dev_free(h->vol_lin));
    h->vol_lin = nullptr;
  } else {
    h->vol_done = true;  // LINEAR: the staging copy is the volume
  }
  return VPTMCM_OK;
}

int vptmcm_set_volume(vptmcm* h, const uint8_t* voxels, uint32_t width, uint32_t height,
                      uint32_t depth) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!voxels) FAIL(h, VPTMCM_EINVAL, "set_volume: null voxels");
  int rc = vptmcm_volume_begin(h, width, height, depth);
  if (rc) return rc;
  rc = vptmcm_volume_write_block(h, voxels, 0, 0, 0, width, height, depth);
  if (rc) return rc;
  return vptmcm_volume_end(h);
}

static int set_material_tf_one(vptmcm* h, const uint8_t* rgba) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!rgba) FAIL(h, VPTMCM_EINVAL, "set_material_tf: null data");
  HIPCHK(h, hipSetDevice(h->device));
  // Re-layout for the march: (albedo, alpha) u16 texels (LDS-staged) and the
  // 4-corner anisotropy cells; texel (row, col) = rgba[(row*256 + col)*4 + ch].
  std::vector<uint16_t> rg(65536);
  std::vector<uint32_t> b4((size_t)kTfCells * kTfCells);
  for (int t = 0; t < 65536; t++)
    rg[t] = (uint16_t)(rgba[t * 4 + 0] | (rgba[t * 4 + 1] << 8));
  auto bch = [&](int r, int c) { return (uint32_t)rgba[(r * 256 + c) * 4 + 2]; };
  for (int cr = 0; cr < (int)kTfCells; cr++)
    for (int cc = 0; cc < (int)kTfCells; cc++) {
      int r0 = cr - 1 < 0 ? 0 : cr - 1, r1 = cr > 255 ? 255 : cr;
      int c0 = cc - 1 < 0 ? 0 : cc - 1, c1 = cc > 255 ? 255 : cc;
      b4[(size_t)cr * kTfCells + cc] =
          bch(r0, c0) | (bch(r0, c1) << 8) | (bch(r1, c0) << 16) | (bch(r1, c1) << 24);
    }
  HIPCHK(h, hipMemcpyAsync(h->tf_rg, rg.data(), rg.size() * 2, hipMemcpyHostToDevice, enq(h)));
  HIPCHK(h, hipMemcpyAsync(h->tf_b4, b4.data(), b4.size() * 4, hipMemcpyHostToDevice, enq(h)));
  // column-invariant anisotropy (the UI's per-material constant case): exact row table
  uint8_t brow[256];
  uint32_t inv = 1;
  for (int r = 0; r < 256; r++) {
    brow[r] = (uint8_t)bch(r, 0);
    for (int c = 1; c < 256 && inv; c++)
      if (bch(r, c) != brow[r]) inv = 0;
  }
  HIPCHK(h, hipMemcpyAsync(h->tf_brow, brow, 256, hipMemcpyHostToDevice, enq(h)));
  h->b_rows = inv;
  // the largest alpha byte of each density row (the macro-cell alpha codes)
  uint8_t rowmax[256];
  for (int r = 0; r < 256; r++) {
    uint8_t m = 0;
    for (int c = 0; c < 256; c++) m = std::max(m, rgba[(r * 256 + c) * 4 + 1]);
    rowmax[r] = m;
  }
  HIPCHK(h, hipMemcpyAsync(h->tf_rowmax, rowmax, 256, hipMemcpyHostToDevice, enq(h)));
  h->maj_valid = false;
  maj_tune_reset(h);
  // Distinct density rows over (albedo, alpha, anisotropy): a UI TF paints one
  // material's wavelength arrays into every row of a density range
  // (MaterialTransferFunction.js:56-75), so it has few; with <= kTfRowsMax of
  // them the non-FAST marches keep all three channels in LDS (P.tf_dedup).
  std::vector<uint32_t> rows;
  uint8_t rowmap[256];
  uint32_t n_rows = 0;
  for (int r = 0; r < 256 && n_rows <= kTfRowsMax; r++) {
    uint32_t texel[256];
    for (int c = 0; c < 256; c++) {
      const uint8_t* t = rgba + (r * 256 + c) * 4;
      texel[c] = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16);
    }
    uint32_t k = 0;
    while (k < n_rows && memcmp(&rows[(size_t)k * 256], texel, sizeof texel) != 0) k++;
    if (k == n_rows) {
      if (n_rows == kTfRowsMax) {
        n_rows++;  // too many: no deduplicated table
        break;
      }
      rows.insert(rows.end(), texel, texel + 256);
      n_rows++;
    }
    rowmap[r] = (uint8_t)k;
  }
  h->tf_dedup = n_rows <= kTfRowsMax ? 1u : 0u;
  if (h->tf_dedup) {
    HIPCHK(h, hipMemcpyAsync(h->tf_rows, rows.data(), rows.size() * sizeof(uint32_t),
                             hipMemcpyHostToDevice, enq(h)));
    HIPCHK(h, hipMemcpyAsync(h->tf_rowmap, rowmap, 256, hipMemcpyHostToDevice, enq(h)));
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));  // the host copies are freed on return
  return VPTMCM_OK;
}

static int set_light_one(vptmcm* h, const uint8_t* spd, const float dir[3]) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!spd || !dir) FAIL(h, VPTMCM_EINVAL, "set_light: null argument");
  HIPCHK(h, hipSetDevice(h->device));
  memcpy(h->light_host, spd, 256);
  memcpy(h->light_dir, dir, sizeof h->light_dir);
  HIPCHK(h, hipMemcpyAsync(h->light, h->light_host, 256, hipMemcpyHostToDevice, enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return VPTMCM_OK;
}

static int set_spectrum_one(vptmcm* h, const float* buf) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!buf) FAIL(h, VPTMCM_EINVAL, "set_spectrum: null buffer");
  float nbf = buf[0] + 0.5f;
  if (!(nbf >= 0.0f) || nbf >= (float)(VPTMCM_MAX_BINS + 1))
    FAIL(h, VPTMCM_EINVAL, "set_spectrum: n_bins = %g exceeds MAX_N_BINS (12)", (double)buf[0]);
  h->bin_lut_ok = false;  // every error path below leaves the bin table disabled
  memcpy(h->spectrum, buf, sizeof h->spectrum);
  maj_tune_reset(h);
  return build_bin_lut(h);
}

static int set_transfer_function_one(vptmcm* h, const uint8_t* rgba, uint32_t width, uint32_t height) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (h->kind != VPTMCM_RENDERER_RGB)
    FAIL(h, VPTMCM_ESTATE, "set_transfer_function: the spectral renderer uses set_material_tf");
  if (!rgba || width == 0 || height == 0 || width > kRgbTfMax)
    FAIL(h, VPTMCM_EINVAL, "set_transfer_function: need 1 <= width <= %u, height >= 1", kRgbTfMax);
  HIPCHK(h, hipSetDevice(h->device));
  // the kernel samples at (density, 0): row 0 only (see MarchParams::tf_w); the
  // rgba8unorm-srgb texel is decoded before filtering, alpha is linear
  std::vector<float4> row(width);
  for (uint32_t i = 0; i < width; i++) {
    const uint8_t* t = rgba + 4 * (size_t)i;
    row[i] = make_float4(srgb_to_linear(t[0]), srgb_to_linear(t[1]), srgb_to_linear(t[2]),
                         (float)t[3] * kInv255);
  }
  HIPCHK(h, hipMemcpyAsync(h->tf_rgb, row.data(), width * sizeof(float4), hipMemcpyHostToDevice,
                           enq(h)));
  // the macro-cell alpha codes' row maxima: per density byte v the largest
  // alpha byte of the texels a density within one byte of v reaches (texel
  // floor(d * width - 0.5) and the next, clamped), one texel of margin more
  // each way; k_macro_alpha widens that to v - 2 .. v + 2
  uint8_t rowmax[256];
  for (int v = 0; v < 256; v++) {
    const double w = (double)width;
    const long lo = std::max(0L, (long)std::floor((v - 1) / 255.0 * w - 0.5) - 1);
    const long hi = std::min((long)width - 1, (long)std::floor((v + 1) / 255.0 * w - 0.5) + 2);
    uint8_t m = 0;
    for (long t = lo; t <= hi; t++) m = std::max(m, rgba[4 * (size_t)t + 3]);
    rowmax[v] = m;
  }
  HIPCHK(h, hipMemcpyAsync(h->tf_rowmax, rowmax, 256, hipMemcpyHostToDevice, enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->tf_rgb_w = width;
  h->maj_valid = false;
  maj_tune_reset(h);
  return VPTMCM_OK;
}

static int set_environment_one(vptmcm* h, const uint8_t* rgba, uint32_t width, uint32_t height) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!rgba || width != 1 || height != 1)
    FAIL(h, VPTMCM_EINVAL, "set_environment: only the 1x1 environment of the rendering context "
                           "(WebGPURenderingContext.js:97-108) is supported");
  for (int k = 0; k < 4; k++) h->env[k] = (float)rgba[k] * kInv255;
  return VPTMCM_OK;
}

static int set_band_one(vptmcm* h, uint32_t y0, uint32_t y1) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!(y0 < y1 && y1 <= h->R && y0 % 8u == 0u && (y1 % 8u == 0u || y1 == h->R)))
    FAIL(h, VPTMCM_EINVAL, "set_band: need y0 < y1 <= R, y0 and y1 multiples of 8 (y1 may be R)");
  HIPCHK(h, hipSetDevice(h->device));
  h->band_y0 = y0;
  h->band_y1 = y1;
  stream_op(h);
  const size_t row = (size_t)h->R * 3 * sizeof(float);
  if (y0 > 0) HIPCHK(h, hipMemsetAsync(h->rgb32, 0, y0 * row, enq(h)));
  if (y1 < h->R)
    HIPCHK(h, hipMemsetAsync((char*)h->rgb32 + y1 * row, 0, (h->R - y1) * row, enq(h)));
  h->grp_dirty = true;
  return VPTMCM_OK;
}

static int set_params_one(vptmcm* h, const vptmcm_params* p) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (!p) FAIL(h, VPTMCM_EINVAL, "set_params: null params");
  // The reference rewrites the same uniform values before every pass
  // (js:295-309); only a change of bits ends the queue of fused passes.
  static_assert(sizeof(vptmcm_params) == 20, "vptmcm_params has no padding");
  if (memcmp(&h->params, p, sizeof *p) == 0) return VPTMCM_OK;
  if (int rc_ = flush_renders(h)) return rc_;
  h->params = *p;
  maj_tune_reset(h);
  return VPTMCM_OK;
}

// ------------------------------------------------------------------ hot path

static int reset_one(vptmcm* h, const float* mvp, uint32_t seed_bits) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!mvp) FAIL(h, VPTMCM_EINVAL, "reset: null matrix");
  HIPCHK(h, hipSetDevice(h->device));
  MarchParams P = make_params(h, mvp, seed_bits);
  stream_op(h);
  if (h->kind == VPTMCM_RENDERER_RGB)
    HIPCHK(h, launch_reset_rgb(P, h->photons, enq(h)));
  else
    HIPCHK(h, launch_reset(P, h->photons, enq(h)));
  h->grp_dirty = true;
  return guard_check(h, "reset");
}

static int render_one(vptmcm* h, const float* mvp, uint32_t seed_bits) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (!mvp) FAIL(h, VPTMCM_EINVAL, "render: null matrix");
  if (!h->volume_ready) FAIL(h, VPTMCM_ESTATE, "render: no volume set (setVolume first)");
  // queue the pass; a different matrix or a full queue launches the queue
  // first (the launch order, and so every result, is unchanged)
  if (h->pend_n == kMaxFusedPasses || (h->pend_n && memcmp(h->pend_mvp, mvp, sizeof h->pend_mvp))) {
    if (int rc = flush_renders(h)) return rc;
  }
  if (h->pend_n == 0) memcpy(h->pend_mvp, mvp, sizeof h->pend_mvp);
  h->pend_seeds[h->pend_n++] = seed_bits;
  return VPTMCM_OK;
}

static int render_passes_one(vptmcm* h, const float* mvp, const uint32_t* seeds, uint32_t n) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!mvp || (!seeds && n)) FAIL(h, VPTMCM_EINVAL, "render_passes: null argument");
  HIPCHK(h, hipSetDevice(h->device));
  const uint32_t fuse = (h->variant & 4u) ? 1u : kMaxFusedPasses;  // variant bit 2: one pass per launch
  for (uint32_t k = 0; k < n; k += fuse) {
    if (int rc = do_march(h, mvp, seeds + k, n - k < fuse ? n - k : fuse)) return rc;
  }
  return VPTMCM_OK;
}

static int synchronize_one(vptmcm* h) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  HIPCHK(h, hipSetDevice(h->device));
  int rc = time_close(h);
  if (rc) return rc;
  // The stream ends with a signalling march: poll its flag word (every wave's
  // stores have landed once it holds the launch's sequence number); past the
  // spin bound, or without a signal, wait for the stream itself.
  bool done = false;
  if (h->done_pending && h->sync_spin_us > 0) {
    const volatile uint32_t* f = h->done_host;
    const int64_t t0 = now_us();
    for (uint32_t k = 0;; k++) {
      if (*f == h->done_seq) {
        std::atomic_thread_fence(std::memory_order_acquire);  // the march's stores before the flag
        done = true;
        break;
      }
      if ((k & 63u) == 0u && now_us() - t0 > h->sync_spin_us) break;
    }
  }
  if (!done && (rc = wait_stream(h, h->stream, "synchronize"))) return rc;
  if (h->comm_stream && (rc = wait_stream(h, h->comm_stream, "synchronize"))) return rc;
  if (h->grp_stream && (rc = wait_stream(h, h->grp_stream, "synchronize"))) return rc;
  // the macro-skip tuner's finished pairs, read here while no region is timed
  // (a timed region's launches never query events)
  if (!h->timing && h->maj_tune.count > 0) maj_tune_harvest(h);
  return guard_check(h, "synchronize");
}

// ------------------------------------------------------------------ outputs

int vptmcm_read_rgba16f(vptmcm* h, uint16_t* out) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!out) FAIL(h, VPTMCM_EINVAL, "read_rgba16f: null output");
  if (sharded(h)) return read_shards(h, kShardRgba, out);
  if (composited(h))
    if (int rc = composite_ready(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipMemcpyAsync(out, composited(h) ? h->grp_rgba : h->rgba, (size_t)h->R * h->R * 8,
                           hipMemcpyDeviceToHost, enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return VPTMCM_OK;
}

int vptmcm_read_rgb(vptmcm* h, float* out) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!out) FAIL(h, VPTMCM_EINVAL, "read_rgb: null output");
  if (sharded(h)) return read_shards(h, kShardRgb, out);
  if (composited(h))
    if (int rc = composite_ready(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipMemcpyAsync(out, composited(h) ? h->grp_rgb32 : h->rgb32,
                           (size_t)h->R * h->R * 3 * sizeof(float), hipMemcpyDeviceToHost, enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return VPTMCM_OK;
}

int vptmcm_pack_radiance(vptmcm* h, float* out) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!out) FAIL(h, VPTMCM_EINVAL, "pack_radiance: null output");
  HIPCHK(h, hipSetDevice(h->device));
  const size_t bytes = (size_t)h->R * h->R * sizeof(float4);
  float4* d = nullptr;
  HIPCHK(h, dev_alloc(&d, bytes));
  MarchParams P = make_params(h, kNoMatrix, 0);
  hipError_t e = launch_pack(P, h->photons, h->rgb32, d, enq(h));
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, enq(h));
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)dev_free(d);
  if (e != hipSuccess) FAIL(h, VPTMCM_EHIP, "pack_radiance: %s", hipGetErrorString(e));
  return VPTMCM_OK;
}

int vptmcm_tonemap_artistic(vptmcm* h, const float params[5], uint8_t* rgba8_out) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!params) FAIL(h, VPTMCM_EINVAL, "tonemap_artistic: null params");
  if (composited(h))
    if (int rc = composite_ready(h)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  const size_t npx = (size_t)h->R * h->R;
  if (!h->ldr) HIPCHK(h, dev_alloc(&h->ldr, npx * 4));
  // uniform-only terms in f32, as the shader evaluates them once per fragment
  const float low = params[0], mid = params[1], high = params[2];
  const float range = high - low;
  ToneParams T;
  T.low = low;
  T.inv_range = 1.0f / range;
  T.saturation = params[3];
  const float midpoint = (mid - low) / range;
  T.exponent = (float)(-std::log((double)midpoint) / std::log(2.0)) / params[4];
  if (sharded(h)) {  // every shard tone-mapped on its own device, copied to its place
    if (h->grp_dirty || h->grp_last < 0)
      if (int rc = group_composite(h)) return rc;
    return for_replicas(h, [&](vptmcm* c) {
      const size_t m = c->grp_p1 - c->grp_p0;
      if (m == 0) return VPTMCM_OK;
      HIPCHK(c, hipSetDevice(c->device));
      if (!c->grp_ldr) HIPCHK(c, dev_alloc(&c->grp_ldr, m * 4));
      HIPCHK(c, launch_tonemap_artistic(c->grp_rgba, (uint32_t)m, T, c->grp_ldr, c->grp_stream));
      if (rgba8_out) {
        HIPCHK(c, hipMemcpyAsync(rgba8_out + c->grp_p0 * 4, c->grp_ldr, m * 4, hipMemcpyDeviceToHost,
                                 c->grp_stream));
        HIPCHK(c, hipStreamSynchronize(c->grp_stream));
      }
      return VPTMCM_OK;
    });
  }
  stream_op(h);
  HIPCHK(h, launch_tonemap_artistic(composited(h) ? h->grp_rgba : h->rgba, (uint32_t)npx, T, h->ldr,
                                    enq(h)));
  if (rgba8_out) {
    HIPCHK(h, hipMemcpyAsync(rgba8_out, h->ldr, npx * 4, hipMemcpyDeviceToHost, enq(h)));
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  return VPTMCM_OK;
}

int vptmcm_read_photons(vptmcm* h, void* out) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!out) FAIL(h, VPTMCM_EINVAL, "read_photons: null output");
  HIPCHK(h, hipSetDevice(h->device));
  std::vector<uint32_t> planes((size_t)kNumPlanes * h->npad);
  HIPCHK(h, hipMemcpyAsync(planes.data(), h->photons, planes.size() * 4, hipMemcpyDeviceToHost,
                           enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint32_t* o = static_cast<uint32_t*>(out);
  if (h->kind == VPTMCM_RENDERER_RGB) {  // struct Photon, Photon.wgsl: 64-B stride
    for (uint32_t y = 0; y < h->R; y++)
      for (uint32_t x = 0; x < h->R; x++) {
        size_t i = (size_t)((y / 8) * h->tiles_x + x / 8) * 64 + (y % 8) * 8 + (x % 8);
        uint32_t* w = o + ((size_t)y * h->R + x) * (VPTMCM_PHOTON_RGB_BYTES / 4);
        for (int k = 0; k < 3; k++) w[k] = planes[(kPx + k) * (size_t)h->npad + i];
        w[3] = planes[kBounces * (size_t)h->npad + i];
        for (int k = 0; k < 3; k++) w[4 + k] = planes[(kDx + k) * (size_t)h->npad + i];
        w[7] = planes[kSamples * (size_t)h->npad + i];
        for (int k = 0; k < 3; k++) w[8 + k] = planes[(kTr0 + k) * (size_t)h->npad + i];
        w[11] = 0u;
        for (int k = 0; k < 3; k++) w[12 + k] = planes[(kRgbRad0 + k) * (size_t)h->npad + i];
        w[15] = 0u;
      }
    return VPTMCM_OK;
  }
  const uint32_t one = 0x3f800000u;
  for (uint32_t y = 0; y < h->R; y++)
    for (uint32_t x = 0; x < h->R; x++) {
      size_t i = (size_t)((y / 8) * h->tiles_x + x / 8) * 64 + (y % 8) * 8 + (x % 8);
      uint32_t* w = o + ((size_t)y * h->R + x) * (VPTMCM_PHOTON_BYTES / 4);
      for (int k = 0; k < 3; k++) w[k] = planes[(kPx + k) * (size_t)h->npad + i];
      w[3] = planes[kBounces * (size_t)h->npad + i];
      for (int k = 0; k < 3; k++) w[4 + k] = planes[(kDx + k) * (size_t)h->npad + i];
      w[7] = planes[kSamples * (size_t)h->npad + i];
      w[8] = planes[kBin * (size_t)h->npad + i];
      w[9] = planes[kLambda * (size_t)h->npad + i];
      for (int b = 0; b < kMaxBins; b++) w[10 + b] = planes[(kRad0 + b) * (size_t)h->npad + i];
      for (int b = 0; b < kMaxBins; b++) w[22 + b] = one;
      w[34] = w[35] = 0u;  // struct padding to the 144-B stride
    }
  return VPTMCM_OK;
}

int vptmcm_write_photons(vptmcm* h, const void* in) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!in) FAIL(h, VPTMCM_EINVAL, "write_photons: null input");
  HIPCHK(h, hipSetDevice(h->device));
  std::vector<uint32_t> planes((size_t)kNumPlanes * h->npad, 0u);
  const uint32_t* src = static_cast<const uint32_t*>(in);
  if (h->kind == VPTMCM_RENDERER_RGB) {
    for (uint32_t y = 0; y < h->R; y++)
      for (uint32_t x = 0; x < h->R; x++) {
        size_t i = (size_t)((y / 8) * h->tiles_x + x / 8) * 64 + (y % 8) * 8 + (x % 8);
        const uint32_t* w = src + ((size_t)y * h->R + x) * (VPTMCM_PHOTON_RGB_BYTES / 4);
        for (int k = 0; k < 3; k++) planes[(kPx + k) * (size_t)h->npad + i] = w[k];
        planes[kBounces * (size_t)h->npad + i] = w[3];
        for (int k = 0; k < 3; k++) planes[(kDx + k) * (size_t)h->npad + i] = w[4 + k];
        planes[kSamples * (size_t)h->npad + i] = w[7];
        for (int k = 0; k < 3; k++) planes[(kTr0 + k) * (size_t)h->npad + i] = w[8 + k];
        for (int k = 0; k < 3; k++) planes[(kRgbRad0 + k) * (size_t)h->npad + i] = w[12 + k];
      }
  }
  for (uint32_t y = 0; h->kind == VPTMCM_RENDERER_SPECTRAL && y < h->R; y++)
    for (uint32_t x = 0; x < h->R; x++) {
      size_t i = (size_t)((y / 8) * h->tiles_x + x / 8) * 64 + (y % 8) * 8 + (x % 8);
      const uint32_t* w = src + ((size_t)y * h->R + x) * (VPTMCM_PHOTON_BYTES / 4);
      for (int k = 0; k < 3; k++) planes[(kPx + k) * (size_t)h->npad + i] = w[k];
      planes[kBounces * (size_t)h->npad + i] = w[3];
      for (int k = 0; k < 3; k++) planes[(kDx + k) * (size_t)h->npad + i] = w[4 + k];
      planes[kSamples * (size_t)h->npad + i] = w[7];
      planes[kBin * (size_t)h->npad + i] = w[8];
      planes[kLambda * (size_t)h->npad + i] = w[9];
      for (int b = 0; b < kMaxBins; b++) planes[(kRad0 + b) * (size_t)h->npad + i] = w[10 + b];
    }
  HIPCHK(h, hipMemcpyAsync(h->photons, planes.data(), planes.size() * 4, hipMemcpyHostToDevice,
                           enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->grp_dirty = true;
  return VPTMCM_OK;
}

// --------------------------------------------------------------- measurement

static int enable_kernel_timing_one(vptmcm* h, int enable) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->timing = enable != 0;
  if (h->timing && !h->region.beg) {  // created and first recorded here, outside the region they time
    HIPCHK(h, hipEventCreateWithFlags(&h->region.beg, hipEventDisableSystemFence));
    HIPCHK(h, hipEventCreateWithFlags(&h->region.end, hipEventDisableSystemFence));
    HIPCHK(h, hipEventRecord(h->region.beg, enq(h)));
    HIPCHK(h, hipEventRecord(h->region.end, enq(h)));
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  h->launches = 0;
  h->region_closed = false;
  return VPTMCM_OK;
}

static int kernel_time_one(vptmcm* h, double* total_ms, uint64_t* launches) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!total_ms || !launches) FAIL(h, VPTMCM_EINVAL, "kernel_time: null output");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = time_close(h);
  if (rc) return rc;
  if ((rc = wait_stream(h, h->stream, "kernel_time"))) return rc;
  float ms = 0.0f;
  if (h->timing && h->launches) HIPCHK(h, hipEventElapsedTime(&ms, h->region.beg, h->region.end));
  *total_ms = ms;
  *launches = h->timing ? h->launches : 0;
  return VPTMCM_OK;
}

// A device-list handle times replica 0 only (vptmcm_enable_kernel_timing):
// every replica runs the same launches, and each timed launch carries event
// stamps that add ≈ 2–4 µs to its enqueue, i.e. to the skew between the first
// and the last replica's start when one host thread forwards the launch.
int vptmcm_kernel_time(vptmcm* h, double* total_ms, uint64_t* launches) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  // their queued passes launch, as for any observation
  if (int rc = for_peers(h, [](vptmcm* c) { return flush_renders(c); })) return rc;
  return kernel_time_one(h, total_ms, launches);
}

// ------------------------------------------------------------------ multi-GPU

int vptmcm_comm_unique_id(uint8_t* out) {
  if (!out) return VPTMCM_EINVAL;
  ncclUniqueId id;
  comm_trace("unique_id: ncclGetUniqueId");
  const ncclResult_t r = ncclGetUniqueId(&id);
  comm_trace("unique_id: returned %d", (int)r);
  if (r != ncclSuccess) {
    g_create_error = "ncclGetUniqueId failed";
    return VPTMCM_ECOMM;
  }
  static_assert(sizeof(id) == VPTMCM_UNIQUE_ID_BYTES, "ncclUniqueId size");
  memcpy(out, &id, sizeof id);
  return VPTMCM_OK;
}

int vptmcm_comm_init(vptmcm* h, const uint8_t* uid, int nranks, int rank) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!uid || nranks < 1 || rank < 0 || rank >= nranks)
    FAIL(h, VPTMCM_EINVAL, "comm_init: bad arguments (nranks=%d rank=%d)", nranks, rank);
  if (h->comm) FAIL(h, VPTMCM_ESTATE, "comm_init: communicator already initialised");
  if (h->grouped && (composited(h) || !h->grp_comms.empty()))
    FAIL(h, VPTMCM_ESTATE, "comm_init: a device-list handle composites its replicas itself");
  HIPCHK(h, hipSetDevice(h->device));
  if (const char* v = getenv("VPTMCM_COMM_TIMEOUT_MS")) {
    const long long t = strtoll(v, nullptr, 10);
    if (t > 0) h->comm_timeout_ms = t;
  }
  ncclUniqueId id;
  memcpy(&id, uid, sizeof id);
  // RCCL 2.27.7 does not return from ncclCommInitRankConfig while its bootstrap
  // waits for a rank that never arrives, with blocking = 0 too: the calling
  // thread sleep-polls inside the call while the init job spins on the
  // bootstrap sockets and the root thread waits in accept()
  // (tools/comm_diag.cpp, profiles/r04/s1/comm_diag_nb.log), and no
  // communicator handle exists to abort until the call returns (aborting one
  // still in bootstrap hung in round 3). Peer liveness is therefore
  // established before this call (rendezvous.join: every rank present,
  // bounded by VPTMCM_COMM_TIMEOUT_MS, ECOMM otherwise). The residual window —
  // a peer that joined and then died before its init — is bounded here: the
  // initialisation runs on a helper thread and the caller waits for it at most
  // VPTMCM_COMM_TIMEOUT_MS. On success the thread is joined. On expiry the
  // call returns ECOMM and the thread, blocked inside RCCL, cannot be
  // reclaimed: it is detached (should the initialisation ever return, it
  // aborts the unused communicator) and the caller must end the process
  // without running exit handlers (_exit), as bench.py does.
  struct InitJob {
    std::atomic<int> state{0};  // 0 running, 1 returned, 2 abandoned by the caller
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclSuccess;
  };
  auto job = std::make_shared<InitJob>();
  comm_trace("comm_init: ncclCommInitRank nranks=%d rank=%d (helper thread)", nranks, rank);
  const int dev = h->device;
  std::thread th;
  try {
    th = std::thread([job, id, nranks, rank, dev]() {
      ncclComm_t c = nullptr;
      (void)hipSetDevice(dev);
      const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
      job->comm = c;
      job->r = r;
      int running = 0;
      if (!job->state.compare_exchange_strong(running, 1) && c) (void)ncclCommAbort(c);  // abandoned
    });
  } catch (const std::exception& e) {
    FAIL(h, VPTMCM_ECOMM, "comm_init: cannot start the initialisation thread: %s", e.what());
  }
  const int64_t t0 = now_ms();
  while (job->state.load() == 0 && now_ms() - t0 <= h->comm_timeout_ms)
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  int running = 0;
  if (job->state.compare_exchange_strong(running, 2)) {  // still inside RCCL: give it up
    th.detach();
    comm_trace("comm_init: no return after %lld ms; helper thread detached", (long long)h->comm_timeout_ms);
    FAIL(h, VPTMCM_ECOMM,
         "ncclCommInitRank (rank %d of %d) did not return within %lld ms (a peer died after the "
         "rendezvous?); its thread is blocked inside RCCL and cannot be reclaimed: end the process "
         "(_exit)", rank, nranks, (long long)h->comm_timeout_ms);
  }
  th.join();
  const ncclResult_t r = job->r;
  ncclComm_t c = job->comm;
  comm_trace("comm_init: ncclCommInitRank returned %d", (int)r);
  if (r != ncclSuccess) {
    if (c) (void)ncclCommAbort(c);
    FAIL(h, VPTMCM_ECOMM, "ncclCommInitRank (rank %d of %d): %s", rank, nranks, ncclGetErrorString(r));
  }
  h->comm = c;
  h->comm_failed = false;
  h->nranks = nranks;
  h->rank = rank;

  HIPCHK(h, hipStreamCreateWithFlags(&h->comm_stream, hipStreamNonBlocking));
  size_t bytes = (size_t)h->R * h->R * sizeof(float4);
  for (int k = 0; k < 2; k++) {
    HIPCHK(h, dev_alloc(&h->comp[k], bytes));
    HIPCHK(h, hipEventCreateWithFlags(&h->comp_ready[k], hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&h->comp_done[k], hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(h->comp_done[k], h->comm_stream));
  }
  HIPCHK(h, dev_alloc(&h->host_scratch, 64 * sizeof(double)));
  return VPTMCM_OK;
}

int vptmcm_comm_allreduce_radiance(vptmcm* h) { return vptmcm_comm_allreduce_radiance_ex(h, 0u); }

int vptmcm_comm_allreduce_radiance_ex(vptmcm* h, uint32_t flags) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!h->comm) FAIL(h, VPTMCM_ECOMM, "comm_allreduce_radiance: no communicator");
  if (flags & ~(uint32_t)(VPTMCM_ALLREDUCE_INLINE | VPTMCM_ALLREDUCE_SHARDED))
    FAIL(h, VPTMCM_EINVAL, "comm_allreduce_radiance: unknown flags");
  HIPCHK(h, hipSetDevice(h->device));
  int k = h->comp_next;
  const size_t words = (size_t)h->R * h->R * 4;  // R*R float4
  // reduce-scatter: equal shards of whole pixels, rank r's in place at r * shard
  const bool shard = (flags & VPTMCM_ALLREDUCE_SHARDED) && h->nranks > 0 &&
                     ((size_t)h->R * h->R) % (size_t)h->nranks == 0;
  const size_t shard_words = shard ? words / (size_t)h->nranks : words;
  float* base = reinterpret_cast<float*>(h->comp[k]);
  auto collective = [&](hipStream_t st) {
    return shard ? ncclReduceScatter(base, base + (size_t)h->rank * shard_words, shard_words, ncclFloat32,
                                     ncclSum, h->comm, st)
                 : ncclAllReduce(base, base, words, ncclFloat32, ncclSum, h->comm, st);
  };
  if (!h->pack_fresh) {  // the stream does not end with a march that packed comp[k]
    stream_op(h);
    // the buffer must be free of the all-reduce issued two passes ago
    HIPCHK(h, hipStreamWaitEvent(enq(h), h->comp_done[k], 0));
    MarchParams P = make_params(h, kNoMatrix, 0);
    HIPCHK(h, launch_pack(P, h->photons, h->rgb32, h->comp[k], enq(h)));
  }
  if (flags & VPTMCM_ALLREDUCE_INLINE) {
    // On the march stream itself, right behind the pack: no event hop to the
    // side stream (the composite about to be shown is ready soonest); the
    // next march waits for it. Ordered after the side stream's last
    // all-reduce, so the communicator's collectives stay in issue order.
    HIPCHK(h, hipStreamWaitEvent(enq(h), h->comp_done[k ^ 1], 0));
    if (int rc = comm_call(h, collective(enq(h)), "comm_allreduce_radiance")) return rc;
    HIPCHK(h, hipEventRecord(h->comp_done[k], enq(h)));
  } else {
    stream_op(h);
    HIPCHK(h, hipEventRecord(h->comp_ready[k], enq(h)));
    HIPCHK(h, hipStreamWaitEvent(h->comm_stream, h->comp_ready[k], 0));
    if (int rc = comm_call(h, collective(h->comm_stream), "comm_allreduce_radiance")) return rc;
    HIPCHK(h, hipEventRecord(h->comp_done[k], h->comm_stream));
  }
  h->comp_sharded[k] = shard;
  h->comp_last = k;
  h->comp_next = k ^ 1;
  return VPTMCM_OK;
}

int vptmcm_comm_read_composite(vptmcm* h, float* rgb, float* counts) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (!rgb) FAIL(h, VPTMCM_EINVAL, "read_composite: null output");
  if (!h->comm || h->comp_last < 0) FAIL(h, VPTMCM_ESTATE, "read_composite: no all-reduce issued");
  return vptmcm_read_composite(h, nullptr, rgb, counts);
}

int vptmcm_read_composite(vptmcm* h, uint16_t* rgba16f, float* rgb, float* counts) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  const size_t npx = (size_t)h->R * h->R;
  if (h->grouped) {  // a device-list handle: over its replicas (N = 1 included)
    if (!h->grp_rgb32) {  // one replica, PEER: the buffers of the composite on first use
      const int32_t dev = h->device;
      if (int rc = group_alloc(h, &dev, 1)) return rc;
    }
    if (h->group_transport == VPTMCM_GROUP_PEER) {  // the shards, every one to its place
      if (rgba16f)
        if (int rc = read_shards(h, kShardRgba, rgba16f)) return rc;
      if (rgb)
        if (int rc = read_shards(h, kShardRgb, rgb)) return rc;
      if (counts)
        if (int rc = read_shards(h, kShardCounts, counts)) return rc;
      return VPTMCM_OK;
    }
    if (int rc = composite_ready(h)) return rc;
    if (counts) {  // sum(n): the composite kernel on the reduced sum, counts only
      CompositeSrc S;
      memset(&S, 0, sizeof S);
      S.n = 1;
      S.p[0] = h->grp_gather;
      if (!h->comp_counts) HIPCHK(h, dev_alloc(&h->comp_counts, npx * sizeof(float)));
      HIPCHK(h, launch_composite(S, (uint32_t)npx, nullptr, nullptr, h->comp_counts, enq(h)));
      HIPCHK(h, hipMemcpyAsync(counts, h->comp_counts, npx * sizeof(float), hipMemcpyDeviceToHost, enq(h)));
    }
    if (rgba16f)
      HIPCHK(h, hipMemcpyAsync(rgba16f, h->grp_rgba, npx * 8, hipMemcpyDeviceToHost, enq(h)));
    if (rgb)
      HIPCHK(h, hipMemcpyAsync(rgb, h->grp_rgb32, npx * 3 * sizeof(float), hipMemcpyDeviceToHost,
                               enq(h)));
    return wait_stream(h, h->stream, "read_composite");
  }
  if (!h->comm || h->comp_last < 0)
    FAIL(h, VPTMCM_ESTATE, "read_composite: no all-reduce issued (and not a device-list handle)");
  HIPCHK(h, hipSetDevice(h->device));
  // on the composite stream, behind the last all-reduce (the march stream keeps running)
  if (!h->comp_rgb32) HIPCHK(h, dev_alloc(&h->comp_rgb32, npx * 3 * sizeof(float)));
  if (!h->comp_rgba) HIPCHK(h, dev_alloc(&h->comp_rgba, npx * 4 * sizeof(uint16_t)));
  if (!h->comp_counts) HIPCHK(h, dev_alloc(&h->comp_counts, npx * sizeof(float)));
  CompositeSrc S;
  memset(&S, 0, sizeof S);
  S.n = 1;
  S.p[0] = h->comp[h->comp_last];
  // (an all-reduce issued inline ran on the march stream)
  HIPCHK(h, hipStreamWaitEvent(h->comm_stream, h->comp_done[h->comp_last], 0));
  if (h->comp_sharded[h->comp_last]) {  // every rank's shard, in place (collective)
    const size_t shard_words = npx * 4 / (size_t)h->nranks;
    float* base = reinterpret_cast<float*>(h->comp[h->comp_last]);
    if (int rc = comm_call(h, ncclAllGather(base + (size_t)h->rank * shard_words, base, shard_words, ncclFloat32,
                                            h->comm, h->comm_stream),
                           "read_composite"))
      return rc;
    HIPCHK(h, hipEventRecord(h->comp_done[h->comp_last], h->comm_stream));
    h->comp_sharded[h->comp_last] = false;
  }
  HIPCHK(h, launch_composite(S, (uint32_t)npx, h->comp_rgb32, h->comp_rgba, h->comp_counts,
                             h->comm_stream));
  if (rgba16f)
    HIPCHK(h, hipMemcpyAsync(rgba16f, h->comp_rgba, npx * 8, hipMemcpyDeviceToHost, h->comm_stream));
  if (rgb)
    HIPCHK(h, hipMemcpyAsync(rgb, h->comp_rgb32, npx * 3 * sizeof(float), hipMemcpyDeviceToHost,
                             h->comm_stream));
  if (counts)
    HIPCHK(h, hipMemcpyAsync(counts, h->comp_counts, npx * sizeof(float), hipMemcpyDeviceToHost,
                             h->comm_stream));
  return wait_stream(h, h->comm_stream, "read_composite");
}

int vptmcm_comm_gather_bands(vptmcm* h, float* rgb) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!h->comm) FAIL(h, VPTMCM_ECOMM, "comm_gather_bands: no communicator");
  if (!rgb) FAIL(h, VPTMCM_EINVAL, "comm_gather_bands: null output");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = 0;
  // The bands must tile the frame: every 8-row tile covered by exactly one rank.
  const uint32_t ty = (h->R + 7) / 8;
  if (!h->band_cover) HIPCHK(h, dev_alloc(&h->band_cover, ty * sizeof(uint32_t)));
  std::vector<uint32_t> cover(ty, 0u);
  for (uint32_t t = h->band_y0 / 8; t < (h->band_y1 + 7) / 8; t++) cover[t] = 1u;
  HIPCHK(h, hipMemcpyAsync(h->band_cover, cover.data(), ty * sizeof(uint32_t), hipMemcpyHostToDevice,
                           h->comm_stream));
  if ((rc = comm_call(h, ncclAllReduce(h->band_cover, h->band_cover, ty, ncclUint32, ncclSum, h->comm,
                                       h->comm_stream), "comm_gather_bands")))
    return rc;
  HIPCHK(h, hipMemcpyAsync(cover.data(), h->band_cover, ty * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           h->comm_stream));
  if ((rc = wait_stream(h, h->comm_stream, "comm_gather_bands"))) return rc;
  for (uint32_t t = 0; t < ty; t++)
    if (cover[t] != 1u)
      FAIL(h, VPTMCM_ECOMM, "comm_gather_bands: rows [%u, %u) are covered by %u ranks' bands (need "
           "exactly 1: the bands must tile the frame)", t * 8, std::min(t * 8 + 8, h->R), cover[t]);
  // Sum of the fp32 images (zero outside each band): exact, up to the sign of
  // a -0.0 pixel (-0 + +0 = +0).
  const size_t n = (size_t)h->R * h->R * 3;
  float* sum = reinterpret_cast<float*>(h->comp[h->comp_next]);  // R*R float4 >= R*R*3 floats
  stream_op(h);
  HIPCHK(h, hipStreamWaitEvent(enq(h), h->comp_done[h->comp_next], 0));
  HIPCHK(h, hipMemcpyAsync(sum, h->rgb32, n * sizeof(float), hipMemcpyDeviceToDevice, enq(h)));
  HIPCHK(h, hipEventRecord(h->comp_ready[h->comp_next], enq(h)));
  HIPCHK(h, hipStreamWaitEvent(h->comm_stream, h->comp_ready[h->comp_next], 0));
  if ((rc = comm_call(h, ncclAllReduce(sum, sum, n, ncclFloat32, ncclSum, h->comm, h->comm_stream),
                      "comm_gather_bands")))
    return rc;
  HIPCHK(h, hipMemcpyAsync(rgb, sum, n * sizeof(float), hipMemcpyDeviceToHost, h->comm_stream));
  HIPCHK(h, hipEventRecord(h->comp_done[h->comp_next], h->comm_stream));
  return wait_stream(h, h->comm_stream, "comm_gather_bands");
}

int vptmcm_comm_barrier(vptmcm* h) {
  double v = 0.0;
  return vptmcm_comm_allreduce_host(h, &v, 1, 0);
}

int vptmcm_comm_allreduce_host(vptmcm* h, double* vals, int n, int op) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!h->comm) FAIL(h, VPTMCM_ECOMM, "comm_allreduce_host: no communicator");
  if (!vals || n < 1 || n > 64 || op < 0 || op > 1)
    FAIL(h, VPTMCM_EINVAL, "comm_allreduce_host: bad arguments");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = wait_stream(h, h->stream, "comm_allreduce_host");
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(h->host_scratch, vals, n * sizeof(double), hipMemcpyHostToDevice,
                           h->comm_stream));
  if ((rc = comm_call(h, ncclAllReduce(h->host_scratch, h->host_scratch, (size_t)n, ncclFloat64,
                                       op ? ncclMax : ncclSum, h->comm, h->comm_stream),
                      "comm_allreduce_host")))
    return rc;
  HIPCHK(h, hipMemcpyAsync(vals, h->host_scratch, n * sizeof(double), hipMemcpyDeviceToHost,
                           h->comm_stream));
  return wait_stream(h, h->comm_stream, "comm_allreduce_host");
}

int vptmcm_debug_last_launch(vptmcm* h, uint32_t info[4], uint64_t* launches) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!info) FAIL(h, VPTMCM_EINVAL, "debug_last_launch: null output");
  info[0] = h->last_launch.mode;
  info[1] = h->last_launch.tpl;
  info[2] = h->last_launch.spec;
  info[3] = h->last_launch.passes;
  if (launches) *launches = h->march_launches;
  return VPTMCM_OK;
}

int vptmcm_debug_schedule(vptmcm* h, uint32_t* out, uint32_t n_words, uint32_t* n_slots) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!n_slots) FAIL(h, VPTMCM_EINVAL, "debug_schedule: null slot count");
  const uint32_t n = sched_slot_words(h->n_tiles);
  *n_slots = n;
  if (!out) return VPTMCM_OK;
  if (n_words < n) FAIL(h, VPTMCM_EINVAL, "debug_schedule: output holds fewer words than slots");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipMemcpyAsync(out, h->sched_prev, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           enq(h)));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return VPTMCM_OK;
}

// --------------------------------------------------------------- diagnostics

int vptmcm_debug_eval(vptmcm* h, int fn, const uint32_t* in, uint32_t* out, uint32_t n) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (fn < 0 || fn > 4 || (!in && n) || (!out && n)) FAIL(h, VPTMCM_EINVAL, "debug_eval: bad args");
  if (n == 0) return VPTMCM_OK;
  HIPCHK(h, hipSetDevice(h->device));
  uint32_t *din = nullptr, *dout = nullptr;
  HIPCHK(h, dev_alloc(&din, (size_t)n * 4));
  if (dev_alloc(&dout, (size_t)n * 4) != hipSuccess) {
    (void)dev_free(din);
    FAIL(h, VPTMCM_ENOMEM, "debug_eval: allocation failed");
  }
  hipError_t e = hipMemcpy(din, in, (size_t)n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_debug_eval(fn, din, dout, n, enq(h));
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)dev_free(din);
  (void)dev_free(dout);
  if (e != hipSuccess) FAIL(h, VPTMCM_EHIP, "debug_eval: %s", hipGetErrorString(e));
  return VPTMCM_OK;
}

int vptmcm_debug_verify(vptmcm* h, int fn, uint32_t lo, uint64_t count, uint64_t* mismatches,
                        uint32_t* first_bad, uint32_t nfirst) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc_ = flush_renders(h)) return rc_;
  if (!mismatches || (nfirst && !first_bad)) FAIL(h, VPTMCM_EINVAL, "debug_verify: bad args");
  HIPCHK(h, hipSetDevice(h->device));
  unsigned long long* dbad = nullptr;
  uint32_t* dfirst = nullptr;
  HIPCHK(h, dev_alloc(&dbad, sizeof(unsigned long long)));
  HIPCHK(h, dev_alloc(&dfirst, (nfirst ? nfirst : 1) * sizeof(uint32_t)));
  HIPCHK(h, hipMemsetAsync(dbad, 0, sizeof(unsigned long long), enq(h)));
  uint64_t done = 0;
  hipError_t e = hipSuccess;
  const MarchParams P = make_params(h, kNoMatrix, 0);  // fn 13 uses the current spectrum
  while (done < count && e == hipSuccess) {  // chunks of 2^31 (u32 range)
    uint64_t chunk = count - done < (1ull << 31) ? count - done : (1ull << 31);
    e = launch_verify(fn, P, (uint32_t)(lo + done), (uint32_t)chunk, dbad, dfirst, nfirst, enq(h));
    done += chunk;
  }
  unsigned long long nb = 0;
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess) e = hipMemcpy(&nb, dbad, sizeof nb, hipMemcpyDeviceToHost);
  if (e == hipSuccess && nfirst)
    e = hipMemcpy(first_bad, dfirst, (size_t)nfirst * sizeof(uint32_t), hipMemcpyDeviceToHost);
  (void)dev_free(dbad);
  (void)dev_free(dfirst);
  if (e != hipSuccess) FAIL(h, VPTMCM_EHIP, "debug_verify: %s", hipGetErrorString(e));
  *mismatches = nb;
  return VPTMCM_OK;
}

// ------------------------------------------------ device-list entry points
// Each input and each pass goes to every replica (replica 0 first, then the
// peers in order); a pass's seed bits become each replica's own stream.

int vptmcm_volume_begin(vptmcm* h, uint32_t width, uint32_t height, uint32_t depth) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return volume_begin_one(c, width, height, depth); });
}

int vptmcm_volume_write_block(vptmcm* h, const uint8_t* data, uint32_t x, uint32_t y, uint32_t z,
                              uint32_t bw, uint32_t bh, uint32_t bd) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return volume_write_block_one(c, data, x, y, z, bw, bh, bd); });
}

int vptmcm_volume_end(vptmcm* h) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return volume_end_one(c); });
}

int vptmcm_set_material_tf(vptmcm* h, const uint8_t* rgba) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_material_tf_one(c, rgba); });
}

int vptmcm_set_light(vptmcm* h, const uint8_t* spd, const float dir[3]) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_light_one(c, spd, dir); });
}

int vptmcm_set_spectrum(vptmcm* h, const float* buf) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_spectrum_one(c, buf); });
}

int vptmcm_set_transfer_function(vptmcm* h, const uint8_t* rgba, uint32_t width, uint32_t height) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_transfer_function_one(c, rgba, width, height); });
}

int vptmcm_set_environment(vptmcm* h, const uint8_t* rgba, uint32_t width, uint32_t height) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_environment_one(c, rgba, width, height); });
}

int vptmcm_set_band(vptmcm* h, uint32_t y0, uint32_t y1) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_band_one(c, y0, y1); });
}

int vptmcm_set_params(vptmcm* h, const vptmcm_params* p) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return set_params_one(c, p); });
}

int vptmcm_reset(vptmcm* h, const float* mvp, uint32_t seed_bits) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return for_replicas(h, [&](vptmcm* c) { return reset_one(c, mvp, replica_seed(seed_bits, c->replica)); });
}

int vptmcm_render(vptmcm* h, const float* mvp, uint32_t seed_bits) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (h->peers.empty()) return render_one(h, mvp, seed_bits);  // the per-pass call: no closure
  return for_replicas(h, [&](vptmcm* c) { return render_one(c, mvp, replica_seed(seed_bits, c->replica)); });
}

int vptmcm_render_passes(vptmcm* h, const float* mvp, const uint32_t* seeds, uint32_t n) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (h->peers.empty()) return render_passes_one(h, mvp, seeds, n);
  if (!seeds && n) FAIL(h, VPTMCM_EINVAL, "render_passes: null argument");
  return for_replicas(h, [&](vptmcm* c) {
    uint32_t rs[kMaxFusedPasses];
    if (n == 0) return render_passes_one(c, mvp, rs, 0);
    for (uint32_t k0 = 0; k0 < n; k0 += kMaxFusedPasses) {
      const uint32_t m = std::min<uint32_t>(n - k0, kMaxFusedPasses);
      for (uint32_t k = 0; k < m; k++) rs[k] = replica_seed(seeds[k0 + k], c->replica);
      if (int rc = render_passes_one(c, mvp, rs, m)) return rc;
    }
    return VPTMCM_OK;
  });
}

int vptmcm_synchronize(vptmcm* h) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (int rc = for_replicas(h, [&](vptmcm* c) { return synchronize_one(c); })) return rc;
  h->grp_synced_seq = h->grp_seq;  // every composite issued so far is complete
  return VPTMCM_OK;
}

int vptmcm_enable_kernel_timing(vptmcm* h, int enable) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  return enable_kernel_timing_one(h, enable);  // replica 0 only (see vptmcm_kernel_time)
}

int vptmcm_set_macro_skip(vptmcm* h, int mode) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (mode < 0 || mode > 2) FAIL(h, VPTMCM_EINVAL, "set_macro_skip: mode %d (0 off, 1 on, 2 auto)", mode);
  if (int rc = flush_renders(h)) return rc;  // queued passes keep the mode they were queued under
  return for_replicas(h, [&](vptmcm* c) {
    c->maj_tune.mode = mode;
    maj_tune_reset(c);
    return VPTMCM_OK;
  });
}

int vptmcm_composite(vptmcm* h) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (!composited(h)) return VPTMCM_OK;
  return group_composite(h);
}

int vptmcm_group_devices(vptmcm* h, int32_t* devices, uint32_t* n) {
  if (check_handle(h)) return VPTMCM_EINVAL;
  if (!n) FAIL(h, VPTMCM_EINVAL, "group_devices: null count");
  *n = 1u + (uint32_t)h->peers.size();
  if (devices) {
    devices[0] = h->device;
    for (size_t k = 0; k < h->peers.size(); k++) devices[k + 1] = h->peers[k]->device;
  }
  return VPTMCM_OK;
}

}  // extern "C"
