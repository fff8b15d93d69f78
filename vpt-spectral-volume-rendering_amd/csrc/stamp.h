// stamp.h — measurement-build hooks of k_march (tools/stamp_profile.py builds
// lib/libvptmcm_stamp.so with -DVPT_STAMP=1). Per wave: s_memtime sums of the
// volume step's segments, the launch's shader cycles, 100 MHz real time, the
// wave's hardware ids; written over the fp32 image, which these builds do not
// store. The product library has VPT_STAMP 0 and every hook is empty.
//
// Segments (two 16-bit cycle sums per word, one-pass launches): [0] step head,
// [1] gather issue + shadow, [2] exposed gather wait, [3] filter + TF + decision,
// [4] decision branches, [5] robust/all-exit steps; word 3 = volume steps,
// word 4 = launch cycles.
#pragma once

#ifndef VPT_STAMP
#define VPT_STAMP 0
#endif

// VPT_STAMP == 2 (timeline build, tools/timeline_profile.py): per wave the
// 100 MHz s_memrealtime at five points of the launch — [0] entry, [1] tile
// scheduled, [2] LDS filled and photon state resident, [3] pass loop done,
// [4] state, image and flag stores complete — plus the words 5 and 7 above.
#if VPT_STAMP == 2
#define TL_DECL() uint32_t tl[6] = {0u, 0u, 0u, 0u, 0u, 0u}
#define TL_MARK(k) (tl[k] = (uint32_t)__builtin_amdgcn_s_memrealtime())
#define TL_MARK_WAIT(k)                   \
  do {                                    \
    __builtin_amdgcn_s_waitcnt(0x0F70);   \
    TL_MARK(k);                           \
  } while (0)
// extra (non-zero): word 6 instead of the probe time (a caller-defined word)
#define TL_END(out, tile, entered, extra)                                                \
  do {                                                                                   \
    TL_MARK_WAIT(4);                                                                     \
    if (lane == 0u) {                                                                    \
      uint32_t* _o = reinterpret_cast<uint32_t*>(out) + (size_t)(tile) * 8u;             \
      for (int _k = 0; _k < 5; _k++) _o[_k] = tl[_k];                                    \
      _o[5] = ((uint32_t)(entered) & 1u) | ((__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xffu) << 8); \
      _o[6] = (extra) ? (uint32_t)(extra) : tl[5];                                       \
      _o[7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                                 \
    }                                                                                    \
  } while (0)
// -DVPT_TL_PROBE=1: word 6 = the time the TF copy issued at entry has landed
// (a vmcnt(0) wait right after it: serialises the copy and the schedule)
#if VPT_TL_PROBE
#define TL_PROBE(k) TL_MARK_WAIT(k)
#else
#define TL_PROBE(k) \
  do {              \
  } while (0)
#endif
#else
#define TL_PROBE(k) \
  do {              \
  } while (0)
#define TL_DECL() \
  do {            \
  } while (0)
#define TL_MARK(k) \
  do {             \
  } while (0)
#define TL_MARK_WAIT(k) \
  do {                  \
  } while (0)
#define TL_END(out, tile, entered, extra) \
  do {                                    \
  } while (0)
#endif

#if VPT_STAMP == 1
#define STAMP_BEGIN()                                             \
  uint32_t prof[5] = {0u, 0u, 0u, 0u, 0u};                            \
  uint32_t t_prev = (uint32_t)__builtin_amdgcn_s_memtime();           \
  const uint32_t t_launch = t_prev;                                   \
  const uint32_t rt_launch = (uint32_t)__builtin_amdgcn_s_memrealtime()
#define STAMP_AT(k)                                                   \
  do {                                                                \
    const uint32_t _t = (uint32_t)__builtin_amdgcn_s_memtime();       \
    prof[(k) >> 1] += (_t - t_prev) << (((k) & 1) * 16);              \
    t_prev = _t;                                                      \
  } while (0)
#define STAMP_RESTART() (t_prev = (uint32_t)__builtin_amdgcn_s_memtime())
// vmcnt(0) between two stamps: the gather's exposed latency is segment 2
#define STAMP_GATHER_WAIT()                 \
  do {                                      \
    STAMP_AT(1);                            \
    __builtin_amdgcn_s_waitcnt(0x0F70);     \
    STAMP_AT(2);                            \
  } while (0)
#define STAMP_COUNT_STEP() (prof[3]++)
// Lane 0 writes 8 words per tile with vector stores: the 5 sums, entered |
// XCC_ID (hwreg 20) << 8, real time, HW_ID (hwreg 4: wave, SIMD, CU, SH, SE).
#define STAMP_END(out, tile, entered)                                                    \
  do {                                                                                   \
    prof[4] = (uint32_t)__builtin_amdgcn_s_memtime() - t_launch;                         \
    const uint32_t _rt = (uint32_t)__builtin_amdgcn_s_memrealtime() - rt_launch;         \
    if (lane == 0u) {                                                                    \
      uint32_t* _o = reinterpret_cast<uint32_t*>(out) + (size_t)(tile) * 8u;             \
      for (int _k = 0; _k < 5; _k++) _o[_k] = prof[_k];                                  \
      _o[5] = ((uint32_t)(entered) & 1u) | ((__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xffu) << 8); \
      _o[6] = _rt;                                                                       \
      _o[7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                                 \
    }                                                                                    \
  } while (0)
#else
#define STAMP_BEGIN() \
  do {                \
  } while (0)
#define STAMP_AT(k) \
  do {              \
  } while (0)
#define STAMP_RESTART() \
  do {                  \
  } while (0)
#define STAMP_GATHER_WAIT() \
  do {                      \
  } while (0)
#define STAMP_COUNT_STEP() \
  do {                     \
  } while (0)
#define STAMP_END(out, tile, entered) \
  do {                                \
  } while (0)
#endif
