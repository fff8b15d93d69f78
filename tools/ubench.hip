// Instruction issue-cost / latency micro-benchmark for gfx950 (tuning aid, not
// part of the product). Each kernel runs REPS unrolled copies of one
// instruction, either on 8 independent registers (issue cost) or as one
// dependent chain (latency), and reports s_memtime cycles per instruction for
// one wave per SIMD (block of 64 threads x 4 waves = 1/SIMD) and two waves per
// SIMD (8 waves per block).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench.hip -o tools/ubench && tools/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REPS 64
#define ITERS 256

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

#define IND8(INS)                                                                          \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS       \
               " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS          \
               " %6, %6, %8\n\t" INS " %7, %7, %8"                                         \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),      \
                 "+v"(a7)                                                                  \
               : "v"(b));
#define DEP8(INS)                                                                          \
  asm volatile(INS " %0, %0, %1\n\t" INS " %0, %0, %1\n\t" INS " %0, %0, %1\n\t" INS       \
               " %0, %0, %1\n\t" INS " %0, %0, %1\n\t" INS " %0, %0, %1\n\t" INS          \
               " %0, %0, %1\n\t" INS " %0, %0, %1"                                         \
               : "+v"(a0)                                                                  \
               : "v"(b));
#define IND8_1(INS)                                                                        \
  asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS \
               " %4, %4\n\t" INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"             \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),      \
                 "+v"(a7));
#define DEP8_1(INS)                                                                        \
  asm volatile(INS " %0, %0\n\t" INS " %0, %0\n\t" INS " %0, %0\n\t" INS " %0, %0\n\t" INS \
               " %0, %0\n\t" INS " %0, %0\n\t" INS " %0, %0\n\t" INS " %0, %0"             \
               : "+v"(a0));

#define KERNEL(NAME, BODY)                                                                 \
  __global__ void NAME(unsigned long long* out, uint32_t seed) {                          \
    uint32_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,  \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1u;                         \
    unsigned long long t0 = now();                                                         \
    for (int it = 0; it < ITERS; it++) {                                                   \
      _Pragma("unroll") for (int r = 0; r < REPS / 8; r++) { BODY }                        \
    }                                                                                      \
    unsigned long long t1 = now();                                                         \
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;       \
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345) out[4096] = 1;                   \
  }

KERNEL(k_mul_lo_ind, IND8("v_mul_lo_u32"))
KERNEL(k_mul_lo_dep, DEP8("v_mul_lo_u32"))
KERNEL(k_mul_u24_ind, IND8("v_mul_u32_u24"))
KERNEL(k_add_ind, IND8("v_add_u32"))
KERNEL(k_add_dep, DEP8("v_add_u32"))
KERNEL(k_fma_ind, IND8("v_fmac_f32"))
KERNEL(k_fma_dep, DEP8("v_fmac_f32"))
KERNEL(k_xor_ind, IND8("v_xor_b32"))
KERNEL(k_lshr_ind, IND8("v_lshrrev_b32"))
KERNEL(k_rcp_ind, IND8_1("v_rcp_f32"))
KERNEL(k_rcp_dep, DEP8_1("v_rcp_f32"))
KERNEL(k_cvt_ind, IND8_1("v_cvt_f32_u32"))
KERNEL(k_cvtub_ind, IND8_1("v_cvt_f32_ubyte1"))
KERNEL(k_snop, asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");)
KERNEL(k_salu, asm volatile("s_add_u32 s0, s0, 1\n\ts_add_u32 s1, s1, 1\n\ts_add_u32 s2, s2, 1\n\ts_add_u32 s3, s3, 1\n\ts_add_u32 s4, s4, 1\n\ts_add_u32 s5, s5, 1\n\ts_add_u32 s6, s6, 1\n\ts_add_u32 s7, s7, 1" ::: "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "scc");)
KERNEL(k_mix_sv, asm volatile("v_add_u32 %0, %0, %2\n\ts_add_u32 s0, s0, 1\n\tv_add_u32 %1, %1, %2\n\ts_add_u32 s1, s1, 1\n\tv_add_u32 %0, %0, %2\n\ts_add_u32 s2, s2, 1\n\tv_add_u32 %1, %1, %2\n\ts_add_u32 s3, s3, 1" : "+v"(a0), "+v"(a1) : "v"(b) : "s0", "s1", "s2", "s3", "scc");)
KERNEL(k_cndmask, asm volatile("v_cmp_gt_u32 vcc, %2, %0\n\tv_cndmask_b32 %1, %1, %0, vcc\n\tv_cmp_gt_u32 vcc, %2, %1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\tv_cmp_gt_u32 vcc, %2, %0\n\tv_cndmask_b32 %1, %1, %0, vcc\n\tv_cmp_gt_u32 vcc, %2, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0), "+v"(a1) : "v"(b) : "vcc");)
KERNEL(k_saveexec, asm volatile("v_cmp_gt_u32 s[0:1], %1, %0\n\ts_and_saveexec_b64 s[2:3], s[0:1]\n\ts_or_b64 exec, exec, s[2:3]\n\tv_add_u32 %0, %0, %1\n\tv_cmp_gt_u32 s[0:1], %1, %0\n\ts_and_saveexec_b64 s[2:3], s[0:1]\n\ts_or_b64 exec, exec, s[2:3]\n\tv_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b) : "s0", "s1", "s2", "s3", "scc");)

typedef void (*kfn)(unsigned long long*, uint32_t);
struct K { const char* name; kfn f; };

int main() {
  K ks[] = {{"v_mul_lo_u32 ind", k_mul_lo_ind}, {"v_mul_lo_u32 dep", k_mul_lo_dep},
            {"v_mul_u32_u24 ind", k_mul_u24_ind}, {"v_add_u32 ind", k_add_ind},
            {"v_add_u32 dep", k_add_dep}, {"v_fmac_f32 ind", k_fma_ind},
            {"v_fmac_f32 dep", k_fma_dep}, {"v_xor_b32 ind", k_xor_ind},
            {"v_lshrrev_b32 ind", k_lshr_ind}, {"v_rcp_f32 ind", k_rcp_ind},
            {"v_rcp_f32 dep", k_rcp_dep}, {"v_cvt_f32_u32 ind", k_cvt_ind},
            {"v_cvt_f32_ubyte1 ind", k_cvtub_ind}, {"s_nop 0", k_snop},
            {"s_add_u32 ind", k_salu}, {"v_add+s_add interleaved (per instr)", k_mix_sv},
            {"v_cmp+v_cndmask dep pair (per instr)", k_cndmask},
            {"cmp+saveexec+or+add (per instr)", k_saveexec}};
  unsigned long long* d;
  hipMalloc(&d, 8 * 8192);
  unsigned long long h[4096];
  for (auto& k : ks) {
    for (int wps = 1; wps <= 4; wps++) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(256 * wps), 0, 0, d, 7u);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(k.f, dim3(1), dim3(256 * wps), 0, 0, d, 7u);
      hipMemcpy(h, d, 8 * 16, hipMemcpyDeviceToHost);
      double m = 0;
      for (int w = 0; w < 4 * wps; w++) m += (double)h[w];
      m /= 4 * wps;
      // s_memtime counts at the shader clock on gfx950 (see MI355X_MICROARCH.md)
      printf("%-40s waves/SIMD=%d  cycles/instr=%.2f\n", k.name, wps, m / (ITERS * REPS));
    }
  }
  hipFree(d);
  return 0;
}
