// tools/issue_probe.hip -- the VALU issue rate of gfx950 on the rules
// engine's own instruction mix, at 1, 2 and 4 waves per SIMD (measurement
// tool, never shipped; its result is the basis of bench.py's ISSUE_PEAK and
// tools/sq_summary.py, committed as profiles/r05/issue_probe/).
//
// Each kernel runs one VALU instruction kind, written as inline asm so the
// count and the opcode are exact: 8 independent accumulators per lane, 32
// instructions per loop trip (no dependent pair closer than 8 apart), one
// workgroup per CU of 256 x W threads (W waves on each of the CU's 4
// SIMDs).  Every wave reads the shader clock (s_memtime) before and after
// its loop, so the result is in cycles, independent of the clock the chip
// holds:  cycles per instruction of one wave, and the SIMD's issue interval
// = cycles / (instructions x W) (the W waves of a SIMD run side by side).
// The same kernels run under rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
// SQ_BUSY_CYCLES SQ_WAVE_CYCLES (tools/issue_probe.py --pmc), each kind a
// distinct kernel name.
//
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o tools/build/libissue_probe.so tools/issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {

constexpr int kAcc = 8;

// one instruction kind: apply(a, b) issues exactly one VALU instruction that
// reads and writes accumulator a (b, c: loop-invariant operands)
#define KIND(NAME, BODY)                                                                      \
  struct NAME {                                                                               \
    static __device__ __forceinline__ void apply(uint32_t& a, uint32_t b, uint32_t c,         \
                                                 uint64_t m) { (void)b; (void)c; (void)m; BODY; } \
  };

KIND(k_add_u32, asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_xor_b32, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_lshlrev_b32, asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a)))
KIND(k_bfe_u32, asm volatile("v_bfe_u32 %0, %0, %1, 4" : "+v"(a) : "v"(b)))
KIND(k_bitop3_b32, asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_add3_u32, asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_cndmask_b32, asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m)))
KIND(k_sub_u32_sdwa,
     asm volatile("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1"
                  : "+v"(a) : "v"(b)))
KIND(k_bcnt_u32_b32, asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_ffbl_b32, asm volatile("v_ffbl_b32 %0, %0" : "+v"(a)))
KIND(k_perm_b32, asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_mul_hi_u32, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_mul_lo_u32, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_fma_f32, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_cmp_eq_u32, asm volatile("v_cmp_eq_u32_e64 s[2:3], %0, %1" : : "v"(a), "v"(b) : "s2", "s3"))
KIND(k_and_b32, asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_or_b32, asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_sub_u32, asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_mov_b32, asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(a ^ b)))
KIND(k_lshrrev_b32, asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a)))
KIND(k_not_b32, asm volatile("v_not_b32 %0, %0" : "+v"(a)))
KIND(k_min_u32, asm volatile("v_min_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_max_i32, asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_or3_b32, asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_and_or_b32, asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)))
KIND(k_lshl_or_b32, asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : "+v"(a) : "v"(b)))
KIND(k_cndmask_vcc, asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a) : "v"(b)))
// a compare writing vcc, then a select reading it (the compiler's usual pair)
KIND(k_cmp_cnd_vcc, asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc"
                                 : "+v"(a) : "v"(b), "v"(c) : "vcc"))
// the same pair through an SGPR pair (e64 forms)
KIND(k_cmp_cnd_sgpr, asm volatile("v_cmp_gt_u32_e64 s[6:7], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %2, s[6:7]"
                                  : "+v"(a) : "v"(b), "v"(c) : "s6", "s7"))
// v_cndmask_b32_e32 reading a vcc that a VALU compare wrote once before the loop
KIND(k_cndmask_vcc_valu, asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a) : "v"(b)))
KIND(k_readlane_b32, asm volatile("v_readlane_b32 s4, %0, 5\n\tv_add_u32 %0, s4, %0" : "+v"(a) : : "s4"))
KIND(k_add_f32, asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_pk_add_u16, asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b)))
KIND(k_mul_u32_u24, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(b)))

// scalar instructions beside the VALU stream of one wave (round 5): what an
// SALU instruction, a lane-mask combine, a not-taken and a taken branch cost
// a lone wave between its VALU instructions
KIND(k_add_sadd, asm volatile("v_add_u32 %0, %0, %1\n\ts_add_u32 s8, s8, 1" : "+v"(a) : "v"(b) : "s8", "scc"))
KIND(k_add_sand64, asm volatile("v_add_u32 %0, %0, %1\n\ts_and_b64 s[8:9], s[8:9], s[10:11]"
                                : "+v"(a) : "v"(b) : "s8", "s9", "scc"))
KIND(k_sadd_only, asm volatile("s_add_u32 s8, s8, 1" : : : "s8", "scc"))
KIND(k_add_cbranch_nt, asm volatile("v_add_u32 %0, %0, %1\n\ts_cmp_eq_u32 s8, 0x12345\n\ts_cbranch_scc1 1f\n1:"
                                    : "+v"(a) : "v"(b) : "scc"))
KIND(k_add_branch_taken, asm volatile("v_add_u32 %0, %0, %1\n\ts_branch 1f\n1:" : "+v"(a) : "v"(b)))

// 64-bit kinds: a 64-bit accumulator, so the register pair is exact (the
// mad's carry-out goes to one SGPR pair, as the product's Philox and mulhi
// code does).  The compiler puts an s_nop after each carry / compare write
// of an SGPR pair here: tools/issue_probe.py reports every loop's exact
// instruction composition from the build's assembly beside its cycles.
struct k_mad_u64_u32 {
  static __device__ __forceinline__ void apply64(uint64_t& a, uint32_t b, uint32_t c) {
    asm volatile("v_mad_u64_u32 %0, s[2:3], %1, %2, %0" : "+v"(a) : "v"(b), "v"(c) : "s2", "s3");
  }
};
struct k_lshlrev_b64 {
  static __device__ __forceinline__ void apply64(uint64_t& a, uint32_t b, uint32_t c) {
    (void)b; (void)c;
    asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(a));
  }
};
struct k_lshl_add_u64 {
  static __device__ __forceinline__ void apply64(uint64_t& a, uint32_t b, uint32_t c) {
    (void)c;
    const uint64_t x = b;
    asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(a) : "v"(x));
  }
};

template <class K> struct requires_vcc { static constexpr bool value = false; };
template <> struct requires_vcc<k_cndmask_vcc_valu> { static constexpr bool value = true; };

struct Clock {
  uint64_t t0, t1;
};

template <class K>
__global__ void __launch_bounds__(1024) probe32(uint32_t* out, Clock* clk, int iters) {
  uint32_t a[kAcc];
  const uint32_t b = threadIdx.x | 1u, c = 0x9E3779B9u ^ threadIdx.x;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) a[k] = threadIdx.x * (2u * k + 3u);
  const uint64_t m = __ballot(threadIdx.x & 1u);  // the cndmask kind's lane mask
  asm volatile("s_mov_b64 vcc, %0" : : "s"(m) : "vcc");  // the vcc cndmask kind's
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 32 / kAcc; ++r) {
#pragma unroll
      for (int k = 0; k < kAcc; ++k) K::apply(a[k], b, c, m);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) x ^= a[k];
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) clk[gw] = Clock{t0, t1};
}

// probe32 with vcc written by a VALU compare before the loop
template <class K>
__global__ void __launch_bounds__(1024) probe32v(uint32_t* out, Clock* clk, int iters) {
  uint32_t a[kAcc];
  const uint32_t b = threadIdx.x | 1u, c = 0x9E3779B9u ^ threadIdx.x;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) a[k] = threadIdx.x * (2u * k + 3u);
  asm volatile("v_cmp_ne_u32_e32 vcc, 0, %0" : : "v"(threadIdx.x & 1u) : "vcc");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 32 / kAcc; ++r) {
#pragma unroll
      for (int k = 0; k < kAcc; ++k) K::apply(a[k], b, c, 0ull);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) x ^= a[k];
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) clk[gw] = Clock{t0, t1};
}

template <class K>
__global__ void __launch_bounds__(1024) probe64(uint32_t* out, Clock* clk, int iters) {
  uint64_t a[kAcc];
  const uint32_t b = threadIdx.x | 1u, c = 0x9E3779B9u ^ threadIdx.x;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) a[k] = threadIdx.x * (2ull * k + 3ull);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 32 / kAcc; ++r) {
#pragma unroll
      for (int k = 0; k < kAcc; ++k) K::apply64(a[k], b, c);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t x = 0;
#pragma unroll
  for (int k = 0; k < kAcc; ++k) x ^= a[k];
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(x ^ (x >> 32));
  if ((threadIdx.x & 63) == 0) clk[gw] = Clock{t0, t1};
}

struct Result {
  float ms;             // best of 5 launches, HIP events
  double cyc_per_wave;  // mean over waves of (t1 - t0), shader cycles
  double cyc_max;       // slowest wave
};

template <class F>
Result run(F launch, Clock* dclk, int nwaves) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  static Clock h[256 * 16];
  hipMemcpy(h, dclk, sizeof(Clock) * nwaves, hipMemcpyDeviceToHost);
  double sum = 0, mx = 0;
  for (int w = 0; w < nwaves; ++w) {
    const double d = (double)(h[w].t1 - h[w].t0);
    sum += d;
    mx = d > mx ? d : mx;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return Result{best, sum / nwaves, mx};
}

template <class K, bool k64>
void one(const char* name, uint32_t* d, Clock* dclk, int iters, bool& first) {
  for (int W : {1, 2, 4}) {
    const int threads = 256 * W, nwaves = 256 * 4 * W;
    Result res = run(
        [&] {
          if constexpr (k64) {
            if constexpr (sizeof(K) == 1 && requires_vcc<K>::value) probe32v<K><<<256, threads>>>(d, dclk, iters);
            else probe64<K><<<256, threads>>>(d, dclk, iters);
          } else {
            probe32<K><<<256, threads>>>(d, dclk, iters);
          }
        },
        dclk, nwaves);
    const double insts = 32.0 * iters;  // VALU instructions of the kind per wave
    std::printf("%s{\"kind\": \"%s\", \"waves_per_simd\": %d, \"insts_per_wave\": %.0f, \"ms\": %.4f, "
                "\"cycles_per_wave\": %.0f, \"cycles_per_wave_max\": %.0f, \"cycles_per_inst_one_wave\": %.3f, "
                "\"simd_issue_interval_cycles\": %.3f, \"clock_ghz_implied\": %.3f}",
                first ? "" : ",\n", name, W, insts, res.ms, res.cyc_per_wave, res.cyc_max,
                res.cyc_per_wave / insts, res.cyc_per_wave / (insts * W), res.cyc_max / (res.ms * 1e6));
    first = false;
  }
}

}  // namespace

// the scalar kinds alone (tools/issue_probe.py --scalar)
extern "C" int issue_probe_scalar(int iters) {
  uint32_t* d;
  Clock* dclk;
  if (hipMalloc(&d, 256 * 1024 * sizeof(uint32_t)) != hipSuccess) return 1;
  if (hipMalloc(&dclk, 256 * 16 * sizeof(Clock)) != hipSuccess) return 1;
  bool first = true;
  std::printf("[\n");
  one<k_add_u32, false>("v_add_u32", d, dclk, iters, first);
  one<k_add_sadd, false>("v_add_u32+s_add_u32", d, dclk, iters, first);
  one<k_add_sand64, false>("v_add_u32+s_and_b64", d, dclk, iters, first);
  one<k_sadd_only, false>("s_add_u32", d, dclk, iters, first);
  one<k_add_cbranch_nt, false>("v_add_u32+s_cmp+s_cbranch (not taken)", d, dclk, iters, first);
  one<k_add_branch_taken, false>("v_add_u32+s_branch (taken)", d, dclk, iters, first);
  std::printf("\n]\n");
  std::fflush(stdout);
  hipFree(d);
  hipFree(dclk);
  return 0;
}

extern "C" int issue_probe_main(int iters) {
  uint32_t* d;
  Clock* dclk;
  if (hipMalloc(&d, 256 * 1024 * sizeof(uint32_t)) != hipSuccess) return 1;
  if (hipMalloc(&dclk, 256 * 16 * sizeof(Clock)) != hipSuccess) return 1;
  bool first = true;
  std::printf("[\n");
  one<k_add_u32, false>("v_add_u32", d, dclk, iters, first);
  one<k_xor_b32, false>("v_xor_b32", d, dclk, iters, first);
  one<k_lshlrev_b32, false>("v_lshlrev_b32", d, dclk, iters, first);
  one<k_bfe_u32, false>("v_bfe_u32", d, dclk, iters, first);
  one<k_bitop3_b32, false>("v_bitop3_b32", d, dclk, iters, first);
  one<k_add3_u32, false>("v_add3_u32", d, dclk, iters, first);
  one<k_cndmask_b32, false>("v_cndmask_b32_e64", d, dclk, iters, first);
  one<k_sub_u32_sdwa, false>("v_sub_u32_sdwa", d, dclk, iters, first);
  one<k_bcnt_u32_b32, false>("v_bcnt_u32_b32", d, dclk, iters, first);
  one<k_ffbl_b32, false>("v_ffbl_b32", d, dclk, iters, first);
  one<k_perm_b32, false>("v_perm_b32", d, dclk, iters, first);
  one<k_cmp_eq_u32, false>("v_cmp_eq_u32_e64", d, dclk, iters, first);
  one<k_mul_hi_u32, false>("v_mul_hi_u32", d, dclk, iters, first);
  one<k_mul_lo_u32, false>("v_mul_lo_u32", d, dclk, iters, first);
  one<k_fma_f32, false>("v_fma_f32", d, dclk, iters, first);
  one<k_and_b32, false>("v_and_b32", d, dclk, iters, first);
  one<k_or_b32, false>("v_or_b32", d, dclk, iters, first);
  one<k_sub_u32, false>("v_sub_u32", d, dclk, iters, first);
  one<k_mov_b32, false>("v_mov_b32", d, dclk, iters, first);
  one<k_lshrrev_b32, false>("v_lshrrev_b32", d, dclk, iters, first);
  one<k_not_b32, false>("v_not_b32", d, dclk, iters, first);
  one<k_min_u32, false>("v_min_u32", d, dclk, iters, first);
  one<k_max_i32, false>("v_max_i32", d, dclk, iters, first);
  one<k_or3_b32, false>("v_or3_b32", d, dclk, iters, first);
  one<k_and_or_b32, false>("v_and_or_b32", d, dclk, iters, first);
  one<k_lshl_or_b32, false>("v_lshl_or_b32", d, dclk, iters, first);
  one<k_cndmask_vcc, false>("v_cndmask_b32_e32", d, dclk, iters, first);
  one<k_readlane_b32, false>("v_readlane_b32", d, dclk, iters, first);
  one<k_cmp_cnd_vcc, false>("v_cmp_e32+v_cndmask_e32 (vcc)", d, dclk, iters, first);
  one<k_cmp_cnd_sgpr, false>("v_cmp_e64+v_cndmask_e64 (sgpr)", d, dclk, iters, first);
  one<k_cndmask_vcc_valu, true>("v_cndmask_b32_e32 (vcc from a VALU compare)", d, dclk, iters, first);
  one<k_add_f32, false>("v_add_f32", d, dclk, iters, first);
  one<k_pk_add_u16, false>("v_pk_add_u16", d, dclk, iters, first);
  one<k_mul_u32_u24, false>("v_mul_u32_u24", d, dclk, iters, first);
  one<k_mad_u64_u32, true>("v_mad_u64_u32", d, dclk, iters, first);
  one<k_lshlrev_b64, true>("v_lshlrev_b64", d, dclk, iters, first);
  one<k_lshl_add_u64, true>("v_lshl_add_u64", d, dclk, iters, first);
  std::printf("\n]\n");
  std::fflush(stdout);
  hipFree(d);
  hipFree(dclk);
  return 0;
}
