// diag.hip -- DIAGNOSTIC build (never shipped): where a k_rollout ply spends
// its cycles.  Same rules engine as the product (narde_rules.h); env_step is
// restated flat here so s_memtime stamps sit between phases at wave level.
// Each wave accumulates per-phase cycles in scalar registers and lane 0
// writes them once.  Read its SHARES, not its length (the stamps' waits
// forbid overlaps the real kernel has).
#include <hip/hip_runtime.h>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

constexpr int kPhases = 7;

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

#define PHASE(k)                 \
  do {                           \
    const uint64_t now = stamp(); \
    acc[k] += now - prev;        \
    prev = now;                  \
  } while (0)

extern "C" __global__ void __launch_bounds__(256)
k_diag(uint4* p0, uint4* p1, int n, uint32_t env0, uint32_t k0, uint32_t k1, int plies,
       int32_t* obs_out, unsigned long long* cycles) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  Side s = side_from_record(p0[i], p1[i]);
  uint64_t acc[kPhases] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t prev = stamp();
  for (int p = 0; p < plies; ++p) {
    uint32_t r[4];
    philox4x32_10(s.t, env0 + i, 0u, 0u, k0, k1, r);
    int d0, d1;
    dice_from(r[0], 0, d0, d1);
    PHASE(0);
    Legal l1;
    legal2(s, d0, d1, l1);
    const int n1 = l1.count;
    PHASE(1);
    int f1 = 0, t1 = 0;
    legal2_entry(l1, n1 >= 2 ? (int)mulhi_u32(r[1], (uint32_t)n1) : 0, f1, t1);
    bool play1 = n1 >= 1;
    if (n1 >= 2 && t1 == 0 && f1 <= 5) {
      t1 = OFF;
      play1 = legal_contains(l1, f1, t1);
    }
    if (play1) apply_move(s, f1, t1);
    PHASE(2);
    if (n1 >= 2 && play1) {
      const int dist = t1 == OFF ? f1 + 1 : (f1 > t1 ? f1 - t1 : t1 - f1);
      const int rem = (d0 == dist) ? d1 : ((d1 == dist) ? d0 : d1);
      const Blocks bl = block_info(s.O, s.P);
      const uint32_t L2 = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, rem), rem);
      const int c2 = __builtin_popcount(L2);
      const int f2 = select_bit(L2, (int)mulhi_u32(r[2], (uint32_t)c2));
      const int t2 = f2 - rem < 0 ? OFF : f2 - rem;
      if (c2 > 0 && !(t2 == 0 && f2 <= 5)) apply_move(s, f2, t2);
    }
    PHASE(3);
    const bool term = s.off_own == 15u;
    if (!term) side_flip(s);
    s.elapsed += 1u;
    if (term || s.elapsed >= 1000u) {
      const uint32_t t = s.t;
      s = side_reset(r[3]);
      s.t = t;
    }
    s.t += 1u;
    PHASE(4);
    int4* o = reinterpret_cast<int4*>(obs_out + ((size_t)p * n + i) * 24);
#pragma unroll
    for (int q = 0; q < 6; ++q)
      o[q] = make_int4(obs_point(s, 4 * q), obs_point(s, 4 * q + 1), obs_point(s, 4 * q + 2),
                       obs_point(s, 4 * q + 3));
    PHASE(5);
  }
  uint4 a, b;
  side_to_record(s, a, b);
  p0[i] = a;
  p1[i] = b;
  PHASE(6);
  if ((threadIdx.x & 63) == 0) {
    const int w = i >> 6;
    for (int k = 0; k < kPhases; ++k) cycles[w * kPhases + k] = acc[k];
  }
}

__global__ void k_diag_init(uint4* p0, uint4* p1, int n, uint32_t env0, uint32_t k0, uint32_t k1) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t r[4];
  philox4x32_10(0u, env0 + i, 0u, 1u, k0, k1, r);
  Side s = side_reset(r[0]);
  uint4 a, b;
  side_to_record(s, a, b);
  p0[i] = a;
  p1[i] = b;
}

// host launcher: n envs, `warm` untimed plies then `plies` stamped plies;
// cycles_out[waves][kPhases] (host); returns kernel ms of the stamped launch
extern "C" float diag_run(int n, int warm, int plies, unsigned long long* cycles_out) {
  uint4 *p0, *p1;
  int32_t* obs;
  unsigned long long* cyc;
  const int waves = (n + 63) / 64;
  (void)hipMalloc(&p0, n * sizeof(uint4));
  (void)hipMalloc(&p1, n * sizeof(uint4));
  (void)hipMalloc(&obs, (size_t)plies * n * 24 * sizeof(int32_t));
  (void)hipMalloc(&cyc, (size_t)waves * kPhases * sizeof(unsigned long long));
  const int g = (n + 255) / 256;
  k_diag_init<<<g, 256>>>(p0, p1, n, 0u, 7u, 0u);
  if (warm > 0) k_diag<<<g, 256>>>(p0, p1, n, 0u, 7u, 0u, warm < plies ? warm : plies, obs, cyc);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, nullptr);
  k_diag<<<g, 256>>>(p0, p1, n, 0u, 7u, 0u, plies, obs, cyc);
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipMemcpy(cycles_out, cyc, (size_t)waves * kPhases * sizeof(unsigned long long),
                  hipMemcpyDeviceToHost);
  (void)hipFree(p0); (void)hipFree(p1); (void)hipFree(obs); (void)hipFree(cyc);
  return ms;
}
