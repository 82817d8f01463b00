// DIAGNOSTIC (never shipped, round 4): what one wave per SIMD pays on gfx950
// for (a) dependent integer VALU chains, (b) a divergent if-region, (c) a
// wave-uniform ballot branch -- the three shapes of the FULL4 turn code.
// One workgroup of 256 threads per CU (one wave per SIMD), HIP events,
// best of 5.  Build:
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o tools/diag/build/libissue_probe.so tools/diag/issue_probe.hip
// run: python3 -c "import ctypes; ctypes.CDLL('tools/diag/build/libissue_probe.so').issue_probe_main()"
#include <hip/hip_runtime.h>

#include <cstdio>

#define STEP(a, s, c) a = ((a) ^ ((a) << (s))) + (c)

template <int K>
__global__ void chains(uint32_t* out, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * (2u * k + 3u);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 32 / K; ++r) {
#pragma unroll
      for (int k = 0; k < K; ++k) STEP(a[k], 3 + k, 0x9E3779B9u + k);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// 8 chains, plus every 8 steps a divergent if-region of 3 VALU taken by ~1/8
// of the lanes (a branch the compiler keeps: the body has a side effect on a
// loop-carried value and an asm barrier)
__global__ void divergent(uint32_t* out, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * (2u * k + 3u);
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) STEP(a[k], 3 + k, 0x9E3779B9u + k);
      if ((a[r] & 7u) == 3u) {
        asm volatile("" ::: "memory");
        acc = (acc ^ a[r + 1]) + (a[r + 2] >> 3);
      }
    }
  }
  uint32_t x = acc;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// 8 chains, plus every 8 steps a wave-uniform branch on a ballot (taken by
// no wave: the test's cost only)
__global__ void uniform(uint32_t* out, int iters) {
  uint32_t a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * (2u * k + 3u);
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) STEP(a[k], 3 + k, 0x9E3779B9u + k);
      if (__ballot(a[r] == 0x12345677u) != 0ull) {
        asm volatile("" ::: "memory");
        acc += a[r + 1];
      }
    }
  }
  uint32_t x = acc;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <class F>
static float run(F launch) {
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
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best;
}

extern "C" int issue_probe_main() {
  uint32_t* d;
  if (hipMalloc(&d, 256 * 512 * sizeof(uint32_t)) != hipSuccess) return 1;
  const int it = 5000;  // 32 chain steps per iteration
  const float c1 = run([&] { chains<1><<<256, 256>>>(d, it); });
  const float c2 = run([&] { chains<2><<<256, 256>>>(d, it); });
  const float c4 = run([&] { chains<4><<<256, 256>>>(d, it); });
  const float c8 = run([&] { chains<8><<<256, 256>>>(d, it); });
  const float c8w2 = run([&] { chains<8><<<256, 512>>>(d, it); });
  const float c1w2 = run([&] { chains<1><<<256, 512>>>(d, it); });
  const float dv = run([&] { divergent<<<256, 256>>>(d, it); });
  const float un = run([&] { uniform<<<256, 256>>>(d, it); });
  // per chain step (2 VALU: shift + xor-add), and per if-region (4 per iteration), cycles at 2.4 GHz
  const double steps = 32.0 * it;
  auto cyc = [&](float ms) { return ms * 1e-3 * 2.4e9 / steps; };
  auto reg = [&](float ms) { return (ms - c8) * 1e-3 * 2.4e9 / (4.0 * it); };
  printf("{\"iters\": %d, \"cycles_per_step\": {\"chain1\": %.2f, \"chain2\": %.2f, \"chain4\": %.2f, "
         "\"chain8\": %.2f, \"chain8_2waves\": %.2f, \"chain1_2waves\": %.2f}, "
         "\"cycles_per_region\": {\"divergent_if\": %.2f, \"ballot_branch\": %.2f}, "
         "\"ms\": [%.4f, %.4f, %.4f, %.4f, %.4f, %.4f, %.4f, %.4f]}\n",
         it, cyc(c1), cyc(c2), cyc(c4), cyc(c8), cyc(c8w2), cyc(c1w2), reg(dv), reg(un), c1, c2, c4, c8, c8w2, c1w2,
         dv, un);
  hipFree(d);
  return 0;
}
