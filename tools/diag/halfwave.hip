// DIAGNOSTIC (never shipped): does a wave64 whose upper 32 lanes are
// inactive issue VALU work faster on gfx950 than a full wave?  Integer VALU
// chains (8 independent accumulators per lane, issue-bound), timed with HIP
// events over 256 workgroups (one per CU):
//   A  4 waves/CU (1 per SIMD), all 64 lanes working         -> 65,536 lanes of work
//   B  8 waves/CU (2 per SIMD), lanes 0-31 working, 32-63 idle -> 65,536 lanes
//   C  8 waves/CU (2 per SIMD), all 64 lanes working          -> 131,072 lanes
//   D  4 waves/CU, lanes 0-31 working                         -> 32,768 lanes
// If B ~ A / 2, a half-empty wave costs half the issue: FULL4 could run two
// 32-env rule waves per SIMD.  Build: hipcc -O3 --offload-arch=gfx950
// -shared -fPIC -o tools/diag/build/libhalfwave.so tools/diag/halfwave.hip;
// run: python3 -c "import ctypes; ctypes.CDLL('tools/diag/build/libhalfwave.so').halfwave_main()"
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void chains(uint32_t* out, int iters, int active_lanes) {
  const int lane = threadIdx.x & 63;
  if (lane >= active_lanes) return;
  uint32_t a0 = threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u,
           a6 = a0 * 17u, a7 = a0 * 19u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a0 = (a0 ^ (a0 << 3)) + 0x9E3779B9u;
      a1 = (a1 ^ (a1 >> 5)) + 0x7F4A7C15u;
      a2 = (a2 ^ (a2 << 7)) + 0x85EBCA6Bu;
      a3 = (a3 ^ (a3 >> 9)) + 0xC2B2AE35u;
      a4 = (a4 ^ (a4 << 11)) + 0x27D4EB2Fu;
      a5 = (a5 ^ (a5 >> 13)) + 0x165667B1u;
      a6 = (a6 ^ (a6 << 2)) + 0xD3A2646Cu;
      a7 = (a7 ^ (a7 >> 4)) + 0xFD7046C5u;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

static float run(uint32_t* d, int threads, int active, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  chains<<<256, threads>>>(d, iters, active);  // warm
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    chains<<<256, threads>>>(d, iters, active);
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

extern "C" int halfwave_main() {
  uint32_t* d;
  if (hipMalloc(&d, 256 * 512 * sizeof(uint32_t)) != hipSuccess) return 1;
  const int iters = 20000;
  const float A = run(d, 256, 64, iters);
  const float B = run(d, 512, 32, iters);
  const float C = run(d, 512, 64, iters);
  const float D = run(d, 256, 32, iters);
  printf("{\"iters\": %d, \"A_4w_full_ms\": %.4f, \"B_8w_half_ms\": %.4f, \"C_8w_full_ms\": %.4f, "
         "\"D_4w_half_ms\": %.4f}\n", iters, A, B, C, D);
  hipFree(d);
  return 0;
}
