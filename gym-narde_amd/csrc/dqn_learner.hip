// dqn_learner.hip -- the learner half of the batched DQN driver (config 4,
// gym_narde/dqn.py BatchedDQNDriver) as a handful of fused HIP kernels.
//
// The reference trainer's replay() (train_deepq_pytorch.py:602-750) runs on a
// 64-sample minibatch as ~100 tiny tensor ops; at B = 65,536 envs the driver
// trains on 4,096 samples per step and those ops are launch-bound (each
// kernel boundary costs ~4.5 us on MI355X even inside a CUDA graph).  These
// kernels fold the chains that are not GEMMs:
//   k_per_sample       prioritized sampling (PrioritizedReplayBuffer.sample,
//   + k_per_finish     :279-342): a 64-ary inverse-CDF search per wave,
//                      importance weights, then their normalisation and the
//                      beta / counter step in one block;
//   k_gather_batch     the minibatch rows of the replay ring;
//   k_heads_gather     the online heads at the stored codes only (what the
//   + k_heads_grad_f   loss reads) and their backward: per-row dot products,
//   + k_heads_grad_w   per-code gradient sums in a fixed order;
//   k_relu_grad_partial  a feature layer's ReLU mask + bias gradient (column
//   + k_bias_grad_sum    sums of 64-row blocks, then the blocks in order);
//   k_rowmax_addend    the target move-2 head's max over codes with the
//                      one-hot column added on the fly;
//   k_dqn_loss         targets, TD errors, the decomposed loss (:653-720) and
//                      its gradient w.r.t. the two Q-values -- one block;
//   k_prio_update      new priorities |td| + eps, the running max priority,
//                      the per-update epsilon decay (:745-746) and the
//                      step's cursor / tag advance -- one block;
//   k_grad_sqnorm      clip_grad_norm_ + Adam: per-block squared-norm
//   + k_adam           partials, then every block adds them in order.
// Every scalar the driver updates per step (sampling counter, beta, max
// priority, epsilon) lives in device memory, so a captured graph replays
// with current values.  fp32 throughout, the same operation order as the
// torch restatement (BatchedDQNDriver._update_torch); tests/test_gpu_dqn.py
// checks each kernel against it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/narde.h"
#include "narde_rules.h"

namespace narde_abi {
int set_error(int code, const char* what);  // narde.hip: narde_last_error()'s buffer
}

namespace {

constexpr int kLearnThreads = 1024;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return narde_abi::set_error(NARDE_EHIP, hipGetErrorString(e));
  (void)what;
  return NARDE_OK;
}

int bad(const char* what) { return narde_abi::set_error(NARDE_EINVAL, what); }

// block-wide max / sum over kLearnThreads threads (wave shuffles, then the
// 16 wave results through LDS); every thread gets the result
__device__ __forceinline__ float block_max(float v, float* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  v = lane < kLearnThreads / 64 ? lds[lane] : -__builtin_inff();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  return v;
}

// a fixed-order tree sum (deterministic from run to run)
__device__ __forceinline__ float block_sum(float v, float* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  v = lane < kLearnThreads / 64 ? lds[lane] : 0.0f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  return v;
}

// ---------------------------------------------------------------- sampling
// batch draws u_j = Philox4x32-10({*counter, j, 0, 7}, seed) r0 / 2^32 (24
// significant bits, as torch.rand), v_j = u_j * total; idx_j = the first k
// with cdf[k] > v_j (torch.searchsorted(right=True)), clamped to n - 1, and
// moved to the nearest row with p > 0 if p[k] == 0 (nearest_positive);
// w_j = (n * p[idx] / total)^-beta normalised by the batch max.  Then beta
// <- min(1, beta + beta_inc) and *counter += 1.
// One WAVE per sample (4 per block): a 64-ary search -- each round the 64
// lanes load 64 evenly spaced pivots of the current range and a ballot
// picks the first pivot > v, so 1M rows take 4 dependent rounds instead of
// a binary search's 20 -- then lane 0 writes idx and the unnormalised w.
// k_per_finish (one block, after the kernel boundary) takes the batch max,
// normalises, and steps beta and the counter.
// (One sample per thread with a binary search and the last block
// normalising behind a ticket: 16.3 us at batch 4,096 over 1M rows, 13.4 of
// them the search's dependent loads; the wave search with every block's
// max meeting in one word by atomicMax: 17.2 + 4.5 us -- 1,024 atomics on
// one address serialise.)
constexpr int kSampleWaves = 4;

// the last row before k with p > 0, else the first one after k, else k
// (all rows zero: the caller never samples then); wave-uniform, lane l
// looks at row k - 1 - l (k + 1 + l) each round
__device__ __noinline__ int64_t nearest_positive(const float* __restrict__ p, int64_t n, int64_t k, int lane) {
  for (int64_t hi = k - 1; hi >= 0; hi -= 64) {
    const int64_t r = hi - lane;
    const uint64_t hit = __ballot(r >= 0 && p[r] > 0.0f);
    if (hit) return hi - (int64_t)__builtin_ctzll(hit);
  }
  for (int64_t lo = k + 1; lo < n; lo += 64) {
    const int64_t r = lo + lane;
    const uint64_t hit = __ballot(r < n && p[r] > 0.0f);
    if (hit) return lo + (int64_t)__builtin_ctzll(hit);
  }
  return k;
}

// sample j's row k and its unnormalised weight x (every lane of the wave
// gets both; the wave must be converged)
__device__ __forceinline__ void per_sample_row(const float* __restrict__ p, const float* __restrict__ cdf, int64_t n,
                                               int j, uint32_t k0, uint32_t k1, uint32_t ctr, double beta, int lane,
                                               int64_t& k_out, float& x_out, float& u_out) {
  const float total = cdf[n - 1];
  uint32_t r[4];
  narde::philox4x32_10(ctr, (uint32_t)j, 0u, 7u, k0, k1, r);
  const float u = (float)(r[0] >> 8) * (1.0f / 16777216.0f);
  const float v = u * total;
  // the first k in [lo, lo + len) with cdf[k] > v, or lo + len if none
  int64_t lo = 0, len = n;
  bool split = false;  // a split range ends in a row > v
  while (len > 1) {
    const int64_t step = (len + 63) / 64;
    const int64_t off = (int64_t)(lane + 1) * step - 1;
    const int64_t piv = lo + (off < len ? off : len - 1);
    const uint64_t hit = __ballot(cdf[piv] > v);
    if (hit == 0ull) {  // only possible in the first round: no row > v
      lo += len;
      len = 0;
      break;
    }
    const int64_t f = (int64_t)__builtin_ctzll(hit);
    const int64_t nlo = lo + f * step;
    const int64_t end = lo + len;
    len = (nlo + step < end ? nlo + step : end) - nlo;
    lo = nlo;
    split = true;
  }
  if (len == 1 && !split && !(cdf[lo] > v)) lo += 1;  // n == 1: the range was never split
  int64_t k = lo < n - 1 ? lo : n - 1;
  // never a zero-priority (pending) row: the clamp above (u * total
  // rounded up to total) or a prefix sum whose flat run steps by an ulp
  // (a scan's association differs across tiles) can land on one, and its
  // weight (n * 0)^-beta = inf would turn the batch's weights into NaN.
  // Take the last row before k with p > 0 (64 rows per round; the first
  // one after k if there is none), as DeviceReplay.sample() does.
  if (!(p[k] > 0.0f)) k = nearest_positive(p, n, k, lane);
  k_out = k;
  x_out = powf((float)n * (p[k] / total), -(float)beta);
  u_out = u;
}

__global__ void __launch_bounds__(64 * kSampleWaves) k_per_sample(const float* __restrict__ p,
                                                                  const float* __restrict__ cdf, int64_t n,
                                                                  int batch, uint32_t k0, uint32_t k1,
                                                                  const int64_t* __restrict__ counter,
                                                                  const double* __restrict__ beta,
                                                                  int64_t* __restrict__ idx_out,
                                                                  float* __restrict__ w_out,
                                                                  float* __restrict__ u_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * kSampleWaves + wave;
  if (j < batch) {  // wave-uniform
    int64_t k;
    float x, u;
    per_sample_row(p, cdf, n, j, k0, k1, (uint32_t)*counter, *beta, lane, k, x, u);
    if (lane == 0) {
      idx_out[j] = k;
      w_out[j] = x;
      if (u_out) u_out[j] = u;
    }
  }
}

// k_per_sample and k_gather_batch in one launch (round 6): the wave that
// found sample j's row copies its minibatch row -- s = obs[k], ns =
// obs[(k + stride) % cap] (lane l: columns l, l + 64, ...), a / r / d -- and
// writes the UNNORMALISED weight: k_dqn_loss_prio divides by the batch max
// and steps beta and the counter (k_per_finish's work, in its one block).
// Same rows, same weights, one launch and one kernel boundary fewer twice.
__global__ void __launch_bounds__(64 * kSampleWaves) k_per_sample_gather(
    const float* __restrict__ p, const float* __restrict__ cdf, int64_t n, int batch, uint32_t k0, uint32_t k1,
    const int64_t* __restrict__ counter, const double* __restrict__ beta, int64_t* __restrict__ idx_out,
    float* __restrict__ w_out, int ss, const float* __restrict__ obs, int64_t stride, int64_t cap,
    const int64_t* __restrict__ action, const float* __restrict__ reward, const float* __restrict__ done,
    float* __restrict__ s, float* __restrict__ ns, int64_t* __restrict__ a, float* __restrict__ r,
    float* __restrict__ d) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * kSampleWaves + wave;
  if (j >= batch) return;  // wave-uniform
  int64_t k;
  float x, u;
  per_sample_row(p, cdf, n, j, k0, k1, (uint32_t)*counter, *beta, lane, k, x, u);
  int64_t kn = k + stride;
  if (kn >= cap) kn -= cap;
  const float* so = obs + k * ss;
  const float* no = obs + kn * ss;
  float* sd = s + (size_t)j * ss;
  float* nd = ns + (size_t)j * ss;
  for (int c = lane; c < ss; c += 64) {
    sd[c] = so[c];
    nd[c] = no[c];
  }
  if (lane == 0) {
    idx_out[j] = k;
    w_out[j] = x;
    a[2 * j] = action[2 * k];
    a[2 * j + 1] = action[2 * k + 1];
    r[j] = reward[k];
    d[j] = done[k];
  }
}

// ---------------------------------------------------------------- PER prefix
// p = prio^alpha and cdf = its inclusive prefix sum, the sampler's inputs
// (round 6: torch's pow kernel and rocPRIM's two-kernel look-back scan were
// three launches, 18.5 us of a 1M-row ring per update).  Rows go in chunks of
// kScanChunk (1,024), 4 consecutive rows per thread: k_per_chunk_sums
// writes each chunk's total, k_per_scan adds a chunk's base (the totals of
// the chunks before it, one fixed-order tree per block) to the block scan of
// its rows -- 6.7 + 7.8 us per 1M-row ring.  The same operation order on
// every run; a prefix sum in another association (torch's) differs by
// rounding only.  (Measured and dropped: 4,096-row chunks, 9.2 + 12.4 us;
// one launch whose blocks take tickets and read the earlier chunks' totals
// from tagged 64-bit status words as they appear, 22.0 us at 1,024-row
// chunks and 16.2 at 4,096 -- the wait for the other blocks' totals
// outlasts a kernel boundary.)
constexpr int kScanThreads = 256;
constexpr int kScanQuads = 1;                            // float4s per thread
constexpr int kScanRows = 4 * kScanQuads;                // consecutive rows per thread
constexpr int kScanChunk = kScanRows * kScanThreads;     // rows per chunk (block)

// a thread's rows r0 .. r0 + kScanRows - 1 of prio^alpha (0 past n) and
// their inclusive in-thread sums s, in order; returns the thread's total
__device__ __forceinline__ float per_pow(const float* __restrict__ prio, int64_t n, int64_t r0, float alpha,
                                         float4 (&x)[kScanQuads], float4 (&s)[kScanQuads]) {
  float run = 0.0f;
#pragma unroll
  for (int q = 0; q < kScanQuads; ++q) {
    const int64_t r = r0 + 4 * q;
    float4 v;
    if (r + 3 < n) {
      v = *reinterpret_cast<const float4*>(prio + r);
    } else {
      v.x = r < n ? prio[r] : 0.0f;
      v.y = r + 1 < n ? prio[r + 1] : 0.0f;
      v.z = r + 2 < n ? prio[r + 2] : 0.0f;
      v.w = 0.0f;
    }
    v.x = powf(v.x, alpha);
    v.y = powf(v.y, alpha);
    v.z = powf(v.z, alpha);
    v.w = powf(v.w, alpha);
    x[q] = v;
    s[q].x = run + v.x;
    s[q].y = s[q].x + v.y;
    s[q].z = s[q].y + v.z;
    s[q].w = s[q].z + v.w;
    run = s[q].w;
  }
  return run;
}

// exclusive prefix of the threads' totals t over the block (a wave scan by
// shuffles, then the 4 wave totals through LDS); `all` gets the block total
__device__ __forceinline__ float per_block_excl(float t, float* lds, float& all) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float inc = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) lds[wave] = inc;
  __syncthreads();
  float wb = 0.0f;
  for (int k = 0; k < wave; ++k) wb += lds[k];
  all = lds[0] + lds[1] + lds[2] + lds[3];
  static_assert(kScanThreads == 256, "four waves");
  return wb + (inc - t);
}

__global__ void __launch_bounds__(kScanThreads) k_per_chunk_sums(const float* __restrict__ prio, int64_t n,
                                                                 float alpha, float* __restrict__ chunk) {
  __shared__ float lds[4];
  float4 x[kScanQuads], s[kScanQuads];
  const int64_t r0 = (int64_t)blockIdx.x * kScanChunk + kScanRows * (int64_t)threadIdx.x;
  const float t = per_pow(prio, n, r0, alpha, x, s);
  float all;
  (void)per_block_excl(t, lds, all);
  if (threadIdx.x == 0) chunk[blockIdx.x] = all;
}

// the chunk's base from thread-strided partial sums b (fixed-order tree),
// after per_block_excl's barrier
__device__ __forceinline__ float per_base(float b, float* lds2) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
  if ((threadIdx.x & 63) == 0) lds2[threadIdx.x >> 6] = b;
  __syncthreads();
  return (lds2[0] + lds2[1]) + (lds2[2] + lds2[3]);
}

__device__ __forceinline__ void per_store(float* __restrict__ p, float* __restrict__ cdf, int64_t n, int64_t r0,
                                          const float4 (&x)[kScanQuads], const float4 (&s)[kScanQuads], float base,
                                          float e) {
#pragma unroll
  for (int q = 0; q < kScanQuads; ++q) {
    const int64_t r = r0 + 4 * q;
    const float4 c =
        make_float4(base + (e + s[q].x), base + (e + s[q].y), base + (e + s[q].z), base + (e + s[q].w));
    if (r + 3 < n) {
      *reinterpret_cast<float4*>(p + r) = x[q];
      *reinterpret_cast<float4*>(cdf + r) = c;
    } else {
      if (r < n) { p[r] = x[q].x; cdf[r] = c.x; }
      if (r + 1 < n) { p[r + 1] = x[q].y; cdf[r + 1] = c.y; }
      if (r + 2 < n) { p[r + 2] = x[q].z; cdf[r + 2] = c.z; }
    }
  }
}

__global__ void __launch_bounds__(kScanThreads) k_per_scan(const float* __restrict__ prio, int64_t n, float alpha,
                                                           const float* __restrict__ chunk, float* __restrict__ p,
                                                           float* __restrict__ cdf) {
  __shared__ float lds[kScanThreads / 64];
  __shared__ float lds2[kScanThreads / 64];
  // thread t's totals t, t + 256, ... in order, four loads at a time (the
  // missing ones 0: adding +0 to a sum of non-negative terms changes nothing)
  float b = 0.0f;
  for (int64_t c0 = threadIdx.x; c0 < (int64_t)blockIdx.x; c0 += 4 * kScanThreads) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t c = c0 + q * kScanThreads;
      v[q] = c < (int64_t)blockIdx.x ? chunk[c] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) b += v[q];
  }
  float4 x[kScanQuads], s[kScanQuads];
  const int64_t r0 = (int64_t)blockIdx.x * kScanChunk + kScanRows * (int64_t)threadIdx.x;
  const float t = per_pow(prio, n, r0, alpha, x, s);
  float all;
  const float e = per_block_excl(t, lds, all);
  per_store(p, cdf, n, r0, x, s, per_base(b, lds2), e);
}

// the batch max of w (one block, in LDS), every w normalised by it, then
// beta and the counter stepped
__global__ void __launch_bounds__(1024) k_per_finish(int batch, int64_t* __restrict__ counter,
                                                     double* __restrict__ beta, double beta_inc,
                                                     float* __restrict__ w_out) {
  __shared__ float red[16];
  float m = 0.0f;
  for (int i = threadIdx.x; i < batch; i += 1024) m = fmaxf(m, w_out[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float wmax = red[0];
#pragma unroll
  for (int q = 1; q < 16; ++q) wmax = fmaxf(wmax, red[q]);
  for (int i = threadIdx.x; i < batch; i += 1024) w_out[i] = w_out[i] / wmax;
  if (threadIdx.x == 0) {
    const double b = *beta + beta_inc;
    *beta = b < 1.0 ? b : 1.0;
    *counter += 1;
  }
}

// ------------------------------------------------------------- minibatch rows
// row k's next observation is row (k + stride) % cap of the same ring (the
// step after k's writes B = stride rows further on; DeviceReplay in dqn.py)
__global__ void __launch_bounds__(256) k_gather_batch(const int64_t* __restrict__ idx, int batch, int ss,
                                                      const float* __restrict__ obs, int64_t stride,
                                                      int64_t cap, const int64_t* __restrict__ action,
                                                      const float* __restrict__ reward,
                                                      const float* __restrict__ done, float* __restrict__ s,
                                                      float* __restrict__ ns, int64_t* __restrict__ a,
                                                      float* __restrict__ r, float* __restrict__ d) {
  const uint32_t e = blockIdx.x * 256u + threadIdx.x;
  if (e >= (uint32_t)batch * (uint32_t)ss) return;
  const int j = (int)(e / (uint32_t)ss);
  const int col = (int)(e - (uint32_t)j * (uint32_t)ss);
  const int64_t k = idx[j];
  int64_t kn = k + stride;
  if (kn >= cap) kn -= cap;
  s[e] = obs[k * ss + col];
  ns[e] = obs[kn * ss + col];
  if (col == 0) {
    a[2 * j] = action[2 * k];
    a[2 * j + 1] = action[2 * k + 1];
    r[j] = reward[k];
    d[j] = done[k];
  }
}

// ------------------------------------------------- target move-2 head max
// out[i] = max_c base[i][c] + tab[rows[i]][c] over the 576 codes: one wave
// per row (the same single fp32 add as the torch path, then max)
__global__ void __launch_bounds__(256) k_rowmax_addend(const float* __restrict__ base, int64_t ld,
                                                       const float* __restrict__ tab, int64_t ld_tab,
                                                       const int64_t* __restrict__ rows, int n,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= n) return;
  const float* br = base + (size_t)i * (size_t)ld;
  const int64_t ri = rows[i] < 0 ? 0 : (rows[i] > 575 ? 575 : rows[i]);  // a move-1 code: one table row each
  const float* tr = tab + (size_t)ri * (size_t)ld_tab;
  float m = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < 9; ++j) m = fmaxf(m, br[64 * j + lane] + tr[64 * j + lane]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) out[i] = m;
}

// The target heads' maxima in one launch (round 6): per row i (one wave),
// m1 = max_c nq1[i][c] and am1 = its argmax with torch.max(dim)'s rules (a
// NaN wins, ties go to the lowest code), then m2 = max_c base[i][c] +
// tab[am1][c] (k_rowmax_addend's sum) -- torch's max reduction and
// k_rowmax_addend were two launches.
__device__ __forceinline__ bool gt_or_nan(float a, int ia, float b, int ib) {
  if (a != a) return b != b ? ia < ib : true;
  if (b != b) return false;
  return a == b ? ia < ib : a > b;
}

__global__ void __launch_bounds__(256) k_target_max2(const float* __restrict__ nq1, int64_t ld1,
                                                     const float* __restrict__ base, int64_t ld,
                                                     const float* __restrict__ tab, int64_t ld_tab, int n,
                                                     float* __restrict__ m1, int64_t* __restrict__ am1,
                                                     float* __restrict__ m2) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= n) return;
  const float* qr = nq1 + (size_t)i * (size_t)ld1;
  float bv = qr[lane];
  int bi = lane;
#pragma unroll
  for (int j = 1; j < 9; ++j) {
    const float v = qr[64 * j + lane];
    if (gt_or_nan(v, 64 * j + lane, bv, bi)) { bv = v; bi = 64 * j + lane; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (gt_or_nan(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  const float* br = base + (size_t)i * (size_t)ld;
  const float* tr = tab + (size_t)bi * (size_t)ld_tab;
  float m = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < 9; ++j) m = fmaxf(m, br[64 * j + lane] + tr[64 * j + lane]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) {
    m1[i] = bv;
    if (am1) am1[i] = bi;
    m2[i] = m;
  }
}

// ------------------------------------------- the online heads, gathered
// The loss reads only q1_i = Q1[i][a1_i] and q2_i = Q2[i][a2_i] (the codes
// the replay stored), so the learner evaluates those entries instead of the
// two dense (batch x 256) x (256 x 576) heads, and backpropagates through
// them alone:
//   q1_i = f_i . W1[a1_i] + b1[a1_i]
//   q2_i = (f_i . W2[a2_i][:256] + b2[a2_i]) + W2[a2_i][256 + a1_i]
//          (DecomposedDQN.move2_from_features' order)
//   gf_i = g1_i W1[a1_i] + g2_i W2[a2_i][:256]
//   gW1[c] = sum over {i: a1_i = c} of g1_i f_i, gb1[c] = the sum of those g1_i
//   gW2[c][:256], gb2[c] likewise over {i: a2_i = c}, and
//   gW2[c][256 + k] = the sum of g2_i over {i: a2_i = c, a1_i = k}
// -- the gradient of the dense path (whose other entries get zero), each
// sum in a fixed order (deterministic).  Codes outside
// 0..575 are clamped (the ring only holds codes the policy produced).
constexpr int kHeadF = 256;   // feature width
constexpr int kCodes = 576;   // move codes
constexpr int kW2 = kHeadF + kCodes;

__device__ __forceinline__ int clamp_code(int64_t a) {
  return a < 0 ? 0 : (a >= kCodes ? kCodes - 1 : (int)a);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// q1, q2 of the batch rows: one wave per row, lane j holds features 4j..4j+3
__global__ void __launch_bounds__(256) k_heads_gather(const float* __restrict__ f, int64_t ldf,
                                                      const float* __restrict__ w1, int64_t ldw1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      int64_t ldw2, const float* __restrict__ b2,
                                                      const int64_t* __restrict__ a, int n,
                                                      float* __restrict__ q1, float* __restrict__ q2) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= n) return;
  const int c1 = clamp_code(a[2 * i]), c2 = clamp_code(a[2 * i + 1]);
  const float4 x = reinterpret_cast<const float4*>(f + (size_t)i * ldf)[lane];
  const float4 u = reinterpret_cast<const float4*>(w1 + (size_t)c1 * ldw1)[lane];
  const float4 v = reinterpret_cast<const float4*>(w2 + (size_t)c2 * ldw2)[lane];
  const float s1 = wave_sum(x.x * u.x + x.y * u.y + x.z * u.z + x.w * u.w);
  const float s2 = wave_sum(x.x * v.x + x.y * v.y + x.z * v.z + x.w * v.w);
  if (lane == 0) {
    q1[i] = s1 + b1[c1];
    q2[i] = (s2 + b2[c2]) + w2[(size_t)c2 * ldw2 + kHeadF + c1];
  }
}

// gf_i = g1_i W1[a1_i] + g2_i W2[a2_i][:256]: one wave per row
__global__ void __launch_bounds__(256) k_heads_grad_f(const float* __restrict__ g1, const float* __restrict__ g2,
                                                      const float* __restrict__ w1, int64_t ldw1,
                                                      const float* __restrict__ w2, int64_t ldw2,
                                                      const int64_t* __restrict__ a, int n,
                                                      float* __restrict__ gf) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= n) return;
  const int c1 = clamp_code(a[2 * i]), c2 = clamp_code(a[2 * i + 1]);
  const float4 u = reinterpret_cast<const float4*>(w1 + (size_t)c1 * ldw1)[lane];
  const float4 v = reinterpret_cast<const float4*>(w2 + (size_t)c2 * ldw2)[lane];
  const float s = g1[i], t = g2[i];
  reinterpret_cast<float4*>(gf + (size_t)i * kHeadF)[lane] =
      make_float4(s * u.x + t * v.x, s * u.y + t * v.y, s * u.z + t * v.z, s * u.w + t * v.w);
}

// gW1 / gb1 (blocks 0..575) and gW2 / gb2 (blocks 576..1151), one code per
// block of 16 waves.  Rows go in passes of 4,096, wave w taking rows 256w ..
// 256w + 255 of each: every lane loads the code, gradient and move-1 code of
// its 4 rows up front; per 64-row chunk a ballot marks the rows holding this
// code, and the wave adds them in ascending order -- lane l the feature
// columns 4l..4l+3 (one 16-byte load of each row, up to 4 rows' loads in
// flight), and for head 2 the one-hot columns l + 64j, the gradient and code
// taken from the owning lane (v_readlane).  At the end the 16 waves' partial
// sums are added in wave order.  A fixed order for given (n, codes):
// deterministic.  Every element of the block's gradient rows is written (zero
// where no row holds the code).  Measured at B = 4,096 (config 4): one
// thread per column over one LDS-staged row list, 157 us (a popular code's
// list -- hundreds of rows -- was one serial chain of loads); that list split
// over 8 waves, 38.6 us (the staging loop and the single-wave list build
// were latency-serialised per block); this form: see DESIGN.md section 11
// (8 waves of 8 chunks: the same at uniform codes, 20 % slower when one
// code holds a quarter of the rows; 8 row loads in flight: 10 % slower).
constexpr int kGwThreads = 1024;
constexpr int kGwWaves = kGwThreads / 64;
constexpr int kGwChunks = 4;                         // 64-row chunks per wave per pass
constexpr int kGwPass = kGwWaves * kGwChunks * 64;   // rows per pass
constexpr int kGwBatch = 4;                          // row loads in flight per wave

struct GwSums {  // the waves' partial sums
  float4 f[kGwWaves][64];
  float oh[kGwWaves][kCodes];
  float b[kGwWaves];
};

__global__ void __launch_bounds__(kGwThreads) k_heads_grad_w(const float* __restrict__ g1,
                                                             const float* __restrict__ g2,
                                                             const float* __restrict__ f, int64_t ldf,
                                                             const int64_t* __restrict__ a, int n,
                                                             float* __restrict__ gw1, float* __restrict__ gb1,
                                                             float* __restrict__ gw2, float* __restrict__ gb2) {
#pragma clang fp contract(off)
  __shared__ GwSums L;
  const int head = blockIdx.x >= kCodes ? 1 : 0;
  const int c = (int)blockIdx.x - head * kCodes;
  const float* __restrict__ g = head ? g2 : g1;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float oh[kCodes / 64];
#pragma unroll
  for (int j = 0; j < kCodes / 64; ++j) oh[j] = 0.0f;
  float gs = 0.0f;
  for (int base = 0; base < n; base += kGwPass) {
    const int r0 = base + wave * kGwChunks * 64;
    int code[kGwChunks], code1[kGwChunks];
    float gv[kGwChunks];
#pragma unroll
    for (int q = 0; q < kGwChunks; ++q) {
      const int r = r0 + q * 64 + lane;
      const bool ok = r < n;
      const int64_t* ar = a + 2 * (size_t)(ok ? r : 0);
      code[q] = ok ? clamp_code(ar[head]) : -1;
      code1[q] = clamp_code(ar[0]);
      gv[q] = ok ? g[r] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < kGwChunks; ++q) {
      uint64_t mask = __ballot(code[q] == c);
      const float* fq = f + (size_t)(r0 + q * 64) * ldf;
      while (mask) {  // wave-uniform
        int bb[kGwBatch];
#pragma unroll
        for (int u = 0; u < kGwBatch; ++u) {
          bb[u] = mask ? __builtin_ctzll(mask) : -1;
          mask &= mask - 1;
        }
        float4 v[kGwBatch];
#pragma unroll
        for (int u = 0; u < kGwBatch; ++u)
          if (bb[u] >= 0) v[u] = reinterpret_cast<const float4*>(fq + (size_t)bb[u] * ldf)[lane];
#pragma unroll
        for (int u = 0; u < kGwBatch; ++u) {
          if (bb[u] < 0) break;
          const float gi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gv[q]), bb[u]));
          acc.x += gi * v[u].x;
          acc.y += gi * v[u].y;
          acc.z += gi * v[u].z;
          acc.w += gi * v[u].w;
          gs += gi;
          if (head) {  // the one-hot column of the row's move-1 code
            const int k1 = __builtin_amdgcn_readlane(code1[q], bb[u]);
            const bool mine = (k1 & 63) == lane;
#pragma unroll
            for (int j = 0; j < kCodes / 64; ++j) oh[j] += mine && (k1 >> 6) == j ? gi : 0.0f;
          }
        }
      }
    }
  }
  L.f[wave][lane] = acc;
  if (head) {
#pragma unroll
    for (int q = 0; q < kCodes / 64; ++q) L.oh[wave][lane + 64 * q] = oh[q];
  }
  if (lane == 0) L.b[wave] = gs;
  __syncthreads();
  if (t < kHeadF) {
    const float* fs = reinterpret_cast<const float*>(&L.f[0][0]);
    float x = 0.0f;
#pragma unroll
    for (int w = 0; w < kGwWaves; ++w) x += fs[w * kHeadF + t];
    (head ? gw2 + (size_t)c * kW2 : gw1 + (size_t)c * kHeadF)[t] = x;
  }
  if (head) {
    for (int col = t; col < kCodes; col += kGwThreads) {
      float x = 0.0f;
#pragma unroll
      for (int w = 0; w < kGwWaves; ++w) x += L.oh[w][col];
      gw2[(size_t)c * kW2 + kHeadF + col] = x;
    }
  }
  if (t == 0) {
    float x = 0.0f;
#pragma unroll
    for (int w = 0; w < kGwWaves; ++w) x += L.b[w];
    (head ? gb2 : gb1)[c] = x;
  }
}

// ------------------------------------- ReLU backward + the bias gradient
// For a layer h = relu(x W^T + b) with upstream gradient gh (n x cols):
// g = gh * (h > 0) (what autograd's threshold_backward gives) and db[c] =
// sum over rows of g[.][c] -- the two kernels autograd runs after every
// Linear + ReLU of the learner's feature layers (torch's column reduction
// took 14 us per 4,096 x 256 layer).  k_relu_grad_partial: blocks of 64
// rows x 64 columns, 4 waves of 16 rows each (lane = column: every row's 64
// columns one coalesced 256-byte access; all 16 rows' loads issued before
// the first use), each block's column sums (its rows in order, then the
// waves in order) to partial[slice][col]; k_bias_grad_sum adds the slices
// in order, 4 threads per column over a quarter of them each, then the
// quarters in order: deterministic.  Measured per 4,096 x 256 layer: one
// kernel whose last block added the slices behind a ticket, 35 us (each
// block's device-scope fence writes back its XCD's L2, full of the g rows
// just stored); a lane per column over 128-row slices, 12.7 + 4.5 us; 16
// rows x 4 columns per lane over 64-row slices (64 blocks), 8.5 + 4.5 us.
constexpr int kRbRows = 64;
constexpr int kRbWaveRows = kRbRows / 4;

__global__ void __launch_bounds__(256) k_relu_grad_partial(const float* __restrict__ gh,
                                                           const float* __restrict__ h, int n, int cols,
                                                           float* __restrict__ g, float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane, slice = blockIdx.y;
  const bool okc = col < cols;
  const int r0 = slice * kRbRows + wave * kRbWaveRows;
  float acc = 0.0f;
  if (okc) {
    float a[kRbWaveRows], m[kRbWaveRows];
#pragma unroll
    for (int k = 0; k < kRbWaveRows; ++k) {
      const int r = r0 + k;
      a[k] = r < n ? gh[(size_t)r * cols + col] : 0.0f;
      m[k] = r < n ? h[(size_t)r * cols + col] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < kRbWaveRows; ++k) {
      const int r = r0 + k;
      const float v = m[k] > 0.0f ? a[k] : 0.0f;
      if (r < n) g[(size_t)r * cols + col] = v;
      acc += v;
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && okc) partial[(size_t)slice * cols + col] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// db[col] = the slices' partial sums of col in slice order; block of 256
// threads = 64 columns x 4 quarters of the slices
__global__ void __launch_bounds__(256) k_bias_grad_sum(const float* __restrict__ partial, int slices, int cols,
                                                       float* __restrict__ db) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, qtr = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int q0 = slices * qtr / 4, q1 = slices * (qtr + 1) / 4;
  float s = 0.0f;
  if (col < cols) {
#pragma unroll 8
    for (int q = q0; q < q1; ++q) s += partial[(size_t)q * cols + col];
  }
  red[qtr][lane] = s;
  __syncthreads();
  if (qtr == 0 && col < cols) db[col] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// --------------------------------------------------------------- the loss
// t1 = r + (1 - d) * gamma * m1, t2 likewise (m = the target heads' maxima);
// td = clamp(|t1 - q1| + |t2 - q2|, 0, 100); loss = mean(w (q1 - t1)^2) +
// mean(w (q2 - t2)^2); g = dloss/dq = (1/B) * w * (2 (q - t)) in torch's
// autograd order.  Each fp32 operation rounds on its own, as torch's
// elementwise kernels do (no contraction).
__global__ void __launch_bounds__(kLearnThreads) k_dqn_loss(const float* __restrict__ q1,
                                                            const float* __restrict__ q2,
                                                            const float* __restrict__ m1,
                                                            const float* __restrict__ m2,
                                                            const float* __restrict__ r,
                                                            const float* __restrict__ d,
                                                            const float* __restrict__ w, int batch,
                                                            float gamma, float* __restrict__ td,
                                                            float* __restrict__ loss,
                                                            float* __restrict__ loss_copy,
                                                            float* __restrict__ g1, float* __restrict__ g2) {
#pragma clang fp contract(off)
  __shared__ float red[kLearnThreads / 64];
  const float inv_b = 1.0f / (float)batch;
  float s1 = 0.0f, s2 = 0.0f;
  for (int j = threadIdx.x; j < batch; j += kLearnThreads) {
    const float nd = (1.0f - d[j]) * gamma;
    const float t1 = r[j] + nd * m1[j];
    const float t2 = r[j] + nd * m2[j];
    const float e1 = q1[j] - t1, e2 = q2[j] - t2;
    const float a = fabsf(t1 - q1[j]) + fabsf(t2 - q2[j]);
    td[j] = fminf(fmaxf(a, 0.0f), 100.0f);
    s1 += w[j] * (e1 * e1);
    s2 += w[j] * (e2 * e2);
    const float gw = inv_b * w[j];
    g1[j] = gw * (2.0f * e1);
    g2[j] = gw * (2.0f * e2);
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) {
    const float l = s1 / (float)batch + s2 / (float)batch;
    *loss = l;
    if (loss_copy) *loss_copy = l;
  }
}

// ------------------------------------------------------ priorities, epsilon
// prio[idx_j] = td_j + eps; max_prio = max(max_prio, max_j prio); then
// epsilon <- epsilon * decay if epsilon > eps_min (one decay per update)
__global__ void __launch_bounds__(kLearnThreads) k_prio_update(const int64_t* __restrict__ idx,
                                                               const float* __restrict__ td, int batch,
                                                               float eps, float* __restrict__ prio,
                                                               float* __restrict__ max_prio,
                                                               float* __restrict__ epsilon, float eps_min,
                                                               float eps_decay, int64_t* __restrict__ cursor,
                                                               int64_t cursor_add, int64_t cursor_mod,
                                                               int64_t* __restrict__ tag) {
  __shared__ float red[kLearnThreads / 64];
  float m = -__builtin_inff();
  for (int j = threadIdx.x; j < batch; j += kLearnThreads) {
    const float pr = td[j] + eps;
    prio[idx[j]] = pr;
    m = fmaxf(m, pr);
  }
  m = block_max(m, red);
  if (threadIdx.x == 0) {
    *max_prio = fmaxf(*max_prio, m);
    if (epsilon) {
      const float e = *epsilon;
      *epsilon = e > eps_min ? e * eps_decay : e;
    }
    // the driver's step bookkeeping, folded in (two torch launches fewer)
    if (cursor) *cursor = (*cursor + cursor_add) % cursor_mod;
    if (tag) *tag += 1;
  }
}

// k_per_finish, k_dqn_loss and k_prio_update in one block (round 6; the
// three were one-block kernels back to back): the batch max of the raw
// importance weights (k_per_sample_gather's) and w_j / max written back to
// w; the loss, td and dloss/dq exactly as k_dqn_loss; then the priorities,
// the running max priority, epsilon, the write cursor and the step tag as
// k_prio_update, and beta / the sampling counter as k_per_finish.  The
// priorities move before the backward and Adam: nothing between reads them
// (the next step's sample does).
__global__ void __launch_bounds__(kLearnThreads) k_dqn_loss_prio(
    const float* __restrict__ q1, const float* __restrict__ q2, const float* __restrict__ m1,
    const float* __restrict__ m2, const float* __restrict__ r, const float* __restrict__ d, float* __restrict__ w,
    int batch, float gamma, float* __restrict__ td, float* __restrict__ loss, float* __restrict__ loss_copy,
    float* __restrict__ g1, float* __restrict__ g2, const int64_t* __restrict__ idx, float eps,
    float* __restrict__ prio, float* __restrict__ max_prio, float* __restrict__ epsilon, float eps_min,
    float eps_decay, int64_t* __restrict__ cursor, int64_t cursor_add, int64_t cursor_mod, int64_t* __restrict__ tag,
    int64_t* __restrict__ counter, double* __restrict__ beta, double beta_inc) {
#pragma clang fp contract(off)
  __shared__ float red[kLearnThreads / 64];
  __shared__ float red3[3][kLearnThreads / 64];
  // the device scalars first: their loads overlap the batch's (thread 0)
  float mp0 = 0.0f, e0 = 0.0f;
  int64_t cur0 = 0, tag0 = 0, ctr0 = 0;
  double beta0 = 0.0;
  if (threadIdx.x == 0) {
    mp0 = *max_prio;
    if (epsilon) e0 = *epsilon;
    if (cursor) cur0 = *cursor;
    if (tag) tag0 = *tag;
    beta0 = *beta;
    ctr0 = *counter;
  }
  // the first kLossCache rows of each thread in registers, loaded with w
  // (one memory round trip for both passes; larger batches read the rest
  // in the second pass)
  constexpr int kLossCache = 4;
  float cw[kLossCache], cd[kLossCache], cr[kLossCache], cm1[kLossCache], cm2[kLossCache], cq1[kLossCache],
      cq2[kLossCache];
  int64_t ci[kLossCache];
  // k_per_finish: the batch max (from 0, as there), then every w normalised
  float wm = 0.0f;
#pragma unroll
  for (int c = 0; c < kLossCache; ++c) {
    const int j = threadIdx.x + c * kLearnThreads;
    if (j < batch) {
      cw[c] = w[j];
      cd[c] = d[j];
      cr[c] = r[j];
      cm1[c] = m1[j];
      cm2[c] = m2[j];
      cq1[c] = q1[j];
      cq2[c] = q2[j];
      ci[c] = idx[j];
      wm = fmaxf(wm, cw[c]);
    }
  }
  for (int j = threadIdx.x + kLossCache * kLearnThreads; j < batch; j += kLearnThreads) wm = fmaxf(wm, w[j]);
  const float wmax = block_max(wm, red);
  const float inv_b = 1.0f / (float)batch;
  float s1 = 0.0f, s2 = 0.0f, pm = -__builtin_inff();
  for (int j = threadIdx.x, c = 0; j < batch; j += kLearnThreads, ++c) {
    const bool hit = c < kLossCache;
    const float wr = hit ? cw[c] : w[j], dj = hit ? cd[c] : d[j], rj = hit ? cr[c] : r[j];
    const float m1j = hit ? cm1[c] : m1[j], m2j = hit ? cm2[c] : m2[j];
    const float q1j = hit ? cq1[c] : q1[j], q2j = hit ? cq2[c] : q2[j];
    const int64_t ij = hit ? ci[c] : idx[j];
    const float wj = wr / wmax;
    w[j] = wj;
    const float nd = (1.0f - dj) * gamma;
    const float t1 = rj + nd * m1j;
    const float t2 = rj + nd * m2j;
    const float e1 = q1j - t1, e2 = q2j - t2;
    const float a = fabsf(t1 - q1j) + fabsf(t2 - q2j);
    const float tdj = fminf(fmaxf(a, 0.0f), 100.0f);
    td[j] = tdj;
    s1 += wj * (e1 * e1);
    s2 += wj * (e2 * e2);
    const float gw = inv_b * wj;
    g1[j] = gw * (2.0f * e1);
    g2[j] = gw * (2.0f * e2);
    const float pr = tdj + eps;
    prio[ij] = pr;
    pm = fmaxf(pm, pr);
  }
  // block_sum(s1), block_sum(s2), block_max(pm) -- the same trees -- in one
  // pass of barriers
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
    pm = fmaxf(pm, __shfl_xor(pm, o, 64));
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red3[0][wave] = s1;
    red3[1][wave] = s2;
    red3[2][wave] = pm;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    s1 = lane < kLearnThreads / 64 ? red3[0][lane] : 0.0f;
    s2 = lane < kLearnThreads / 64 ? red3[1][lane] : 0.0f;
    pm = lane < kLearnThreads / 64 ? red3[2][lane] : -__builtin_inff();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
      pm = fmaxf(pm, __shfl_xor(pm, o, 64));
    }
  }
  if (threadIdx.x == 0) {
    const float l = s1 / (float)batch + s2 / (float)batch;
    *loss = l;
    if (loss_copy) *loss_copy = l;
    *max_prio = fmaxf(mp0, pm);
    if (epsilon) *epsilon = e0 > eps_min ? e0 * eps_decay : e0;
    if (cursor) *cursor = (cur0 + cursor_add) % cursor_mod;
    if (tag) *tag = tag0 + 1;
    const double b = beta0 + beta_inc;
    *beta = b < 1.0 ? b : 1.0;
    *counter = ctr0 + 1;
  }
}

// ------------------------------------------------ grad clip + Adam, fused
// clip_grad_norm_(max_norm) followed by Adam (torch.optim.Adam's update:
// m <- lerp(m, g, 1 - b1), v <- b2 v + (1 - b2) g^2, p -= lr / bc1 * m /
// (sqrt(v) / sqrt(bc2) + eps)) over up to 8 parameter tensors, in two
// kernels with enough blocks to fill the chip (torch's multi-tensor kernels
// run one block per 64 K-element chunk: ~12 blocks for this network).
constexpr int kMaxTensors = 8;
constexpr int kNormBlocks = 1024;

struct ParamTable {
  float* p[kMaxTensors];
  const float* g[kMaxTensors];
  float* m[kMaxTensors];
  float* v[kMaxTensors];
  int64_t off[kMaxTensors + 1];  // prefix sums of the sizes
  int count;
};

__device__ __forceinline__ int tensor_of(const ParamTable& t, int64_t e) {
  int k = 0;
#pragma unroll
  for (int j = 1; j < kMaxTensors; ++j) k += (j < t.count && e >= t.off[j]) ? 1 : 0;
  return k;
}

// pass 1: sum of g^2 per block -> partial[]; block 0 advances the Adam step
// (pass 2 reads it after the kernel boundary).  (Before, the last block to
// finish added the partials behind a ticket and a device-scope fence per
// block: 15.7 + 9.6 us for the two passes at config 4, now 11.1 + 11.1.)
__global__ void __launch_bounds__(256) k_grad_sqnorm(ParamTable t, float* __restrict__ partial,
                                                     int64_t* __restrict__ step) {
  __shared__ float red[4];
  const int64_t total = t.off[t.count];
  float acc = 0.0f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int k = tensor_of(t, e);
    const float g = t.g[k][e - t.off[k]];
    acc += g * g;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    if (blockIdx.x == 0) *step += 1;
  }
}

// pass 2: every block adds the nb partials in the same fixed order (the same
// bits in every block), forms the clip coefficient min(1, max_norm / (norm +
// 1e-6)), then the Adam update of its elements with the clipped gradient
__global__ void __launch_bounds__(256) k_adam(ParamTable t, const float* __restrict__ partial, int nb,
                                              float max_norm, const int64_t* __restrict__ step, float lr, float b1,
                                              float b2, float eps) {
  __shared__ float sc[3];
  __shared__ float red[4];
  float s = 0.0f;
  for (int b = threadIdx.x; b < nb; b += 256) s += partial[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float c = max_norm / (norm + 1e-6f);
    const float st = (float)*step;
    const float bc1 = 1.0f - powf(b1, st), bc2 = 1.0f - powf(b2, st);
    sc[0] = lr / bc1;
    sc[1] = sqrtf(bc2);
    sc[2] = c < 1.0f ? c : 1.0f;
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= t.off[t.count]) return;
  const int k = tensor_of(t, e);
  const int64_t i = e - t.off[k];
  const float g = t.g[k][i] * sc[2];
  float m = t.m[k][i], v = t.v[k][i];
  m = m + (1.0f - b1) * (g - m);
  v = b2 * v + (1.0f - b2) * (g * g);
  t.m[k][i] = m;
  t.v[k][i] = v;
  t.p[k][i] -= sc[0] * m / (sqrtf(v) / sc[1] + eps);
}

// The same two passes over float4s (round 6), when every tensor's size is a
// multiple of 4 and every pointer 16-byte aligned: one 16-byte load per
// thread and operand instead of a loop of dependent 4-byte loads (k_grad_sqnorm
// ran ~16 per thread, each an L2 round trip: 11.4 us; k_adam 11.5 us, 2,900
// blocks each adding the partials first).  A float4 never spans two tensors.
__global__ void __launch_bounds__(256) k_grad_sqnorm4(ParamTable t, float* __restrict__ partial,
                                                      int64_t* __restrict__ step) {
  __shared__ float red[4];
  const int64_t total4 = t.off[t.count] >> 2;
  float acc = 0.0f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total4; e += (int64_t)gridDim.x * 256) {
    const int k = tensor_of(t, 4 * e);
    const float4 g = reinterpret_cast<const float4*>(t.g[k] + (4 * e - t.off[k]))[0];
    acc += ((g.x * g.x + g.y * g.y) + g.z * g.z) + g.w * g.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    if (blockIdx.x == 0) *step += 1;
  }
}

__global__ void __launch_bounds__(256) k_adam4(ParamTable t, const float* __restrict__ partial, int nb,
                                               float max_norm, const int64_t* __restrict__ step, float lr, float b1,
                                               float b2, float eps) {
  __shared__ float sc[3];
  __shared__ float red[4];
  float s = 0.0f;
  for (int b = threadIdx.x; b < nb; b += 256) s += partial[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float c = max_norm / (norm + 1e-6f);
    const float st = (float)*step;
    const float bc1 = 1.0f - powf(b1, st), bc2 = 1.0f - powf(b2, st);
    sc[0] = lr / bc1;
    sc[1] = sqrtf(bc2);
    sc[2] = c < 1.0f ? c : 1.0f;
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (4 * e >= t.off[t.count]) return;
  const int k = tensor_of(t, 4 * e);
  const int64_t i = 4 * e - t.off[k];
  const float4 g4 = reinterpret_cast<const float4*>(t.g[k] + i)[0];
  float4 m4 = reinterpret_cast<const float4*>(t.m[k] + i)[0];
  float4 v4 = reinterpret_cast<const float4*>(t.v[k] + i)[0];
  float4 p4 = reinterpret_cast<const float4*>(t.p[k] + i)[0];
  float* gp = &m4.x;
  float* vp = &v4.x;
  float* pp = &p4.x;
  const float* gg = &g4.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float g = gg[q] * sc[2];
    float m = gp[q], v = vp[q];
    m = m + (1.0f - b1) * (g - m);
    v = b2 * v + (1.0f - b2) * (g * g);
    gp[q] = m;
    vp[q] = v;
    pp[q] -= sc[0] * m / (sqrtf(v) / sc[1] + eps);
  }
  reinterpret_cast<float4*>(t.m[k] + i)[0] = m4;
  reinterpret_cast<float4*>(t.v[k] + i)[0] = v4;
  reinterpret_cast<float4*>(t.p[k] + i)[0] = p4;
}

}  // namespace

// narde_adam_clip's form: float4 passes (default) or round 5's scalar ones
// (narde_learner_variant, for A/B timing)
static bool adam_vec4 = true;

extern "C" {

int narde_per_sample(int device, const float* p, const float* cdf, int64_t n, int64_t batch, uint64_t seed,
                     int64_t* counter, double* beta, double beta_inc, int64_t* idx, float* w, float* u,
                     uint32_t* scratch, void* stream) {
  if (!p || !cdf || !counter || !beta || !idx || !w) return bad("NULL argument");
  if (n <= 0 || batch <= 0 || batch > (int64_t(1) << 24)) return bad("need n > 0 and 0 < batch <= 2^24");
  DeviceGuard dg(device);
  const unsigned blocks = (unsigned)((batch + kSampleWaves - 1) / kSampleWaves);
  k_per_sample<<<blocks, 64 * kSampleWaves, 0, (hipStream_t)stream>>>(p, cdf, n, (int)batch, (uint32_t)seed,
                                                                      (uint32_t)(seed >> 32), counter, beta, idx, w, u);
  const int rc = check_launch("k_per_sample");
  if (rc != NARDE_OK) return rc;
  k_per_finish<<<1, 1024, 0, (hipStream_t)stream>>>((int)batch, counter, beta, beta_inc, w);
  return check_launch("k_per_finish");
}

int narde_per_prefix(int device, const float* prio, int64_t n, double alpha, float* p, float* cdf, float* chunk,
                     int64_t chunks, void* stream) {
  if (!prio || !p || !cdf || !chunk) return bad("NULL argument");
  if (n <= 0 || n > (int64_t(1) << 31) - kScanChunk) return bad("need 0 < n < 2^31 - 1024");
  if ((((uintptr_t)prio | (uintptr_t)p | (uintptr_t)cdf) & 15u) != 0u) return bad("prio, p and cdf must be 16-byte aligned");
  const int64_t blocks64 = (n + kScanChunk - 1) / kScanChunk;
  if (chunks < blocks64) return bad("chunk holds fewer totals than n needs");
  DeviceGuard dg(device);
  const unsigned blocks = (unsigned)blocks64;
  k_per_chunk_sums<<<blocks, kScanThreads, 0, (hipStream_t)stream>>>(prio, n, (float)alpha, chunk);
  const int rc = check_launch("k_per_chunk_sums");
  if (rc != NARDE_OK) return rc;
  k_per_scan<<<blocks, kScanThreads, 0, (hipStream_t)stream>>>(prio, n, (float)alpha, chunk, p, cdf);
  return check_launch("k_per_scan");
}

int narde_gather_batch(int device, const int64_t* idx, int64_t batch, int state_size, const float* obs,
                       int64_t next_stride, int64_t capacity, const int64_t* action, const float* reward,
                       const float* done, float* s, float* ns, int64_t* a, float* r, float* d, void* stream) {
  if (!idx || !obs || !action || !reward || !done || !s || !ns || !a || !r || !d)
    return bad("NULL argument");
  if (batch <= 0 || state_size <= 0 || batch * state_size >= (int64_t(1) << 31)) return bad("bad sizes");
  if (capacity <= 0 || next_stride < 0 || next_stride >= capacity) return bad("bad ring geometry");
  DeviceGuard dg(device);
  const int64_t total = batch * state_size;
  k_gather_batch<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      idx, (int)batch, state_size, obs, next_stride, capacity, action, reward, done, s, ns, a, r, d);
  return check_launch("k_gather_batch");
}

int narde_rowmax_addend(int device, const float* base, int64_t ld, const float* tab, int64_t ld_tab,
                        const int64_t* rows, int64_t n, float* out, void* stream) {
  if (!base || !tab || !rows || !out) return bad("NULL argument");
  if (n < 0 || n > (int64_t(1) << 31) - 4 || ld < 576 || ld_tab < 576) return bad("bad sizes");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_rowmax_addend<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(base, ld, tab, ld_tab, rows, (int)n,
                                                                            out);
  return check_launch("k_rowmax_addend");
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0u; }

int narde_dqn_heads_forward(int device, const float* f, int64_t ldf, const float* w1, int64_t ldw1,
                            const float* b1, const float* w2, int64_t ldw2, const float* b2, const int64_t* a,
                            int64_t n, float* q1, float* q2, void* stream) {
  if (!f || !w1 || !b1 || !w2 || !b2 || !a || !q1 || !q2) return bad("NULL argument");
  if (n < 0 || n > (int64_t(1) << 31) - 4) return bad("bad batch");
  if (ldf < kHeadF || ldw1 < kHeadF || ldw2 < kW2 || (ldf | ldw1 | ldw2) & 3) return bad("bad leading dimensions");
  if (!aligned16(f) || !aligned16(w1) || !aligned16(w2)) return bad("f / w1 / w2 must be 16-byte aligned");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_heads_gather<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(f, ldf, w1, ldw1, b1, w2, ldw2, b2, a,
                                                                           (int)n, q1, q2);
  return check_launch("k_heads_gather");
}

int narde_dqn_heads_backward(int device, const float* g1, const float* g2, const float* f, int64_t ldf,
                             const float* w1, int64_t ldw1, const float* w2, int64_t ldw2, const int64_t* a,
                             int64_t n, float* gf, float* gw1, float* gb1, float* gw2, float* gb2, void* stream) {
  if (!g1 || !g2 || !f || !w1 || !w2 || !a || !gf || !gw1 || !gb1 || !gw2 || !gb2) return bad("NULL argument");
  if (n < 0 || n > (int64_t(1) << 31) - 4) return bad("bad batch");
  if (ldf < kHeadF || ldw1 < kHeadF || ldw2 < kW2 || (ldw1 | ldw2) & 3) return bad("bad leading dimensions");
  if (!aligned16(w1) || !aligned16(w2) || !aligned16(gf)) return bad("w1 / w2 / gf must be 16-byte aligned");
  DeviceGuard dg(device);
  if (n > 0) {
    k_heads_grad_f<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(g1, g2, w1, ldw1, w2, ldw2, a, (int)n,
                                                                             gf);
    const int rc = check_launch("k_heads_grad_f");
    if (rc != NARDE_OK) return rc;
  }
  k_heads_grad_w<<<2 * kCodes, kGwThreads, 0, (hipStream_t)stream>>>(g1, g2, f, ldf, a, (int)n, gw1, gb1, gw2, gb2);
  return check_launch("k_heads_grad_w");
}


int narde_relu_bias_grad(int device, const float* gh, const float* h, int64_t n, int64_t cols, float* g,
                         float* db, float* scratch, void* stream) {
  if (!gh || !h || !g || !db || !scratch) return bad("NULL argument");
  if (n <= 0 || cols <= 0 || cols > 4096 || n * cols >= (int64_t(1) << 31)) return bad("bad sizes");
  DeviceGuard dg(device);
  const int slices = (int)((n + kRbRows - 1) / kRbRows);
  // scratch: slices x cols partial sums
  const unsigned groups = (unsigned)((cols + 63) / 64);
  k_relu_grad_partial<<<dim3(groups, (unsigned)slices), 256, 0, (hipStream_t)stream>>>(gh, h, (int)n, (int)cols, g,
                                                                                     scratch);
  const int rc = check_launch("k_relu_grad_partial");
  if (rc != NARDE_OK) return rc;
  k_bias_grad_sum<<<groups, 256, 0, (hipStream_t)stream>>>(scratch, slices, (int)cols, db);
  return check_launch("k_bias_grad_sum");
}

int narde_dqn_loss(int device, const float* q1, const float* q2, const float* m1, const float* m2, const float* r,
                   const float* d, const float* w, int64_t batch, float gamma, float* td, float* loss,
                   float* loss_copy, float* g1, float* g2, void* stream) {
  if (!q1 || !q2 || !m1 || !m2 || !r || !d || !w || !td || !loss || !g1 || !g2) return bad("NULL argument");
  if (batch <= 0 || batch > (int64_t(1) << 24)) return bad("bad batch");
  DeviceGuard dg(device);
  k_dqn_loss<<<1, kLearnThreads, 0, (hipStream_t)stream>>>(q1, q2, m1, m2, r, d, w, (int)batch, gamma, td, loss,
                                                           loss_copy, g1, g2);
  return check_launch("k_dqn_loss");
}

int narde_prio_update(int device, const int64_t* idx, const float* td, int64_t batch, float eps, float* prio,
                      float* max_prio, float* epsilon, float eps_min, float eps_decay, int64_t* cursor,
                      int64_t cursor_add, int64_t cursor_mod, int64_t* tag, void* stream) {
  if (!idx || !td || !prio || !max_prio) return bad("NULL argument");
  if (batch <= 0 || batch > (int64_t(1) << 24)) return bad("bad batch");
  if (cursor && (cursor_mod <= 0 || cursor_add < 0)) return bad("bad cursor step");
  DeviceGuard dg(device);
  k_prio_update<<<1, kLearnThreads, 0, (hipStream_t)stream>>>(idx, td, (int)batch, eps, prio, max_prio, epsilon,
                                                              eps_min, eps_decay, cursor, cursor_add, cursor_mod,
                                                              tag);
  return check_launch("k_prio_update");
}


int narde_adam_clip(int device, int n_tensors, float* const* params, const float* const* grads, float* const* m,
                    float* const* v, const int64_t* sizes, int64_t* step, float lr, float beta1, float beta2,
                    float eps, float max_norm, float* scratch, void* stream) {
  if (n_tensors <= 0 || n_tensors > kMaxTensors) return bad("1..8 tensors");
  if (!params || !grads || !m || !v || !sizes || !step || !scratch) return bad("NULL argument");
  ParamTable t{};
  t.count = n_tensors;
  t.off[0] = 0;
  for (int k = 0; k < n_tensors; ++k) {
    if (!params[k] || !grads[k] || !m[k] || !v[k] || sizes[k] <= 0) return bad("bad tensor");
    t.p[k] = params[k];
    t.g[k] = grads[k];
    t.m[k] = m[k];
    t.v[k] = v[k];
    t.off[k + 1] = t.off[k] + sizes[k];
  }
  for (int k = n_tensors; k < kMaxTensors; ++k) t.off[k + 1] = t.off[n_tensors];
  const int64_t total = t.off[n_tensors];
  if (total >= (int64_t(1) << 31)) return bad("too many parameters");
  // scratch: kNormBlocks partial sums (the words after them are unused)
  float* partial = scratch;
  DeviceGuard dg(device);
  bool vec = adam_vec4;
  for (int k = 0; k < n_tensors && vec; ++k)
    vec = sizes[k] % 4 == 0 && aligned16(params[k]) && aligned16(grads[k]) && aligned16(m[k]) && aligned16(v[k]);
  if (vec) {  // one float4 per thread (round 6)
    const int64_t total4 = total / 4;
    int nb4 = (int)((total4 + 255) / 256);
    nb4 = nb4 < kNormBlocks ? nb4 : kNormBlocks;
    k_grad_sqnorm4<<<nb4, 256, 0, (hipStream_t)stream>>>(t, partial, step);
    const int rc = check_launch("k_grad_sqnorm4");
    if (rc != NARDE_OK) return rc;
    k_adam4<<<(unsigned)((total4 + 255) / 256), 256, 0, (hipStream_t)stream>>>(t, partial, nb4, max_norm, step, lr,
                                                                              beta1, beta2, eps);
    return check_launch("k_adam4");
  }
  int nb = (int)((total + 256 * 16 - 1) / (256 * 16));  // ~16 elements per thread
  nb = nb < kNormBlocks ? nb : kNormBlocks;
  k_grad_sqnorm<<<nb, 256, 0, (hipStream_t)stream>>>(t, partial, step);
  const int rc = check_launch("k_grad_sqnorm");
  if (rc != NARDE_OK) return rc;
  k_adam<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(t, partial, nb, max_norm, step, lr, beta1,
                                                                           beta2, eps);
  return check_launch("k_adam");
}

int narde_per_sample_gather(int device, const float* p, const float* cdf, int64_t n, int64_t batch, uint64_t seed,
                            const int64_t* counter, const double* beta, int64_t* idx, float* w, int state_size,
                            const float* obs, int64_t next_stride, int64_t capacity, const int64_t* action,
                            const float* reward, const float* done, float* s, float* ns, int64_t* a, float* r,
                            float* d, void* stream) {
  if (!p || !cdf || !counter || !beta || !idx || !w || !obs || !action || !reward || !done || !s || !ns || !a || !r ||
      !d)
    return bad("NULL argument");
  if (n <= 0 || batch <= 0 || batch > (int64_t(1) << 24)) return bad("need n > 0 and 0 < batch <= 2^24");
  if (state_size <= 0 || batch * state_size >= (int64_t(1) << 31)) return bad("bad sizes");
  if (capacity <= 0 || n > capacity || next_stride < 0 || next_stride >= capacity) return bad("bad ring geometry");
  DeviceGuard dg(device);
  const unsigned blocks = (unsigned)((batch + kSampleWaves - 1) / kSampleWaves);
  k_per_sample_gather<<<blocks, 64 * kSampleWaves, 0, (hipStream_t)stream>>>(
      p, cdf, n, (int)batch, (uint32_t)seed, (uint32_t)(seed >> 32), counter, beta, idx, w, state_size, obs,
      next_stride, capacity, action, reward, done, s, ns, a, r, d);
  return check_launch("k_per_sample_gather");
}

int narde_target_max2(int device, const float* nq1, int64_t ld1, const float* base, int64_t ld, const float* tab,
                      int64_t ld_tab, int64_t n, float* m1, int64_t* am1, float* m2, void* stream) {
  if (!nq1 || !base || !tab || !m1 || !m2) return bad("NULL argument");
  if (n < 0 || n > (int64_t(1) << 31) - 4 || ld1 < 576 || ld < 576 || ld_tab < 576) return bad("bad sizes");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_target_max2<<<(unsigned)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(nq1, ld1, base, ld, tab, ld_tab, (int)n,
                                                                          m1, am1, m2);
  return check_launch("k_target_max2");
}

int narde_dqn_loss_prio(int device, const float* q1, const float* q2, const float* m1, const float* m2,
                        const float* r, const float* d, float* w, int64_t batch, float gamma, float* td, float* loss,
                        float* loss_copy, float* g1, float* g2, const int64_t* idx, float eps, float* prio,
                        float* max_prio, float* epsilon, float eps_min, float eps_decay, int64_t* cursor,
                        int64_t cursor_add, int64_t cursor_mod, int64_t* tag, int64_t* counter, double* beta,
                        double beta_inc, void* stream) {
  if (!q1 || !q2 || !m1 || !m2 || !r || !d || !w || !td || !loss || !g1 || !g2 || !idx || !prio || !max_prio ||
      !counter || !beta)
    return bad("NULL argument");
  if (batch <= 0 || batch > (int64_t(1) << 24)) return bad("bad batch");
  if (cursor && (cursor_mod <= 0 || cursor_add < 0)) return bad("bad cursor step");
  DeviceGuard dg(device);
  k_dqn_loss_prio<<<1, kLearnThreads, 0, (hipStream_t)stream>>>(q1, q2, m1, m2, r, d, w, (int)batch, gamma, td, loss,
                                                                loss_copy, g1, g2, idx, eps, prio, max_prio, epsilon,
                                                                eps_min, eps_decay, cursor, cursor_add, cursor_mod,
                                                                tag, counter, beta, beta_inc);
  return check_launch("k_dqn_loss_prio");
}

// A/B switch of the round-6 learner forms (tools, tests): bit 1 = the
// float4 clip + Adam.  Returns the previous value.
int narde_learner_variant(int flags) {
  const int prev = adam_vec4 ? 2 : 0;
  adam_vec4 = (flags & 2) != 0;
  return prev;
}

}  // extern "C"
