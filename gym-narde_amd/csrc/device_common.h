// device_common.h -- env planes, launch shape and the device RNG draws
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

// ---- build knobs (-D...; the defaults are the product build) -------------
// REF2 rollout kernel: 1 = producer/consumer k_rollout_pc, 0 = one wave per
// 64 envs (k_rollout; A/B diagnostic builds only)
#ifndef NARDE_ROLLOUT_PC
#define NARDE_ROLLOUT_PC 1
#endif

// Output store strategy (tools/diag/variants.sh):
//   0: each lane stores its own 96-B obs row (6 x 16 B at a 96-B lane stride:
//      every wave-instruction touches ~48 partial 128-B lines);
//   1: the wave transposes its 64 rows (6 KiB) through LDS so each
//      wave-instruction stores one contiguous 1 KiB (8 whole lines);
//   2: as 1 with non-temporal (streaming) stores for every per-ply output;
//   3: non-temporal obs only; 4: non-temporal narrow outputs only.
// Sustained 1,000-ply REF2 rollouts (tools/diag/gpu_sus_libs.sh, one box):
// 1 and 4 0.1265 ms per 100 plies, 2 and 3 0.135 -- non-temporal obs
// stores cost 6 %.
#ifndef NARDE_OBS_STORE
#define NARDE_OBS_STORE 1
#endif

// wave priority in k_rollout_pc: 0 none (age decides), 1 consumers first,
// 2 producers first
#ifndef NARDE_PC_PRIO
#define NARDE_PC_PRIO 0
#endif

// unroll the rule waves' plies of a full barrier block (k_rollout_pc;
// measured within noise, +-2 %: off)
#ifndef NARDE_PC_UNROLL
#define NARDE_PC_UNROLL 0
#endif

// DIAGNOSTIC ablations (timing only; results are wrong): FULL4 turn bits
// 1 no first-sub-move pass, 2 no later doubles passes, 4 all turns treated as
// block-free; REF2 consumer bits 8 no obs arithmetic, 16 no Philox; REF2
// k_rollout_pc bits 32 rule waves skip the rules (results from the draws
// only), 64 consumers compute everything but issue no global store; FULL4
// pass tasks 128 skip the doubles search, 256 skip the pair check; REF2
// k_rollout_pc 512 consumers store the obs rows only; FULL4 1024 two-dice
// turns treated as block-free, 2048 doubles turns treated as block-free
#ifndef NARDE_DIAG_ABLATE
#define NARDE_DIAG_ABLATE 0
#endif

// DIAGNOSTIC in-kernel clock stamps of k_rollout_pc (narde_diag_clock)
#ifndef NARDE_DIAG_CLOCK
#define NARDE_DIAG_CLOCK 0
#endif

namespace {

constexpr int kBlock = 256;

struct Planes {
  uint4* p0;
  uint4* p1;
  int4* stats;
};

struct Rng {
  uint32_t env0, k0, k1;
  int dice_mode;
};

__device__ __forceinline__ void draw(const Rng& g, uint32_t t, uint32_t i, uint32_t stream,
                                     uint32_t r[4]) {
  philox4x32_10(t, g.env0 + i, 0u, stream, g.k0, g.k1, r);
}

// the four words of ply t of env i (narde_rules.h ply_words: one Philox
// block per two plies; a kernel that runs consecutive plies keeps the block)
__device__ __forceinline__ void ply_draw(const Rng& g, uint32_t t, uint32_t i, uint32_t r[4]) {
  uint32_t R[4];
  ply_block(t, g.env0 + i, g.k0, g.k1, R);
  ply_words_of(R, t, g.dice_mode, r);
}

}  // namespace
