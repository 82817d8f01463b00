// device_common.h -- env planes, launch shape and the device RNG draws
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

namespace {

constexpr int kBlock = 256;
constexpr int kTotalRows = NARDE_TOTAL_ROWS;  // narde_get_totals' partial rows

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

// Hand-over of a wave's own LDS writes to other lanes of the same wave: the
// LDS ops of one wave retire in issue order, so no hardware wait is needed,
// but the wave barrier alone is not a memory fence in the IR -- the
// wavefront-scope release/acquire pair makes the cross-lane read-after-write
// explicit to the compiler (no instruction on gfx950).
__device__ __forceinline__ void wave_lds_handoff() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the four words of ply t of env i (narde_rules.h ply_words: one Philox
// block per two plies; a kernel that runs consecutive plies keeps the block)
__device__ __forceinline__ void ply_draw(const Rng& g, uint32_t t, uint32_t i, uint32_t r[4]) {
  uint32_t R[4];
  ply_block(t, g.env0 + i, g.k0, g.k1, R);
  ply_words_of(R, t, g.dice_mode, r);
}

}  // namespace
