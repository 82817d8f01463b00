#!/usr/bin/env python3
"""DIAGNOSTIC: build tools/diag/build/libnarde_ppclock.so -- the working
tree's library with per-ply clocks in k_rollout_pp_full's producer waves
(lane 0, wall_clock64 at 100 MHz, vector stores) and an export
narde_diag_pp(int64 *host) that copies them out: [1024 producer waves][plies
<= 160][12] = {ply start (after the draw wait), ply end (results in LDS),
kind bits, searching lanes (NOT trusted: it reads 0.1-0.4 % of wave-plies
where round 5's k_step clocks found 6.7 %), 8 segment
cycle counts (s_memtime): 0 block
test, 1 turn_c0_free, 2 the turn, 3 / 4 / 5 the bound turn's pair-bound C_0,
doubles-bound C_0 and sub-moves, 6 the close}.  kind bit 0: the wave holds a block-bound
doubles lane (ply_bound_turn_c0), bit 1: a block-bound two-dice lane, bit 2:
some lane searched (coop_pair_w / coop_depth_w).  Read by
tools/diag/pp_phase.py.  The product source is untouched."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MAXP = 160


def sub(s, old, new, count=1):
    assert s.count(old) >= count, old
    return s.replace(old, new, count)


def main():
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(ROOT, "gym-narde_amd"), os.path.join(tmp, "gym-narde_amd"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    csrc = os.path.join(tmp, "gym-narde_amd", "csrc")
    # the searching lanes of the wave, left in a per-wave LDS word
    # per-wave segment cycle accumulators (s_memtime, lane 0), in LDS
    p = os.path.join(csrc, "device_common.h")
    s = open(p).read()
    s += ("\nnamespace {\n__shared__ uint32_t g_dbg_srch[16];\n__shared__ long long g_seg[16][8];\n"
          "#define SEG_T0() const long long seg_t0_ = (long long)__builtin_amdgcn_s_memtime()\n"
          "#define SEG_MARK(k) do { const long long seg_t_ = (long long)__builtin_amdgcn_s_memtime(); "
          "if ((threadIdx.x & 63) == 0) g_seg[threadIdx.x >> 6][k] += seg_t_; } while (0)\n"
          "#define SEG_START(k) do { const long long seg_t_ = (long long)__builtin_amdgcn_s_memtime(); "
          "if ((threadIdx.x & 63) == 0) g_seg[threadIdx.x >> 6][k] -= seg_t_; } while (0)\n}\n")
    open(p, "w").write(s)
    p = os.path.join(csrc, "full4_wave.h")
    s = open(p).read()
    # segments inside the bound turn: 3 pair-bound C_0, 4 doubles-bound C_0 (reject, safe bound, searches), 5 sub-moves
    s = sub(s, "  if (__ballot(b2) != 0ull) {\n    if (b2) turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh, Ll, Ch, Cl, M);\n  }\n",
            "  SEG_START(3);\n  if (__ballot(b2) != 0ull) {\n    if (b2) turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh, Ll, Ch, Cl, M);\n  }\n  SEG_MARK(3);\n  SEG_START(4);\n")
    s = sub(s, "    M = bd ? (fast ? 4 : (Lb ? Ms : 0)) : M;\n  }\n",
            "    M = bd ? (fast ? 4 : (Lb ? Ms : 0)) : M;\n  }\n  SEG_MARK(4);\n  SEG_START(5);\n")
    s = sub(s, "  o.played = (uint64_t)pl0 | ((uint64_t)pl1 << 32);\n  o.max_dice = M;\n  o.term = s.off_own == 15u;\n  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;\n  if (flip_always) side_flip(s);\n  else side_flip_if(s, !o.term);\n}\n\n__device__ __forceinline__ void ply_bound_turn(",
            "  SEG_MARK(5);\n  o.played = (uint64_t)pl0 | ((uint64_t)pl1 << 32);\n  o.max_dice = M;\n  o.term = s.off_own == 15u;\n  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;\n  if (flip_always) side_flip(s);\n  else side_flip_if(s, !o.term);\n}\n\n__device__ __forceinline__ void ply_bound_turn(")
    s = sub(s, "    coop_pair_w(s, fw, dh, hl0, srch ? Lb : 0u, w[0], lane, r0, c1p, pairs);\n",
            "    coop_pair_w(s, fw, dh, hl0, srch ? Lb : 0u, w[0], lane, r0, c1p, pairs);\n"
            "    if (lane == 0) g_dbg_srch[threadIdx.x >> 6] = (uint32_t)__builtin_popcountll(__ballot(srch));\n")
    open(p, "w").write(s)
    p = os.path.join(csrc, "kernels_rollout.h")
    s = open(p).read()
    # segments of ply_full_dice: 0 block test, 1 turn_c0_free, 2 the turn (free or bound), 6 the close
    s = sub(s, "  const uint32_t low = block_lowmask(s.P);\n  uint32_t fw;\n  const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl, fw);\n  TurnC0 c;\n  turn_c0_free(s, dh, dl, c.Lh, c.Ll, c.Ch, c.Cl, c.M, c.hl0);\n",
            "  SEG_START(0);\n  const uint32_t low = block_lowmask(s.P);\n  uint32_t fw;\n  const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl, fw);\n  SEG_MARK(0);\n  SEG_START(1);\n  TurnC0 c;\n  turn_c0_free(s, dh, dl, c.Lh, c.Ll, c.Ch, c.Cl, c.M, c.hl0);\n  SEG_MARK(1);\n")
    s = sub(s, "  const uint32_t mover_black = s.black;\n  // three kinds of wave",
            "  const uint32_t mover_black = s.black;\n  SEG_START(2);\n  // three kinds of wave")
    s = sub(s, "    ply_bound_turn_c0(s, dh, dl, bs, fw, w, autoreset, o, (int)(threadIdx.x & 63), c);\n  }\n  if (autoreset) ply_close_sl_b(s, st, o.term, o.reward, mover_black, rb, max_steps, term, trunc);\n"
               "  else ply_close(s, st, o.term, o.reward, mover_black, 0u, max_steps, false, term, trunc);\n",
            "    ply_bound_turn_c0(s, dh, dl, bs, fw, w, autoreset, o, (int)(threadIdx.x & 63), c);\n  }\n  SEG_MARK(2);\n  SEG_START(6);\n  if (autoreset) ply_close_sl_b(s, st, o.term, o.reward, mover_black, rb, max_steps, term, trunc);\n"
            "  else ply_close(s, st, o.term, o.reward, mover_black, 0u, max_steps, false, term, trunc);\n  SEG_MARK(6);\n")
    s = sub(s, "// spin until f(counter value) holds",
             f"__device__ long long g_pp[1024 * {MAXP} * 12];\n// spin until f(counter value) holds")
    s = sub(s, "      const uint4 wv = L.draw_w[cw][sl][lane];\n      const uint32_t dw = L.draw_d[cw][sl][lane];\n",
            "      const uint4 wv = L.draw_w[cw][sl][lane];\n      const uint32_t dw = L.draw_d[cw][sl][lane];\n"
            f"      long long* TP = g_pp + ((size_t)(blockIdx.x * 4 + cw) * {MAXP} + (p < {MAXP} ? p : {MAXP} - 1)) * 12;\n"
            "      if (lane == 0) { TP[0] = wall_clock64(); g_dbg_srch[wave] = 0u; for (int q = 0; q < 8; ++q) g_seg[wave][q] = 0; }\n"
            "      {\n"
            "        const int ddh = (int)(dw & 15u), ddl = (int)((dw >> 4) & 15u);\n"
            "        uint32_t dfw;\n"
            "        const uint32_t dbs = turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), ddh, ddl, dfw);\n"
            "        const uint32_t kd = (__ballot(dbs != 0u && ddh == ddl) ? 1u : 0u) | (__ballot(dbs != 0u && ddh != ddl) ? 2u : 0u);\n"
            "        if (lane == 0) TP[2] = kd;\n"
            "        if (lane == 0) TP[0] = wall_clock64();\n"
            "      }\n")
    s = sub(s, "        L.rtt[cw][sl][lane] = (uint32_t)o.reward | ((uint32_t)term << 8) | ((uint32_t)trunc << 16);\n      }\n",
            "        L.rtt[cw][sl][lane] = (uint32_t)o.reward | ((uint32_t)term << 8) | ((uint32_t)trunc << 16);\n      }\n"
            "      if (lane == 0) { TP[1] = wall_clock64(); TP[3] = g_dbg_srch[wave]; for (int q = 0; q < 8; ++q) TP[4 + q] = g_seg[wave][q]; }\n")
    open(p, "w").write(s)
    p = os.path.join(csrc, "narde.hip")
    s = open(p).read()
    s += ('\nextern "C" int narde_diag_pp(long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pp), sizeof(g_pp));\n}\n')
    open(p, "w").write(s)
    out = os.path.join(ROOT, "tools", "diag", "build", "libnarde_ppclock.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                           "-o", out, os.path.join(csrc, "narde.hip"), os.path.join(csrc, "dqn_learner.hip")])
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    main()
