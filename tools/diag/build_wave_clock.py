#!/usr/bin/env python3
"""DIAGNOSTIC: build tools/diag/build/libnarde_wclock{,_full}.so -- the working
tree's library with wall_clock64() stamps (lane 0 of every wave: entry and
the end of its ply loop) in the FULL4 rollouts k_rollout_wave and
k_rollout_full, and an export narde_diag_wts(int64 *host) that copies them
out ([4096 waves][2]).  The _full build takes k_rollout_full at every launch
length (kFxMinPlies = 1).  Read by tools/diag/wave_clock.py: is a short
FULL4 launch bound by its mean wave or by its slowest one?  The product
source is untouched."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sub(s, old, new, count=1):
    assert s.count(old) >= count, old
    return s.replace(old, new, count)


WAVE_PLY = ("    ply(s, st, g, (uint32_t)i, valid, (const int8_t*)nullptr, nullptr, max_steps, true, o, term, trunc, R,\n"
            "        p == 0);\n")
# k_rollout_wave with the block test first: a wave with no block-bound lane
# plays turn_free, else the cooperative turn ("free"); or turn_free for every
# lane -- wrong results, timing only ("allfree")
WAVE_FAST = """    uint32_t r[4];
    ply_draw_cached(g, s.t, (uint32_t)i, R, p == 0, r);
    int d0, d1;
    dice_from(r[0], g.dice_mode, d0, d1);
    const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
    const uint32_t bs = turn_block_set(s.O, s.S1o, s.P, block_lowmask(s.P), dh, dl);
    uint32_t w[4];
    turn_words(r, w);
    const uint32_t mover_black = s.black;
    if (%s) turn_free(s, dh, dl, w, o);
    else coop_turn_full(s, d0, d1, false, ~0ull, w, o, (int)(threadIdx.x & 63));
    ply_close(s, st, o.term, o.reward, mover_black, r[3], max_steps, true, term, trunc);
"""


# timing-only block-test probes (turn_free for every lane, the test kept alive
# through the played word): the product test ("bsonly"), the prefilter alone
# ("pre"), the test with a branch-free window-loop body ("bsbf")
PROBE_FNS = """
__device__ __forceinline__ uint32_t pre_block(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);
  uint32_t U = A | land_step(A, P, dh) | land_step(A, P, dl);
  const uint32_t V = land_step(U, P, dh);
  U |= dbl ? (V | land_step(V, P, dh)) : 0u;
  (void)S1;
  return runs6(U) & low & windows_few_holes(O, dbl ? 4 : 2);
}
__device__ __forceinline__ uint32_t tbs_bf(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  uint32_t win = pre_block(O, S1, P, low, dh, dl), out = 0u;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    const uint32_t src = O & ~(W & S1);
    uint32_t T = src, seen = 0u, cost = 0u;
#pragma unroll
    for (int j = 1; j <= 4; ++j) {
      T = land_step(T, P, dh);
      const uint32_t nw = H & T & ~seen;
      cost += (uint32_t)j * (uint32_t)__builtin_popcount(nw);
      seen |= nw;
    }
    const uint32_t fd = (seen == H && cost <= 4u) ? W : 0u;
    const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
    const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
    const int i1 = __builtin_ctz(H | 0x80000000u), i2 = __builtin_ctz(h2 | 0x80000000u);
    const uint32_t a1 = (Lh >> i1) & (Ll >> i2), a2 = (Ll >> i1) & (Lh >> i2);
    const uint32_t reach = Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh);
    const uint32_t f1 = (H & reach) ? H : 0u, f2 = ((a1 | a2) & 1u) ? H : 0u;
    const uint32_t ft = h2 ? f2 : f1;
    out |= H == 0u ? ~0u : (dbl ? fd : ft);
  }
  return out;
}
"""


def build(tag, force_full, drift=None, cut=None, wave=None, prio=None):
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(ROOT, "gym-narde_amd"), os.path.join(tmp, "gym-narde_amd"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    csrc = os.path.join(tmp, "gym-narde_amd", "csrc")
    p = os.path.join(csrc, "kernels_rollout.h")
    s = open(p).read()
    s = sub(s, "template <bool kOut>\n__global__ void __launch_bounds__(kBlock, 1) k_rollout_wave(",
            "__device__ long long g_wts[4096 * 2];\n"
            "template <bool kOut>\n__global__ void __launch_bounds__(kBlock, 1) k_rollout_wave(")
    # k_rollout_wave: entry / after the ply loop
    s = sub(s, "  Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);\n"
               "  int4 st = make_int4(0, 0, 0, 0);\n  uint32_t R[4];  // the Philox block of the current ply pair\n",
            "  long long* TS = g_wts + (size_t)(i >> 6) * 2;\n"
            "  if ((threadIdx.x & 63) == 0) TS[0] = wall_clock64();\n"
            "  Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);\n"
            "  int4 st = make_int4(0, 0, 0, 0);\n  uint32_t R[4];  // the Philox block of the current ply pair\n")
    s = sub(s, "    if (kOut && valid) store_outs(out, (size_t)p * n + i, s, o, term, trunc, nullptr, false);\n  }\n",
            "    if (kOut && valid) store_outs(out, (size_t)p * n + i, s, o, term, trunc, nullptr, false);\n  }\n"
            "  if ((threadIdx.x & 63) == 0) TS[1] = wall_clock64();\n")
    # k_rollout_full: entry of every wave, end of the rule loop / helper loop
    s = sub(s, "  int4 cum = make_int4(0, 0, 0, 0);  // the env's statistics after the launch (wg_totals)\n"
               "  if (wave < kFxGroups) {\n",
            "  int4 cum = make_int4(0, 0, 0, 0);  // the env's statistics after the launch (wg_totals)\n"
            "  long long* TS = g_wts + (size_t)(blockIdx.x * 8 + wave) * 2;\n"
            "  if (lane == 0) TS[0] = wall_clock64();\n"
            "  if (wave < kFxGroups) {\n")
    s = sub(s, "    lds_publish(&M.fin, 1u);\n", "    lds_publish(&M.fin, 1u);\n    if (lane == 0) TS[1] = wall_clock64();\n")
    s = sub(s, "      __builtin_amdgcn_s_sleep(24);\n    }\n",
            "      __builtin_amdgcn_s_sleep(24);\n    }\n    if (lane == 0) TS[1] = wall_clock64();\n")
    if wave == "passes":  # count the cooperative passes (owners > 0) per wave, by mode
        q = os.path.join(csrc, "kernels_full4.h")
        t = open(q).read()
        t = sub(t, "__device__ void coop_run(", "__device__ unsigned g_passes[4096 * 2];\n__device__ void coop_run(")
        t = sub(t, "  const int which = lane >> 5, p = lane & 31;\n  while (owners) {",
                "  const int which = lane >> 5, p = lane & 31;\n"
                "  if (owners != 0ull && lane == 0)\n"
                "    atomicAdd(&g_passes[((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 2 + (mode ? 1 : 0)],\n"
                "              (unsigned)__builtin_popcountll(owners));\n"
                "  while (owners) {")
        open(q, "w").write(t)
        s2 = open(os.path.join(csrc, "narde.hip")).read()
        s2 += ('\nextern "C" int narde_diag_passes(unsigned* host, int zero) {\n'
               '  if (zero) { static unsigned z[4096 * 2]; return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_passes), z, sizeof(z)); }\n'
               '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_passes), sizeof(g_passes));\n}\n')
        open(os.path.join(csrc, "narde.hip"), "w").write(s2)
    if wave == "free":
        s = sub(s, WAVE_PLY, WAVE_FAST % "__ballot(bs != 0u) == 0ull")
    elif wave == "allfree":
        s = sub(s, WAVE_PLY, WAVE_FAST % "true || bs == 0u")
    elif wave == "unroll":  # turn_play's later sub-moves unrolled (product semantics)
        q = os.path.join(csrc, "kernels_full4.h")
        t = open(q).read()
        t = sub(t, "  for (int k = 1; k < 4; ++k) {\n    const bool act = go && k < M;",
                "#pragma unroll\n  for (int k = 1; k < 4; ++k) {\n    const bool act = go && k < M;")
        open(q, "w").write(t)
    elif wave in ("nc_nofilt0", "nc_nolater", "nc_nosure", "nc_min"):
        # on top of "nocoop" (timing only): no root block filter ("nc_nofilt0"),
        # no block filter in the later sub-moves ("nc_nolater"), no sure-move
        # masks ("nc_nosure"), none of the three ("nc_min")
        q = os.path.join(csrc, "kernels_full4.h")
        t = open(q).read()
        t = sub(t, "fast = dbl && !bf && f4_safe_bound(s, dh, hl0, ws) >= 4;", "fast = dbl && !bf;")
        if wave in ("nc_nosure", "nc_min"):
            t = sub(t, "sh = nbf2 ? f4_sure_pair(s.O, s.P, dl, Lh, hs) : 0u;", "sh = nbf2 ? Lh : 0u;")
            t = sub(t, "sl = nbf2 ? f4_sure_pair(s.O, s.P, dh, Ll, hs) : 0u;", "sl = nbf2 ? Ll : 0u;")
        else:
            t = sub(t, "sh = nbf2 ? f4_sure_pair(s.O, s.P, dl, Lh, hs) : 0u;", "sh = nbf2 ? (Lh | f4_sure_pair(s.O, s.P, dl, Lh, hs)) : 0u;")
            t = sub(t, "sl = nbf2 ? f4_sure_pair(s.O, s.P, dh, Ll, hs) : 0u;", "sl = nbf2 ? (Ll | f4_sure_pair(s.O, s.P, dh, Ll, hs)) : 0u;")
        if wave in ("nc_nofilt0", "nc_min"):
            t = sub(t, "  if (!bf) {\n    const Blocks bl = block_info_low(s.O, low);", "  if (false) {\n    const Blocks bl = block_info_low(s.O, low);")
        if wave in ("nc_nolater", "nc_min"):
            t = sub(t, "if (act && !bf) Lk = die_filter(s.O, s.S1o, block_info_low(s.O, low), Lk, dk);", "")
        open(q, "w").write(t)
    elif wave in ("nodsearch", "notask", "nocoop"):
        # timing only (wrong results): block-bound doubles never search
        # ("nodsearch"), block-bound two-dice first moves all sure ("notask"), both ("nocoop")
        q = os.path.join(csrc, "kernels_full4.h")
        t = open(q).read()
        if wave in ("nodsearch", "nocoop"):
            t = sub(t, "fast = dbl && !bf && f4_safe_bound(s, dh, hl0, ws) >= 4;", "fast = dbl && !bf;")
        if wave in ("notask", "nocoop"):
            t = sub(t, "sh = nbf2 ? f4_sure_pair(s.O, s.P, dl, Lh, hs) : 0u;", "sh = nbf2 ? Lh : 0u;")
            t = sub(t, "sl = nbf2 ? f4_sure_pair(s.O, s.P, dh, Ll, hs) : 0u;", "sl = nbf2 ? Ll : 0u;")
        open(q, "w").write(t)
    elif wave in ("bsonly", "pre", "bsbf"):
        fn = {"bsonly": "turn_block_set", "pre": "pre_block", "bsbf": "tbs_bf"}[wave]
        body = (WAVE_FAST % "true || bs == 0u").replace("turn_block_set(", fn + "(")
        body = body.replace("    ply_close(", "    o.played ^= (uint64_t)bs;\n    ply_close(")
        s = sub(s, WAVE_PLY, body)
        s = sub(s, "// k_rollout_wave: the FULL4 rollout", PROBE_FNS + "// k_rollout_wave: the FULL4 rollout")
    if prio is not None:  # the helper's turn at a raised wave priority (s_setprio)
        s = sub(s, "        coop_turn_full<true>(s, d0, d1, false, ~0ull, w, o, lane, bs);",
                f"        __builtin_amdgcn_s_setprio({prio});\n"
                "        coop_turn_full<true>(s, d0, d1, false, ~0ull, w, o, lane, bs);")
        s = sub(s, "          lds_publish(&M.back[lane], want);\n        }\n",
                "          lds_publish(&M.back[lane], want);\n        }\n        __builtin_amdgcn_s_setprio(0);\n")
    if force_full:
        s = sub(s, "constexpr int kFxMinPlies = 48;", "constexpr int kFxMinPlies = 1;")
    if drift is not None:
        s = sub(s, "constexpr int kFxDrift = 16;", f"constexpr int kFxDrift = {drift};")
    open(p, "w").write(s)
    if cut is not None:  # the block-free cut inside the cooperative depth search, top `cut` levels
        p = os.path.join(csrc, "kernels_full4.h")
        s = open(p).read()
        for n in (1, 2, 3):
            s = sub(s, f"f4_depth<{n}, 0>", f"f4_depth<{n}, {min(n, cut)}>")
        open(p, "w").write(s)
    p = os.path.join(csrc, "narde.hip")
    s = open(p).read()
    s += ('\nextern "C" int narde_diag_wts(long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wts), sizeof(g_wts));\n}\n')
    open(p, "w").write(s)
    out = os.path.join(ROOT, "tools", "diag", "build", f"libnarde_{tag}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                           "-o", out, os.path.join(csrc, "narde.hip"), os.path.join(csrc, "dqn_learner.hip")])
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "wave":  # build_wave_clock.py wave free allfree
        for v in sys.argv[2:]:
            build(f"wclock_{v}", False, wave=v)
    elif len(sys.argv) > 1 and sys.argv[1] == "prio":  # build_wave_clock.py prio 1 3
        for q in sys.argv[2:]:
            build(f"wclock_full_p{q}", True, prio=int(q))
            build(f"wclock_full_d4p{q}", True, drift=4, prio=int(q))
    elif len(sys.argv) > 1 and sys.argv[1] == "cut":  # build_wave_clock.py cut 1 3
        for c in sys.argv[2:]:
            build(f"wclock_cut{c}", False, cut=int(c))
    elif len(sys.argv) > 1:  # drift variants of the forced k_rollout_full: build_wave_clock.py 4 8
        for d in sys.argv[1:]:
            build(f"wclock_full_d{d}", True, int(d))
    else:
        build("wclock", False)
        build("wclock_full", True)
