#!/usr/bin/env python3
"""DIAGNOSTIC: build tools/diag/build/libnarde_f4count.so -- the working
tree's library with per-rule-wave counters in k_rollout_full (loop passes
that play, passes that only wait for the helper, lanes playing per pass,
parks) and an export narde_diag_f4(uint64 *host) copying them out
([4096 waves][4]).  Read by tools/diag/f4_counts.py.  Product untouched."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sub(s, old, new):
    assert s.count(old) >= 1, old
    return s.replace(old, new, 1)


def main():
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(ROOT, "gym-narde_amd"), os.path.join(tmp, "gym-narde_amd"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    csrc = os.path.join(tmp, "gym-narde_amd", "csrc")
    p = os.path.join(csrc, "kernels_rollout.h")
    s = open(p).read()
    s = sub(s, "template <bool kOut>\n__global__ void __launch_bounds__(kFxThreads) k_rollout_full(",
            "__device__ unsigned long long g_f4[4096 * 4];\n"
            "template <bool kOut>\n__global__ void __launch_bounds__(kFxThreads) k_rollout_full(")
    s = sub(s, "    int lo = 0;          // the slowest lane's next ply (wave-uniform)\n    for (;;) {\n",
            "    int lo = 0;          // the slowest lane's next ply (wave-uniform)\n"
            "    unsigned long long c_pass = 0, c_wait = 0, c_lanes = 0, c_parks = 0;\n    for (;;) {\n")
    s = sub(s, "        // parked lanes hold the wave: wait for the helper\n",
            "        ++c_wait;\n        // parked lanes hold the wave: wait for the helper\n")
    s = sub(s, "      uint32_t r[4] = {0u, 0u, 0u, 0u};\n      int dh = 1, dl = 1;\n",
            "      ++c_pass;\n      c_lanes += __builtin_popcountll(__ballot(act));\n"
            "      uint32_t r[4] = {0u, 0u, 0u, 0u};\n      int dh = 1, dl = 1;\n")
    s = sub(s, "      if (__ballot(pk) != 0ull) wake_workgroup();  // the helper sleeps\n",
            "      c_parks += __builtin_popcountll(__ballot(pk));\n"
            "      if (__ballot(pk) != 0ull) wake_workgroup();  // the helper sleeps\n")
    # helper wave: passes with work, lanes served, clock ticks spent in them
    s = sub(s, "    uint32_t done = 0u;  // parks of rule lane `lane` answered\n",
            "    uint32_t done = 0u;  // parks of rule lane `lane` answered\n"
            "    unsigned long long h_pass = 0, h_lanes = 0, h_ticks = 0;\n")
    s = sub(s, "      if (__ballot(mine) != 0ull) {  // wave-uniform\n",
            "      if (__ballot(mine) != 0ull) {  // wave-uniform\n"
            "        ++h_pass;\n        h_lanes += __builtin_popcountll(__ballot(mine));\n"
            "        const unsigned long long h_t0 = wall_clock64();\n")
    s = sub(s, "          lds_publish(&M.back[lane], want);\n        }\n        continue;\n",
            "          lds_publish(&M.back[lane], want);\n        }\n"
            "        h_ticks += wall_clock64() - h_t0;\n        continue;\n")
    s = sub(s, "      if (__builtin_amdgcn_readfirstlane((int)lds_acquire(&M.fin)) != 0) break;\n",
            "      if (__builtin_amdgcn_readfirstlane((int)lds_acquire(&M.fin)) != 0) {\n"
            "        if (lane < 3) {\n"
            "          const unsigned long long v = lane == 0 ? h_pass : (lane == 1 ? h_lanes : h_ticks);\n"
            "          g_f4h[(size_t)(blockIdx.x * kFxGroups + grp) * 4 + lane] = v;\n"
            "        }\n"
            "        break;\n      }\n")
    s = sub(s, "__device__ unsigned long long g_f4[4096 * 4];\n",
            "__device__ unsigned long long g_f4[4096 * 4];\n__device__ unsigned long long g_f4h[4096 * 4];\n")
    # rule wave: clock ticks of the whole loop
    s = sub(s, "    unsigned long long c_pass = 0, c_wait = 0, c_lanes = 0, c_parks = 0;\n",
            "    unsigned long long c_pass = 0, c_wait = 0, c_lanes = 0, c_parks = 0;\n"
            "    const unsigned long long r_t0 = wall_clock64();\n")
    s = sub(s, "    lds_publish(&M.fin, 1u);\n",
            "    lds_publish(&M.fin, 1u);\n"
            "    const unsigned long long r_ticks = wall_clock64() - r_t0;\n"
            "    if (lane < 4) {\n"
            "      const unsigned long long v = lane == 0 ? c_pass : (lane == 1 ? c_wait : (lane == 2 ? c_lanes : c_parks));\n"
            "      g_f4[(size_t)(blockIdx.x * kFxGroups + grp) * 4 + lane] = v;\n"
            "    }\n"
            "    if (lane == 4) g_f4h[(size_t)(blockIdx.x * kFxGroups + grp) * 4 + 3] = r_ticks;\n")
    open(p, "w").write(s)
    p = os.path.join(csrc, "narde.hip")
    s = open(p).read()
    s += ('\nextern "C" int narde_diag_f4(unsigned long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_f4), sizeof(g_f4));\n}\n'
          'extern "C" int narde_diag_f4h(unsigned long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_f4h), sizeof(g_f4h));\n}\n')
    open(p, "w").write(s)
    out = os.path.join(ROOT, "tools", "diag", "build", "libnarde_f4count.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                           "-o", out, os.path.join(csrc, "narde.hip"), os.path.join(csrc, "dqn_learner.hip")])
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    main()
