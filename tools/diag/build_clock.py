#!/usr/bin/env python3
"""DIAGNOSTIC: build tools/diag/build/libnarde_clock.so -- the working tree's
library with wall_clock64() stamps in k_rollout_pc (lane 0 of every wave:
entry, the start barrier, every block barrier, the end) and an export
narde_diag_ts(int64 *host) that copies them out ([2048 waves][64]).  Read by
tools/diag/clock_anatomy.py.  The product source is untouched."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sub(s, old, new, count=1):
    assert s.count(old) >= count, old
    return s.replace(old, new, count)


def main():
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(ROOT, "gym-narde_amd"), os.path.join(tmp, "gym-narde_amd"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    csrc = os.path.join(tmp, "gym-narde_amd", "csrc")
    p = os.path.join(csrc, "kernels_rollout.h")
    s = open(p).read()
    s = sub(s, "template <bool kOut, bool kNt>\n__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(",
            "__device__ long long g_ts[4096 * 64];\n"
            "template <bool kOut, bool kNt>\n__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(")
    s = sub(s, "  const int nb = pc_nblocks(plies);\n",
            "  const int nb = pc_nblocks(plies);\n"
            "  long long* TS = g_ts + (size_t)(blockIdx.x * 8 + wave) * 64;\n"
            "  if (lane == 0) TS[0] = wall_clock64();\n")
    s = sub(s, "  if (!producer) draw_block(0);\n  __syncthreads();\n",
            "  if (!producer) draw_block(0);\n  __syncthreads();\n  if (lane == 0) TS[1] = wall_clock64();\n")
    s = sub(s, "    __syncthreads();\n  }\n  if (kOut && !producer && nb > 0) {",
            "    __syncthreads();\n    if (lane == 0 && b < 60) TS[2 + b] = wall_clock64();\n  }\n"
            "  if (kOut && !producer && nb > 0) {")
    s = sub(s, "    add_stats(pl.stats, i, st);\n  }\n}\n\n}  // namespace",
            "    add_stats(pl.stats, i, st);\n  }\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
            "  if (lane == 0) TS[63] = wall_clock64();\n}\n\n}  // namespace")
    open(p, "w").write(s)
    p = os.path.join(csrc, "narde.hip")
    s = open(p).read()
    s += ('\nextern "C" int narde_diag_ts(long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ts), sizeof(g_ts));\n}\n')
    open(p, "w").write(s)
    out = os.path.join(ROOT, "tools", "diag", "build", "libnarde_clock.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                           "-o", out, os.path.join(csrc, "narde.hip"), os.path.join(csrc, "dqn_learner.hip")])
    # the device assembly, to check that the stamps are vector stores
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-S",
                           "--cuda-device-only", "-o", out[:-3] + ".s", os.path.join(csrc, "narde.hip")])
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    main()
