#!/usr/bin/env python3
"""DIAGNOSTIC: build tools/diag/build/libnarde_clock.so -- the working tree's
library with wall_clock64() stamps (100 MHz, lane 0 of every wave, vector
stores) in k_rollout_pc and an export narde_diag_ts(int64 *host) that copies
them out ([2048 waves][64]).  Read by tools/diag/clock_anatomy.py.  The
product source is untouched.  Stamp columns:
  0 entry;  1 producer: record loaded (a vmcnt wait) / consumer: block 0 drawn;
  2 the start barrier passed;  3 + b: block b's closing barrier passed
  (b < 56);  59 consumer: last block emitted (stores issued);  60 producer:
  record + statistics stored;  61 the statistics load returned;  62 after
  wg_totals;  63 the end, after every store of the wave was acknowledged."""
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
    s = sub(s, "template <bool kOut>\n__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(",
            "__device__ long long g_ts[4096 * 64];\n"
            "#define TSTAMP(c) do { if (lane == 0) TS[c] = wall_clock64(); } while (0)\n"
            "template <bool kOut>\n__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(")
    s = sub(s, "  const int nb = pc_nblocks(plies, R);\n\n  Side s;\n",
            "  const int nb = pc_nblocks(plies, R);\n"
            "  long long* TS = g_ts + (size_t)(blockIdx.x * 8 + wave) * 64;\n"
            "  TSTAMP(0);\n\n  Side s;\n")
    s = sub(s, "    if (valid) s = side_from_record(pl.p0[i], pl.p1[i]);\n  } else if (valid) {\n",
            "    if (valid) s = side_from_record(pl.p0[i], pl.p1[i]);\n"
            "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    TSTAMP(1);\n"
            "  } else if (valid) {\n")
    s = sub(s, "  if (!producer) draw_block(0);\n  __syncthreads();\n",
            "  if (!producer) { draw_block(0); TSTAMP(1); }\n  __syncthreads();\n  TSTAMP(2);\n")
    s = sub(s, "    __syncthreads();\n  }\n  if (kOut && !producer && nb > 0) {",
            "    __syncthreads();\n    if (b < 56) TSTAMP(3 + b);\n  }\n"
            "  if (kOut && !producer && nb > 0) {")
    s = sub(s, "    pc_emit(L, (nb - 1) % kPcSlots, np, p0, n, wg_env0, cw, lane, out);\n  }\n"
               "  int4 cum = make_int4(0, 0, 0, 0);\n",
            "    pc_emit(L, (nb - 1) % kPcSlots, np, p0, n, wg_env0, cw, lane, out);\n    TSTAMP(59);\n  }\n"
            "  int4 cum = make_int4(0, 0, 0, 0);\n")
    s = sub(s, "    cum = stats_after(pl.stats, i, st, out.totals != nullptr);\n  }\n"
               "  if (out.totals) wg_totals(cum, out.totals);\n}\n",
            "    TSTAMP(60);\n"
            "    cum = stats_after(pl.stats, i, st, out.totals != nullptr);\n"
            "    if (lane == 0) TS[61] = wall_clock64() + 0 * cum.x;\n  }\n"
            "  if (out.totals) wg_totals(cum, out.totals);\n  TSTAMP(62);\n"
            "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n  TSTAMP(63);\n}\n")
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
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    main()
