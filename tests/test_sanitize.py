"""Host-side sanitizers: the C oracle and the CPU build
of the device rules engine under AddressSanitizer + UndefinedBehaviorSanitizer,
driven by the golden-vector, random-position and self-play CPU tests
(tools/sanitize.sh).  GPU code is not sanitized (not available on the pool)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"),
                    reason="clang ASan runtime not present")
def test_oracle_and_rules_engine_clean_under_asan_ubsan():
    if os.environ.get("NARDE_HOSTCHECK_LIB") or os.environ.get("NARDE_ORACLE_LIB"):
        pytest.skip("already running under tools/sanitize.sh")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh")], cwd=ROOT, capture_output=True,
                       text=True, timeout=600, env={**os.environ, "PYTHON": sys.executable})
    assert r.returncode == 0, (r.stdout[-3000:] + r.stderr[-3000:])
    assert " passed" in r.stdout
