set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/ab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ab/pytest.log
[ $rc -eq 0 ] && bash tools/diag/ab_rollout.sh run 2>&1 | grep -v amdgpu.ids
