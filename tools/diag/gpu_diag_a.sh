set -o pipefail
mkdir -p gpurun_out/diag_a
timeout -k 10 120 python tools/diag/host_overheads.py > gpurun_out/diag_a/yield.txt 2>&1 && cat gpurun_out/diag_a/yield.txt && \
NARDE_SPIN=1 timeout -k 10 120 python tools/diag/host_overheads.py > gpurun_out/diag_a/spin.txt 2>&1 && cat gpurun_out/diag_a/spin.txt && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_dqn.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/diag_a/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/diag_a/pytest.log; exit $rc
