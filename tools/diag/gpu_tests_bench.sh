set -o pipefail
mkdir -p gpurun_out/r01b
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01b/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r01b/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r01b/bench.json 2> gpurun_out/r01b/bench.err; rc=$?
cat gpurun_out/r01b/bench.json; tail -5 gpurun_out/r01b/bench.err
exit $rc
