# full GPU suite + default bench (round 2, step b)
set -o pipefail
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r2b/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r2b/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r2b/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r2b/bench.log
exit $rc
