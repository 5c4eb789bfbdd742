set -o pipefail
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_formats_group.py tests/test_cli.py -m gpu -p no:cacheprovider > gpurun_out/r2a/new_tests.log 2>&1
rc=$?; echo "new_tests rc=$rc"; tail -5 gpurun_out/r2a/new_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r2a/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r2a/bench.log
exit $rc
