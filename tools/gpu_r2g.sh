# round 2 re-entry check: full GPU suite, smoke, default bench, driver-style short bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 3000 $O/bench_default.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_short.log 2>&1; rc=$?; echo "bench short rc=$rc"; tail -c 1500 $O/bench_short.log; exit $rc
