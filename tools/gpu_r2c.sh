# f-1 parity + config 6/7 bench (round 2, step c)
set -o pipefail
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_raytrace.py tests/test_perspective.py tests/test_formats_group.py tests/test_cli.py tests/test_sdf.py -m gpu -p no:cacheprovider > gpurun_out/r2c/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2c/pytest.log
[ $rc -ne 0 ] && exit $rc
for c in 6 7; do
timeout -k 10 300 python -u bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --no-alt --tile-gather-steps 0 > gpurun_out/r2c/bench$c.log 2>&1
rc=$?; echo "bench$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r2c/bench$c.log; exit $rc; }
python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/r2c/bench$c.log') if l.startswith('{')][0])
print($c, d['value'], d['kernels'], d['roofline']['bound'], d['roofline']['frac'])"
done
