# full GPU suite + benches of configs 2, 3, 7 (batching), 6 (round 2, step e)
set -o pipefail
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "batch or lanes" -m gpu -p no:cacheprovider > gpurun_out/r2e/pytest_batch.log 2>&1 && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/r2e/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r2e/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for c in 7 2 3; do
timeout -k 10 300 python -u bench.py --config $c --steps 2000 --warmup 200 --no-cpu-baseline --tile-gather-steps 0 --no-host-output > gpurun_out/r2e/bench$c.log 2>&1
rc=$?; echo "bench$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r2e/bench$c.log; exit $rc; }
python -c "
import json
d=json.loads([l for l in open('gpurun_out/r2e/bench$c.log') if l.startswith('{')][0])
print($c, d['value'], d['kernels'], d['frames_per_launch'], d['lanes'], d['roofline_frame']['frac'], (d.get('alt_fused_shadow') or {}).get('value'))"
done
