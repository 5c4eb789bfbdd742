# coded shadow map: new tests, full GPU suite, A/B benches (coded vs RTM_SMAP=f64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_smap_codes.py tests/test_gpu_parity.py -k "smap or shadow_map or lean_shadow or general" -m gpu -p no:cacheprovider > $O/pytest_smap.log 2>&1
rc=$?; echo "pytest smap rc=$rc"; tail -5 $O/pytest_smap.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in 3 2 5 7; do for m in coded f64 coded f64; do
if [ $m = f64 ]; then export RTM_SMAP=f64; else unset RTM_SMAP; fi
timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output > $O/b${c}_$m.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b${c}_$m.log; exit $rc; }
python -c "
import json
d=json.loads([l for l in open('$O/b${c}_$m.log') if l.startswith('{')][0])
print('config $c $m', d['value'], d['ms_per_frame'], d['kernels'], (d.get('one_lane') or {}).get('value'))"
done; done
