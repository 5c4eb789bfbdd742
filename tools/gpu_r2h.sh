# upper bound of a smaller shadow map: the frame with the shadow pass storing (almost) nothing (diag 4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2h; mkdir -p $O
for c in 3 2; do for d in 0 4 0 4; do
RTM_DIAG_SHADOW=$d timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --no-alt --tile-gather-steps 0 --no-host-output > $O/b${c}_d$d.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b${c}_d$d.log; exit $rc; }
python -c "
import json
d=json.loads([l for l in open('$O/b${c}_d$d.log') if l.startswith('{')][0])
print('config $c diag $d', d['value'], d['ms_per_frame'], d['kernels'], (d.get('kernels_in_lanes') or {}))"
done; done
