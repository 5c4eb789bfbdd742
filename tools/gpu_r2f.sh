set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2f
timeout -k 10 200 python -u tools/probes/batch_probe.py --config 7 > gpurun_out/r2f/c7.log 2>&1; rc=$?; cat gpurun_out/r2f/c7.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/probes/batch_probe.py --config 2 --lanes 1,3 --batches 1,2,4 > gpurun_out/r2f/c2.log 2>&1; rc=$?; cat gpurun_out/r2f/c2.log; exit $rc
