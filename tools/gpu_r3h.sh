#!/bin/bash
# Pulled batch tables (pull_kernel) vs the async copy: GPU tests, then bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02_v10
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02_v10/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r02_v10/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFGS="3 2 7" VARIANTS="X=1 RTM_BATCH_COPY=copy RTM_BATCH=8 RTM_BATCH=16" TAG=r02_v10ab bash tools/gpu_r3d.sh
