#!/bin/bash
# In-process A/B of kernel variants: tools/ab_bench.py <variants.json> [rounds] [config]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_bench.py "$(cat ${AB_FILE:-tools/ab/shadow_variants.json})" ${AB_ROUNDS:-3} ${AB_CFG:-3} > gpurun_out/ab.txt 2>&1
rc=$?; cat gpurun_out/ab.txt; exit $rc
