#!/bin/bash
# In-process A/B of kernel variants: tools/ab_bench.py <variants> [rounds] [config].
# AB_FILE: a JSON file of variants ({"name": {"env": {"RTM_LIB": "__ROOT__/..."}}}: builds
# of the library side by side; the product library has no A/B switches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$(cat "${AB_FILE:?AB_FILE: a JSON file of variants}")
timeout -k 10 600 python tools/ab_bench.py "$V" ${AB_ROUNDS:-3} ${AB_CFG:-3} > gpurun_out/ab.txt 2>&1
rc=$?; cat gpurun_out/ab.txt; exit $rc
