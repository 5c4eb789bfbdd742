#!/bin/bash
# In-process A/B of kernel variants: tools/ab_bench.py <variants> [rounds] [config].
# AB_SET names a variant set of tools/ab_variants.json (the sets used for the A/Bs
# recorded under profiles/); AB_FILE a JSON file of variants instead.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${AB_FILE:-}" ]; then
  V=$(cat "$AB_FILE")
else
  V=$(python -c "import json,sys; print(json.dumps(json.load(open('tools/ab_variants.json'))[sys.argv[1]]))" "${AB_SET:-shadow_variants}")
fi
timeout -k 10 600 python tools/ab_bench.py "$V" ${AB_ROUNDS:-3} ${AB_CFG:-3} > gpurun_out/ab.txt 2>&1
rc=$?; cat gpurun_out/ab.txt; exit $rc
