#!/bin/bash
# PMC passes (tools/profile_pmc.sh) for a list of bench configurations, one after
# another; stops at the first fatal exit.  Usage: TAG=r02_v1 bash tools/round_pmc.sh 3 3f 6 9
# ("3f": config 3 with --fused, the fused-shadow frame)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02_v1}
for c in "$@"; do
  if [ "${c%f}" != "$c" ]; then cfg=${c%f}; args="--fused --no-alt"; tag=${TAG}_fused; else cfg=$c; args="--no-alt"; tag=$TAG; fi
  echo "=== pmc config $cfg ($args) $(date +%T)"
  TAG=${tag}_c$cfg CFG=$cfg BENCH_ARGS="$args" bash tools/profile_pmc.sh > /dev/null 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  cp "gpurun_out/pmc_${tag}_c$cfg/summary.json" "gpurun_out/pmc_${tag}_c$cfg.summary.json"
  # the raw per-dispatch CSVs are large (gpurun copies back at most 64 MiB): keep the summary and logs
  rm -rf "gpurun_out/pmc_${tag}_c$cfg"/p[0-9]*/
done
echo done
