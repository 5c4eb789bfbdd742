#!/bin/bash
# PMC passes for the bench workload (one rocprofv3 run per counter group; no
# tracing domains combined with --pmc).  Output: gpurun_out/pmc_$TAG/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r01}
CFG=${CFG:-3}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --tile-gather-steps 0 --no-host-output --config "$CFG" ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -gt 128 ]; then exit $rc; fi
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" --config "$CFG" --tag "$TAG" > "$OUT/summary.json" && cat "$OUT/summary.json"
rc=$?
# the raw passes stay on the box unless KEEP_RAW=1 (gpurun merges back at most 64 MiB)
[ "${KEEP_RAW:-0}" = 1 ] || rm -rf "$OUT"/p[0-9]*
exit $rc
