# PMC passes of config 6 (row f-1 eye pass) + asm resource usage
set -o pipefail
export TMPDIR=/tmp
TAG=r02_f1a CFG=6 BENCH_ARGS="--no-alt --tile-gather-steps 0 --preroll-ms 0" timeout -k 10 900 bash tools/profile_pmc.sh > gpurun_out/r2d_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -60 gpurun_out/r2d_pmc.log
exit $rc
