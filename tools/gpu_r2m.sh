set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2m; mkdir -p $O
true

TAG=r02_v2 timeout -k 10 1000 bash tools/round_pmc.sh 3 3f 6 9
