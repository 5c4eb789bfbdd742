set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2n; mkdir -p $O
bash tools/ab_env.sh $O "3 2" "RTM_LANES=2;RTM_LANES=3;RTM_LANES=4;RTM_LANES=5" 1 && \
bash tools/ab_env.sh $O/c69 "6 9" "-" 1
