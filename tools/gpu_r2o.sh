set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2o; mkdir -p $O
bash tools/ab_env.sh $O "2 3" "RTM_LANES=1;RTM_LANES=2;RTM_LANES=3" 2 && \
bash tools/ab_env.sh $O/b "6 8 9 4" "RTM_LANES=1;RTM_LANES=2;RTM_LANES=3" 1
