set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2k; mkdir -p $O
RTM_LEAN_COMP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_smap_codes.py tests/test_gpu_parity.py tests/test_general_march.py -m gpu -p no:cacheprovider > $O/pytest_comp.log 2>&1
rc=$?; echo "pytest comp rc=$rc"; tail -3 $O/pytest_comp.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh $O "3 2 5" "-;RTM_LEAN_COMP=1" 2
