# Round 3: parity suite with the envelope bar (n = 4000 K = 20, B = 128 K = 5, Stiefel (200,50)x256)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest ${@:-tests/test_gpu_n4000.py tests/test_gpu_parity.py tests/test_gpu_stiefel.py} \
  -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|classified|excursions" $O/tests.log | tail -60
exit $rc
