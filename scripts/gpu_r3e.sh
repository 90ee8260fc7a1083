# Round 3: Exact_RepMat above dim 96 (HBM path, rocSOLVER dsyevd)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/test_gpu_trs.py "tests/test_gpu_parity.py::test_exact_repmat_reference_defaults_drop_in" \
  "tests/test_gpu_parity.py::test_exact_repmat_above_lds_size_matches_oracle" "tests/test_gpu_parity.py::test_exact_repmat_configs1_size_drop_in" \
  -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
echo "t rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $O/t.log | tail -40
exit $rc
