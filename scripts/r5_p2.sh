# exact tests on the default eigensolver, then the Exact profiles and the SI d=8 Exact line
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "exact or Exact or sym_eig or above_lds or hard_case" \
  tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/exact_tests.log 2>&1 || { tail -60 $O/exact_tests.log; exit 1; }
tail -1 $O/exact_tests.log
OUT=${OUT:-r5q} STEPS="si_d8_exact_prof si_d8_exact" bash scripts/gate.sh
