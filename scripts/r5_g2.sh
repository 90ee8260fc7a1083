set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1700 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu -s \
  "tests/test_gpu_si_scaled.py::test_si_scaled_trajectory_matches_oracle" \
  "tests/test_gpu_parity.py::test_batched_solve_matches_oracle" \
  "tests/test_gpu_parity.py::test_shared_multistart_solve_matches_oracle" \
  "tests/test_gpu_parity.py::test_exact_repmat_lds_and_hbm_paths_agree_near_97" tests/test_gpu_n4000.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
