set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s \
  "tests/test_gpu_si_scaled.py::test_si_exact_cg_skip_is_bitwise_neutral" \
  "tests/test_gpu_distributed.py::test_bench_rccl_one_rank_matches_no_dist_bitwise" \
  "tests/test_gpu_si_scaled.py::test_si_exact_hbm_eigensolve_failure_stops_one_instance" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u scripts/dump_gpu_logs.py $O/n4000 4000 16 20 4000 > $O/dump.log 2>&1 || { tail $O/dump.log; exit 1; }
tail -2 $O/dump.log
