# round 6 final: every -m gpu test except tests/test_gpu_n4000.py (order 4000: the rocSOLVER path, 7 min,
# profiles/r6_gpu_tests_n4000.log), smoke(), and the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6full}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --ignore=tests/test_gpu_n4000.py \
  > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && tail -1 $O/bench.json
