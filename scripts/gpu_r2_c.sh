# Round-2 gate c: the persistent lock-step mode first (fast fail), then every GPU test, then the
# configs[1] bench (n = 1000, one instance) with and without it, and a rocprofv3 stats of it.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_persistent.py -x -v --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1; rc=$?
echo "persistent tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/persist_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dim 1000 --batch 1 --cpu-budget 0 > $O/bench_cfg1.json 2> $O/bench_cfg1.err; rc=$?
echo "bench cfg1 rc=$rc"; cat $O/bench_cfg1.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -15
exit $rc
