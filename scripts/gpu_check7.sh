set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "shared or run_batch" > gpurun_out/gpu_tests_shared.log 2>&1; rc=$?
echo "pytest shared rc=$rc"; tail -15 gpurun_out/gpu_tests_shared.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --layout shared --cpu-budget 0 > gpurun_out/bench_shared.json 2> gpurun_out/bench_shared.err; rc=$?
echo "bench shared rc=$rc"; cat gpurun_out/bench_shared.json; tail -3 gpurun_out/bench_shared.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest all rc=$rc"; tail -5 gpurun_out/gpu_tests.log
exit $rc
