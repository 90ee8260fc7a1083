# Full GPU gate: build, smoke, all GPU tests, default bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json
exit $rc
