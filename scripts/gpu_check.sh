set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --dim 1000 --batch 8 --steps 4 --warmup 1 --cpu-budget 5 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err; rc=$?
echo "bench small rc=$rc"; cat gpurun_out/bench_small.json; tail -3 gpurun_out/bench_small.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
echo "bench default rc=$rc"; cat gpurun_out/bench_default.json; tail -5 gpurun_out/bench_default.err
exit $rc
