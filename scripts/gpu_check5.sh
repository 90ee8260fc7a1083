set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_sym.json 2> gpurun_out/bench_sym.err; rc=$?
echo "bench sym rc=$rc"; cat gpurun_out/bench_sym.json; tail -3 gpurun_out/bench_sym.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --dim 1000 --batch 8 --steps 45 --warmup 2 --cpu-budget 0 > gpurun_out/bench_cycle.json 2> gpurun_out/bench_cycle.err; rc=$?
echo "bench cycle rc=$rc"; cat gpurun_out/bench_cycle.json
exit $rc
