set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_sym.json 2> gpurun_out/bench_sym.err; rc=$?
echo "bench sym rc=$rc"; cat gpurun_out/bench_sym.json; tail -3 gpurun_out/bench_sym.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --layout full --cpu-budget 0 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?
echo "bench full rc=$rc"; cat gpurun_out/bench_full.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sym -o bench -- python bench.py --cpu-budget 0 > gpurun_out/prof_sym.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_sym.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o fetch -- python bench.py --cpu-budget 0 --steps 8 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; tail -2 gpurun_out/pmc_fetch.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o write -- python bench.py --cpu-budget 0 --steps 8 --warmup 1 > gpurun_out/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"; tail -2 gpurun_out/pmc_write.log
find gpurun_out/prof_sym gpurun_out/pmc_fetch gpurun_out/pmc_write -type f | head -20
exit $rc
