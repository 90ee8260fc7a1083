# Round-1 final evidence: smoke, every GPU test, PMC traffic passes of the S-pass, the default bench
# line (with that traffic) and rocprofv3 kernel stats of the same command.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r1d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python bench.py --cpu-budget 0 --steps 8 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.log; rc=$?
echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python bench.py --cpu-budget 0 --steps 8 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.log; rc=$?
echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
python scripts/pmc_summarize.py $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv \
  $O/pmc_summary.json $O/pmc_gemv.json --n 4000 --batch 128 --instances 64 \
  --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python bench.py --cpu-budget 0 --steps 8 --warmup 1"
timeout -k 10 600 python bench.py --traffic-json $O/pmc_gemv.json > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --cpu-budget 0 --traffic-json $O/pmc_gemv.json > $O/prof_bench.json 2> $O/prof.log; rc=$?
echo "rocprof rc=$rc"; cat $O/prof_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --cpu-budget 0 --spass-kind 2 > $O/bench_super_forced.json 2> $O/bench_super_forced.err; rc=$?
echo "bench (super-tile forced) rc=$rc"; cat $O/bench_super_forced.json
exit $rc
