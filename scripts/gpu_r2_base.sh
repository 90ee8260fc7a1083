# Round-2 baseline on a fresh box: smoke, GPU tests, headline bench, configs[1] bench.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dim 1000 --batch 1 --cpu-budget 0 > $O/bench_cfg1.json 2> $O/bench_cfg1.err; rc=$?
echo "bench cfg1 rc=$rc"; cat $O/bench_cfg1.json
exit $rc
