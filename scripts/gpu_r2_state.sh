# State-kernel change check: n = 4000 parity tests, the shared-layout bench under kernel stats, and
# the headline bench (no CPU leg), each under its own limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_n4000.py tests/test_gpu_parity.py -k "n4000 or shared or batched" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --layout shared --cpu-budget 0 > $O/bench_shared.json 2> $O/rocprof.log; rc=$?
echo "shared rc=$rc"; head -c 250 $O/bench_shared.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/bench_head.json 2> $O/bench_head.err; rc=$?
echo "head rc=$rc"; head -c 250 $O/bench_head.json; echo
exit $rc
