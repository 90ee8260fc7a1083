# A/B of the S-pass unit order (static vs ticket counter) on the headline bench, plus the n = 4000
# and persistent parity tests with the new default; each step under its own limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2dyn}
mkdir -p $O
export TMPDIR=/tmp
RIPTRM_SUP_DYNAMIC=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_n4000.py tests/test_gpu_parity.py -k "n4000 or batched or spass or layouts" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
RIPTRM_SUP_DYNAMIC=0 timeout -k 10 400 python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/bench_static.json 2> $O/bench_static.err; rc=$?
echo "static rc=$rc"; head -c 200 $O/bench_static.json; echo
[ $rc -eq 0 ] || exit $rc
RIPTRM_SUP_DYNAMIC=1 timeout -k 10 400 python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/bench_dyn.json 2> $O/bench_dyn.err; rc=$?
echo "dyn rc=$rc"; head -c 200 $O/bench_dyn.json; echo
[ $rc -eq 0 ] || exit $rc
RIPTRM_SUP_DYNAMIC=0 timeout -k 10 400 python bench.py --cpu-budget 0 --warmup 5 --steps 20 > $O/bench_static2.json 2> $O/bench_static2.err; rc=$?
echo "static2 rc=$rc"; head -c 200 $O/bench_static2.json; echo
exit $rc
