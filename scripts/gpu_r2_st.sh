# Stiefel kernels: GPU tests, the (200,50) x 256 bench, and its rocprofv3 kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2st}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stiefel.py > $O/tests.log 2>&1; rc=$?
tail -12 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json; tail -3 $O/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > $O/bench_rocprof.json 2> $O/rocprof.log; rc=$?
echo "rocprof rc=$rc"
exit $rc
