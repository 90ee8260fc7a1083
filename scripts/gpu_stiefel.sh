set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_gpu_stiefel.py -q -x -m gpu > gpurun_out/gpu_stiefel.log 2>&1; rc=$?
echo "pytest stiefel rc=$rc"; tail -30 gpurun_out/gpu_stiefel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --problem stiefel --dim 200 --batch 256 --steps 50 --warmup 3 > gpurun_out/bench_stiefel.json 2> gpurun_out/bench_stiefel.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_stiefel.json; tail -3 gpurun_out/bench_stiefel.err
exit $rc
