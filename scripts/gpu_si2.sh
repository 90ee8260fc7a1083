set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 600 python -m pytest tests/test_gpu_si.py -q -x -m gpu > gpurun_out/gpu_si.log 2>&1; rc=$?
echo "pytest si rc=$rc"; tail -5 gpurun_out/gpu_si.log
[ $rc -eq 0 ] || exit $rc
for B in 256 4096; do
timeout -k 10 600 python bench.py --problem si --batch $B --steps 20 --warmup 1 --cpu-budget 0 > gpurun_out/bench_si_$B.json 2> gpurun_out/bench_si_$B.err; rc=$?
echo "bench si B=$B rc=$rc"; cat gpurun_out/bench_si_$B.json
[ $rc -eq 0 ] || exit $rc
done
