# wave-reduction change: full GPU tests, then small/shared/SI benches
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dim 1000 --batch 8 --steps 10 --warmup 2 --cpu-budget 0 > gpurun_out/b_small.json 2>/dev/null; rc=$?; echo "small rc=$rc"; cat gpurun_out/b_small.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dim 1000 --batch 1 --steps 10 --warmup 2 --cpu-budget 0 > gpurun_out/b_one.json 2>/dev/null; rc=$?; echo "one rc=$rc"; cat gpurun_out/b_one.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --layout shared --cpu-budget 0 > gpurun_out/b_shared.json 2>/dev/null; rc=$?; echo "shared rc=$rc"; cat gpurun_out/b_shared.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --problem si --batch 256 --steps 20 --cpu-budget 0 > gpurun_out/b_si.json 2>/dev/null; rc=$?; echo "si rc=$rc"; cat gpurun_out/b_si.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --cpu-budget 0 > gpurun_out/b_head.json 2>/dev/null; rc=$?; echo "headline rc=$rc"; cat gpurun_out/b_head.json
exit $rc
