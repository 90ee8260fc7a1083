# Round 3 gate after the Stiefel blocked factor: smoke, the full GPU suite, Stiefel bench under rocprofv3
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3g4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python bench.py --problem stiefel --dim 200 --batch 256 --cpu-budget 20 > $O/bench_stiefel_rocprof.json 2> $O/st_rocprof.log || exit $?
echo "stiefel rocprof ok"
timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 2048 --cpu-budget 20 > $O/bench_stiefel_2048.json 2> $O/st2048.err || exit $?
echo done
