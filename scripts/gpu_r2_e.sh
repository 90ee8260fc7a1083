# Round-2 gate e: smoke, every GPU test, the headline bench (like-for-like CPU window) and the
# configs[1] bench (persistent mode), each step under its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -15
timeout -k 10 900 python bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err; rc2=$?
echo "bench rc=$rc2"; head -c 400 $O/bench.json; echo
timeout -k 10 300 python bench.py --dim 1000 --batch 1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err; rc3=$?
echo "bench cfg1 rc=$rc3"; head -c 400 $O/bench_cfg1.json; echo
exit $(( rc | rc2 | rc3 ))
