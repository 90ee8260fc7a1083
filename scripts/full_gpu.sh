# The round-end GPU tiers as the driver runs them: smoke, then the whole -m gpu suite (timed).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-full}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
start=$(date +%s)
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1
rc=$?
echo "suite rc=$rc wall=$(( $(date +%s) - start ))s"
tail -40 $O/gpu_tests.log
exit $rc
