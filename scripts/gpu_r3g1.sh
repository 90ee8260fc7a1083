# Round 3 final gate, part 1: the whole GPU test suite as the driver runs it, plus smoke().
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3g1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
exit $rc
