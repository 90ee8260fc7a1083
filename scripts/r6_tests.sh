# round 6: run a selection of GPU tests (-k expression in $K, or files in $F) with per-test timeouts;
# the parity tables land in gpurun_out/parity/
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6t}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 ${TO:-1100} python -u -m pytest ${F:-tests} -m gpu -v --timeout ${PT:-900} --timeout-method thread -k "${K:-}" \
  > $O/tests.log 2>&1
rc=$?
mkdir -p $O/parity && cp -r gpurun_out/parity/* $O/parity/ 2>/dev/null
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -30
exit $rc
