# Round-2 gate b: smoke, every GPU test (incl. the n = 4000 parity tests), the parity deviation
# probe, and the default bench line (like-for-like CPU window).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -15
timeout -k 10 600 python -u scripts/parity_probe.py > $O/parity_probe.jsonl 2> $O/parity_probe.err; rc2=$?
echo "probe rc=$rc2"
timeout -k 10 900 python bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err; rc3=$?
echo "bench rc=$rc3"; cat $O/bench.json
exit $(( rc | rc2 | rc3 ))
