# Round 3, first GPU pass: new tests (launcher, persistent fallback/concurrency, non-finite guard),
# then configs[1] A/B (cooperative vs plain k_persist launch) and the headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_failure.py tests/test_gpu_persistent.py tests/test_gpu_distributed.py \
  -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for m in 1 2 1 2; do
  timeout -k 10 120 python bench.py --dim 1000 --batch 1 --cpu-budget 0 --persistent $m >> $O/cfg1_ab.jsonl 2>> $O/cfg1.err || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/r3a/cfg1_ab.jsonl"):
    d = json.loads(l); print("cfg1", d["value"], d["roofline"].get("us_per_pass"))
PY
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'])"
exit $rc
