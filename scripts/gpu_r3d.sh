# Round 3: bitwise-preserving tCG reduction fusion (model + r_r): persistent vs lock-step bitwise,
# configs[1] bench + trace, then the parity suite
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_failure.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/t1.log 2>&1; rc=$?
echo "t1 rc=$rc"; grep -E "passed|failed" $O/t1.log | tail -3
[ $rc -eq 0 ] || exit $rc
for m in 1 1; do
  timeout -k 10 120 python bench.py --dim 1000 --batch 1 --cpu-budget 0 >> $O/cfg1.jsonl 2>> $O/cfg1.err || exit $?
done
python -c "
import json
for l in open('$O/cfg1.jsonl'):
    d = json.loads(l); print('cfg1', d['value'], d['roofline'].get('us_per_pass'))"
timeout -k 10 120 python scripts/persist_trace.py > $O/trace.txt 2>&1 || exit $?
tail -12 $O/trace.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_n4000.py tests/test_gpu_parity.py tests/test_gpu_stiefel.py \
  -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/t2.log 2>&1; rc=$?
echo "t2 rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|classified|excursions" $O/t2.log | tail -70
exit $rc
