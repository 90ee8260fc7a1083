# Round 3: k_persist lean-pass exchange in two hops (default build) vs every replica gathering all
# partial sums (libriptrm_hip_x1.so, -DRIPTRM_PERSIST_XCHG=1): persistent tests (bitwise vs
# lock-step), configs[1] A/B on one box, device-clock trace of the new build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_failure.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $O/t1.log 2>&1; rc=$?
echo "t1 rc=$rc"; grep -E "passed|failed" $O/t1.log | tail -3
[ $rc -eq 0 ] || exit $rc
PKG=riemannian-interior-point-trust-region-method_amd
for v in x2 x1 x2 x1; do
  if [ $v = x1 ]; then export RIPTRM_LIB=$GRAFT_REPO_ROOT/$PKG/libriptrm_hip_x1.so; else unset RIPTRM_LIB; fi
  timeout -k 10 120 python bench.py --dim 1000 --batch 1 --cpu-budget 0 > $O/cfg1_$v.json 2>> $O/cfg1.err || exit $?
  python -c "import json; d=json.load(open('$O/cfg1_$v.json')); print('$v', round(d['value'],2), d['roofline'].get('us_per_pass'))"
  cat $O/cfg1_$v.json >> $O/ab.jsonl
done
unset RIPTRM_LIB
timeout -k 10 120 python scripts/persist_trace.py > $O/trace.txt 2>&1 || exit $?
tail -4 $O/trace.txt
