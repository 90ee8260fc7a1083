# round 6: tridiagonal exchange pacing A/B (RIPTRM_TRI_SLEEP) with the hop trace, then the tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6tri13}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('avg_launch_us'))"; }
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
for SL in 1 4 12 30; do
  RIPTRM_TRI_SLEEP=$SL RIPTRM_TRI_STAMPS=2 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/hops_$SL.json 2> $O/hops_$SL.err || exit 1
  echo "sleep $SL: $(grep 'tri hops' $O/hops_$SL.err | head -2 | tail -1)"
  RIPTRM_TRI_SLEEP=$SL RIPTRM_TRI_STAMPS=1 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/st_$SL.json 2> $O/st_$SL.err || exit 1
  echo "sleep $SL: $(grep 'tri stamps' $O/st_$SL.err | head -2 | tail -1)"
  RIPTRM_TRI_SLEEP=$SL timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_$SL.json 2> $O/e1000_$SL.err && v $O/e1000_$SL.json || exit 1
done
timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200.json 2> $O/e200.err && v $O/e200.json &&
RIPTRM_EIG_TRI=1 timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200_tri.json 2> $O/e200_tri.err && v $O/e200_tri.json &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py -m gpu -v -s --timeout 600 --timeout-method thread -k "test_gpu_trs or exact_repmat or cg_skip" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
exit $rc
