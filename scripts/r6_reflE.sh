# round 6: k_refl_blk with one element per thread (1024 threads, RIPTRM_TRI_REFL_E=1) against two (512):
# phase clocks at m = 999, the n = 1000 / n = 200 x 64 Exact lines, the tridiagonal-path tests under E=1
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6reflE}; mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
for E in 2 1; do
  RIPTRM_TRI_REFL_E=$E RIPTRM_TRI_STAMPS=3 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/st$E.json 2> $O/st$E.err || exit 1
  echo "E=$E $(grep 'refl stamps' $O/st$E.err | sort | uniq -c | sort -rn | head -1)"
  RIPTRM_TRI_REFL_E=$E timeout -k 10 200 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_$E.json 2> $O/e1000_$E.err || exit 1
  RIPTRM_TRI_REFL_E=$E timeout -k 10 200 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200_$E.json 2> $O/e200_$E.err || exit 1
  python -c "import json; f=lambda p: round(json.loads(open(p).read().strip().splitlines()[-1])['value'],2); print('  E=$E e1000', f('$O/e1000_$E.json'), 'e200', f('$O/e200_$E.json'))"
done
RIPTRM_TRI_REFL_E=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_trs.py tests/test_gpu_parity.py -m gpu -v -s --timeout 600 \
  --timeout-method thread -k "test_gpu_trs or exact_repmat or cg_skip" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
exit $rc
