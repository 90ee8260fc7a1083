# round 6: k_refl_blk's L2 prefetch workgroups (RIPTRM_TRI_REFL_HELPERS) A/B at m = 999 (phase clocks +
# the n = 1000 Exact line), then the tridiagonal-path tests at the default
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6help}; mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0 --dim 1000 --batch 1"
for H in ${HS:-0 1 2 4}; do
  RIPTRM_TRI_REFL_HELPERS=$H RIPTRM_TRI_STAMPS=3 timeout -k 10 120 $B --steps 1 --warmup 1 > $O/st$H.json 2> $O/st$H.err || exit 1
  echo "H=$H $(grep 'refl stamps' $O/st$H.err | sort | uniq -c | sort -rn | head -2 | tr '\n' ' ')"
  RIPTRM_TRI_REFL_HELPERS=$H timeout -k 10 200 $B --steps 3 --warmup 1 > $O/e$H.json 2> $O/e$H.err || exit 1
  python -c "import json; d=json.loads(open('$O/e$H.json').read().strip().splitlines()[-1]); print('  H=$H value', round(d['value'],2))"
done
[ "${TESTS:-1}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py -m gpu -v -s --timeout 600 \
  --timeout-method thread -k "test_gpu_trs or exact_repmat or cg_skip or hbm" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
exit $rc
