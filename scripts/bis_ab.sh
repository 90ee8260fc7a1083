# A/B of the bisection's eigenvalues per workgroup (RIPTRM_EIG_BIS=n; default ~25 up to order 128,
# ~50 above): eigensolver timing at m = 100 / 199 and the two Exact benches per setting, then the
# TRS eigensolver and SI Exact GPU tests on the default
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-bisab}
mkdir -p $O
export TMPDIR=/tmp
for v in ${BIS:-13 25 50}; do
  export RIPTRM_EIG_BIS=$v
  for m in 100 199; do
    timeout -k 10 120 python scripts/eig_stamps.py $m 64 > $O/eig_${v}_$m.txt 2>&1 || { tail $O/eig_${v}_$m.txt; exit 1; }
    echo "bis $v: $(grep 'compact:\|values:' $O/eig_${v}_$m.txt | tail -2 | tr '\n' ' ')"
  done
  timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si_$v.json 2> $O/si_$v.err || { tail $O/si_$v.err; exit 1; }
  timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/e200_$v.json 2> $O/e200_$v.err || { tail $O/e200_$v.err; exit 1; }
  python -c "import json; print('bis $v si d8 exact', json.load(open('$O/si_$v.json'))['value'], 'exact200', json.load(open('$O/e200_$v.json'))['value'])"
done
unset RIPTRM_EIG_BIS
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trs.py tests/test_gpu_si_scaled.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
