# SI Exact: the exact-path tests (TRS service, cache / skip / prep neutrality, parity) + the d=8 bench,
# with and without k_si_prep (RIPTRM_SI_PREP=0)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-siex}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "exact or Exact" \
  tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/si_tests.log 2>&1 || { tail -40 $O/si_tests.log; exit 1; }
tail -1 $O/si_tests.log
for v in 1 0; do
  RIPTRM_SI_PREP=$v timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 \
    > $O/si_prep$v.json 2> $O/si_prep$v.err || { tail $O/si_prep$v.err; exit 1; }
  python -c "import json; print('prep=$v', json.load(open('$O/si_prep$v.json'))['value'])"
done
