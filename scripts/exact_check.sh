# the Exact_RepMat path end to end: its GPU tests (TRS service, eigensolver, parity, SI) and the
# NonnegPCA n=200 x 64 and SI d=8 x 64 Exact benches (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-excheck}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "exact or Exact or sym_eig or above_lds or hard_case or trs" \
  tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/exact_tests.log 2>&1 || { tail -60 $O/exact_tests.log; exit 1; }
tail -1 $O/exact_tests.log
timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si.json 2> $O/si.err || { tail $O/si.err; exit 1; }
timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/e200.json 2> $O/e200.err || { tail $O/e200.err; exit 1; }
python -c "import json; print('si d8 exact', json.load(open('$O/si.json'))['value'], 'exact200', json.load(open('$O/e200.json'))['value'])"
