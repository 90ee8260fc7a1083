set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_trs.py > $O/trs_tests.log 2>&1 || { tail -60 $O/trs_tests.log; exit 1; }
tail -2 $O/trs_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -k "exact or Exact" \
  tests/test_gpu_parity.py tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/exact_tests.log 2>&1 || { tail -60 $O/exact_tests.log; exit 1; }
tail -2 $O/exact_tests.log
timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 \
  > $O/bench_exact_200.json 2> $O/bench_exact.err || { tail $O/bench_exact.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_exact_200.json')); print('exact200', d['value'], d['detail'].get('trs_cache'))"
RIPTRM_BIG_EIG=r timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 \
  > $O/bench_exact_200_rocsolver.json 2> $O/bench_exact_r.err || { tail $O/bench_exact_r.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_exact_200_rocsolver.json')); print('exact200 rocsolver', d['value'])"
