# Exact tests (TRS, parity, SI) on the default path, then the SI d=8 and NonnegPCA n=200 Exact benches
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "exact or Exact or sym_eig or above_lds or hard_case or trs" \
  tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/exact_tests.log 2>&1 || { tail -60 $O/exact_tests.log; exit 1; }
tail -1 $O/exact_tests.log
timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 \
  > $O/bench_si_d8_exact.json 2> $O/bench_si_d8_exact.err || { tail $O/bench_si_d8_exact.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_si_d8_exact.json')); print('si d8 exact', d['value'], d['detail']['trs_cg_checked_skipped'])"
timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 \
  > $O/bench_exact_200.json 2> $O/bench_exact.err || { tail $O/bench_exact.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_exact_200.json')); print('exact200', d['value'], d['detail'].get('trs_cache'))"
