# CG-skip neutrality + SI d=8 Exact tests, then the SI d=8 Exact bench (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "exact or Exact" \
  tests/test_gpu_si_scaled.py tests/test_gpu_si.py > $O/si_exact_tests.log 2>&1 || { tail -60 $O/si_exact_tests.log; exit 1; }
tail -1 $O/si_exact_tests.log
timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 \
  > $O/bench_si_d8_exact.json 2> $O/bench_si_d8_exact.err || { tail $O/bench_si_d8_exact.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_si_d8_exact.json')); print('si d8 exact', d['value'], d['detail']['trs_cg_checked_skipped'])"
