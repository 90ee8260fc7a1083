# every StableIdentification GPU test, then the SI fixture (tCG) and d=8 Exact benches (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-sicheck}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_si.py tests/test_gpu_si_scaled.py \
  > $O/si_tests.log 2>&1 || { tail -40 $O/si_tests.log; exit 1; }
tail -1 $O/si_tests.log
timeout -k 10 300 python bench.py --problem si --batch 256 --cpu-budget 0 > $O/si5.json 2> $O/si5.err || { tail $O/si5.err; exit 1; }
timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si8.json 2> $O/si8.err || { tail $O/si8.err; exit 1; }
python -c "import json; print('si d5 tCG', json.load(open('$O/si5.json'))['value'], 'si d8 exact', json.load(open('$O/si8.json'))['value'])"
