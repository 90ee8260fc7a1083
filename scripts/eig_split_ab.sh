# split eigensolver timing (m = 100, 199) + the TRS eigensolver tests + the two Exact benches
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-eigab}
mkdir -p $O
export TMPDIR=/tmp
for m in 100 199; do
  timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/split.txt 2>&1 || { tail $O/split.txt; exit 1; }
done
grep "compact:\|values:" $O/split.txt | awk 'NR%3==0'
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "sym_eig or above_lds or hard_case" tests/test_gpu_trs.py > $O/trs.log 2>&1 || { tail -30 $O/trs.log; exit 1; }
tail -1 $O/trs.log
timeout -k 10 600 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/si.json 2> $O/si.err || { tail $O/si.err; exit 1; }
timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/e200.json 2> $O/e200.err || { tail $O/e200.err; exit 1; }
python -c "import json; print('si', json.load(open('$O/si.json'))['value'], 'exact200', json.load(open('$O/e200.json'))['value'])"
