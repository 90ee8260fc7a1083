# eigensolver A/B: 512 vs 1024 threads per matrix (stamps, TRS tests, exact tests, exact bench)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5n}
mkdir -p $O
export TMPDIR=/tmp
for t in 512 1024; do
  for m in 100 199; do
    echo "threads $t" >> $O/stamps.txt
    RIPTRM_EIG_THREADS=$t RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
  done
done
grep -v "^/opt" $O/stamps.txt | grep -v "values\|vectors:" 
RIPTRM_EIG_THREADS=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "sym_eig or above_lds or hard_case" tests/test_gpu_trs.py > $O/trs1024.log 2>&1 || { tail -30 $O/trs1024.log; exit 1; }
tail -1 $O/trs1024.log
OUT=${OUT:-r5n} bash scripts/r5_g3.sh
RIPTRM_EIG_THREADS=1024 timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 \
  > $O/bench_exact_200_t1024.json 2> $O/bench_exact_t1024.err || { tail $O/bench_exact_t1024.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_exact_200_t1024.json')); print('exact200 t1024', d['value'])"
