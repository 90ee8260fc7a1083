# Same-box A/B of the HBM Exact_RepMat eigensolver choice (RIPTRM_BIG_EIG: d = batched dsyevd,
# s = one rocsolver_dsyevd call per matrix, j / dj = rocSOLVER's Jacobi solvers).
#   OUT=r4x EIGS="d s" SHAPES="1000:1 1000:4 200:64" bash scripts/ab_exact.sh
# VAR names another knob to alternate instead (e.g. VAR=RIPTRM_CG_LDS EIGS="1 0").
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-ab_exact}; mkdir -p $O
for sh in ${SHAPES:-1000:1 200:64}; do
  n=${sh%%:*}; b=${sh##*:}
  for r in 1 2; do
    for e in ${EIGS:-d s}; do
      env ${VAR:-RIPTRM_BIG_EIG}=$e timeout -k 10 300 python bench.py --trs Exact_RepMat --dim $n --batch $b --steps 3 --warmup 1 --cpu-budget 0 \
        > $O/exact_${n}_${b}_${e}_$r.json 2> $O/exact_${n}_${b}_${e}_$r.err || { tail $O/exact_${n}_${b}_${e}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/exact_${n}_${b}_${e}_$r.json')); print('n=$n b=$b eig=$e run $r', round(d['value'], 2), round(d['ms_per_step'], 2))"
    done
  done
done
