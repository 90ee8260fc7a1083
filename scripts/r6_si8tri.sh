# round 6: StableIdentification d = 8 Exact (manifold.dim 100) on the eigensolver path vs the tridiagonal
# path (RIPTRM_TRI_MIN=96), and the n = 130 NonnegPCA Exact line (order 129) the same way
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6si8}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'))"; }
for T in 200 96 200 96; do
  RIPTRM_TRI_MIN=$T timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 --cpu-procs 0 \
    > $O/si8_$T.json 2> $O/si8_$T.err && v $O/si8_$T.json || exit 1
  RIPTRM_TRI_MIN=$T timeout -k 10 300 python bench.py --trs Exact_RepMat --dim 130 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 \
    --cpu-procs 0 > $O/e130_$T.json 2> $O/e130_$T.err && v $O/e130_$T.json || exit 1
done
