# round 6: the tridiagonal update's loop order (columns outer, default, vs rows outer: RIPTRM_TRI_UPD=r),
# same box: phase stamps at m = 999 and the reduction's time at 199 x 64 / 999 x 1
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6upd}; mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('avg_launch_us'))"; }
for U in c r c r; do
  RIPTRM_TRI_UPD=$U RIPTRM_TRI_STAMPS=1 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/st_$U.json 2> $O/st_$U.err || exit 1
  echo "upd $U: $(grep 'tri stamps' $O/st_$U.err | head -2 | tail -1)"
  RIPTRM_TRI_UPD=$U timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200_$U.json 2> $O/e200_$U.err && v $O/e200_$U.json || exit 1
  RIPTRM_TRI_UPD=$U timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_$U.json 2> $O/e1000_$U.err && v $O/e1000_$U.json || exit 1
done
