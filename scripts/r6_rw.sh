# round 6: the tridiagonal reduction with half the workgroups (RIPTRM_TRI_RW=4: four rows per wave)
# against the default, hop trace + n = 1000 Exact line + the reduction's parity test under each
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6rw}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('avg_launch_us'))"; }
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
for RW in 2 4; do
  RIPTRM_TRI_RW=$RW RIPTRM_TRI_STAMPS=2 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/hops_$RW.json 2> $O/hops_$RW.err || exit 1
  echo "rw $RW: $(grep 'tri hops' $O/hops_$RW.err | head -2 | tail -1)"
  RIPTRM_TRI_RW=$RW RIPTRM_TRI_STAMPS=1 timeout -k 10 120 $B --dim 1000 --batch 1 --steps 1 --warmup 1 > $O/st_$RW.json 2> $O/st_$RW.err || exit 1
  echo "rw $RW: $(grep 'tri stamps' $O/st_$RW.err | head -2 | tail -1)"
  RIPTRM_TRI_RW=$RW timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_$RW.json 2> $O/e1000_$RW.err && v $O/e1000_$RW.json || exit 1
  RIPTRM_TRI_RW=$RW timeout -k 10 300 python -u -m pytest tests/test_gpu_trs.py -m gpu -q --timeout 200 --timeout-method thread \
    -k "sym_tridiag or gep_above or trs_gep" > $O/t_$RW.log 2>&1 || { tail -20 $O/t_$RW.log; exit 1; }
  tail -1 $O/t_$RW.log
done
