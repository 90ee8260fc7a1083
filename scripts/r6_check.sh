# round 6: after moving the tridiagonal path's lower bound to order 150 -- the Exact tests (trs, NonnegPCA
# Exact solves, CG-skip neutrality, the SI HBM service) and the n = 200 x 64 / n = 1000 Exact lines
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6chk}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('avg_launch_us'))"; }
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
timeout -k 10 900 python -u -m pytest tests/test_gpu_trs.py tests/test_gpu_parity.py tests/test_gpu_si_scaled.py -m gpu -v -s --timeout 600 \
  --timeout-method thread -k "test_gpu_trs or exact_repmat or cg_skip or hbm" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200.json 2> $O/e200.err && v $O/e200.json &&
timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000.json 2> $O/e1000.err && v $O/e1000.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1000 -o p -- python bench.py --trs Exact_RepMat \
  --dim 1000 --batch 1 --steps 3 --warmup 1 --cpu-budget 0 --cpu-procs 0 > $O/e1000_prof.json 2> $O/e1000_prof.err
[ -f $O/p1000/p_kernel_stats.csv ] || exit 1
find $O -name "*kernel_trace.csv" -delete
python - <<PY
import csv
rows=list(csv.DictReader(open("$O/p1000/p_kernel_stats.csv")))
for r in rows[:8]:
    print(f'  {r["Name"][:50]:50s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.1f} pct {float(r["Percentage"]):5.1f}')
PY
