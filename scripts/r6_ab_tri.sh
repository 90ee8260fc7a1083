# round 6 A/B of the tridiagonal path: the Exact_RepMat lines with the default (riptrm_tri.h above order
# 199) vs RIPTRM_BIG_EIG=r (rocSOLVER dsyevd), and the hand-written eigensolver's first phase on the chip
# (RIPTRM_EIG_TRI=1) vs one workgroup per matrix, same box; then rocprofv3 of the n = 1000 line
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6ab}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2))"; }
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0"
timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_tri.json 2> $O/e1000_tri.err && v $O/e1000_tri.json &&
RIPTRM_BIG_EIG=r timeout -k 10 300 $B --dim 1000 --batch 1 --steps 3 --warmup 1 > $O/e1000_r.json 2> $O/e1000_r.err && v $O/e1000_r.json &&
timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200.json 2> $O/e200.err && v $O/e200.json &&
RIPTRM_EIG_TRI=1 timeout -k 10 300 $B --dim 200 --batch 64 --steps 4 --warmup 1 > $O/e200_tri.json 2> $O/e200_tri.err && v $O/e200_tri.json &&
timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 --cpu-procs 0 > $O/si8.json 2> $O/si8.err && v $O/si8.json &&
RIPTRM_EIG_TRI=1 timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 --cpu-procs 0 > $O/si8_tri.json 2> $O/si8_tri.err && v $O/si8_tri.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1000 -o p -- python bench.py --trs Exact_RepMat \
  --dim 1000 --batch 1 --steps 3 --warmup 1 --cpu-budget 0 --cpu-procs 0 > $O/e1000_prof.json 2> $O/e1000_prof.err && v $O/e1000_prof.json &&
find $O -name "*kernel_trace.csv" -delete &&
python - <<PY
import csv
rows=list(csv.DictReader(open("$O/p1000/p_kernel_stats.csv")))
tot=sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot/1e6,1))
for r in rows[:12]:
    print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.1f} pct {float(r["Percentage"]):5.1f}')
PY
