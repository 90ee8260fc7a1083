# rocprofv3 of the Exact_RepMat line at configs[1]'s size (n = 1000, one instance, class defaults)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-p1000}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1000 -o p -- python bench.py --trs Exact_RepMat \
  --dim 1000 --batch 1 --steps 3 --warmup 1 --cpu-budget 0 > $O/b1000.json 2> $O/b1000.log || { tail $O/b1000.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
python - <<PY
import csv
rows=list(csv.DictReader(open("$O/p1000/p_kernel_stats.csv")))
tot=sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot/1e6,1))
for r in rows[:15]:
    print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.1f} pct {float(r["Percentage"]):5.1f}')
PY
