# round 6: n = 200 x 64 Exact line, the compact eigensolver's front: one workgroup per matrix (k_eig_lds)
# vs the cooperative reduction (RIPTRM_EIG_TRI=1), benches and rocprofv3 summaries of both
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6e200}; mkdir -p $O
export TMPDIR=/tmp
v() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('avg_launch_us'))"; }
B="python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0 --dim 200 --batch 64"
for T in 0 1 2; do
  E="RIPTRM_EIG_TRI=$T"; [ $T = 2 ] && E="RIPTRM_TRI_MIN=150"
  env $E timeout -k 10 300 $B --steps 4 --warmup 1 > $O/e200_$T.json 2> $O/e200_$T.err && v $O/e200_$T.json || exit 1
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p200_$T -o p -- python bench.py \
    --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0 --dim 200 --batch 64 --steps 3 --warmup 1 > $O/prof_$T.json 2> $O/prof_$T.err
  [ -f $O/p200_$T/p_kernel_stats.csv ] || exit 1
  find $O -name "*kernel_trace.csv" -delete
  python - <<PY
import csv
rows=list(csv.DictReader(open("$O/p200_$T/p_kernel_stats.csv")))
print("$E total ms", round(sum(float(r["TotalDurationNs"]) for r in rows)/1e6,1))
for r in rows[:10]:
    print(f'  {r["Name"][:50]:50s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.1f} pct {float(r["Percentage"]):5.1f}')
PY
done
