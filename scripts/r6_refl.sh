# round 6: the blocked reflector application's phase clocks (RIPTRM_TRI_STAMPS=3) at m = 999
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6refl}; mkdir -p $O
RIPTRM_TRI_STAMPS=3 timeout -k 10 120 python bench.py --trs Exact_RepMat --cpu-budget 0 --cpu-procs 0 --dim 1000 --batch 1 --steps 1 \
  --warmup 1 > $O/st.json 2> $O/st.err || exit 1
grep "refl stamps" $O/st.err | sort | uniq -c | sort -rn | head -6
