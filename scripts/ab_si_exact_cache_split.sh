# SI d=8 Exact A/B: keyed cache and split eigensolver on/off, plus a rocprofv3 summary of the default
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-absi}
mkdir -p $O
export TMPDIR=/tmp
run() {
  env $2 timeout -k 10 300 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 \
    > $O/si_$1.json 2> $O/si_$1.err || { tail $O/si_$1.err; return 1; }
  python -c "import json; d=json.load(open('$O/si_$1.json')); print('$1', d['value'], d['detail']['trs_cache_hits_subproblems'])"
}
run default "RIPTRM_X=1" && run nocache "RIPTRM_SI_CACHE=0" && run nosplit "RIPTRM_EIG_SPLIT=0" && run neither "RIPTRM_SI_CACHE=0 RIPTRM_EIG_SPLIT=0" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python bench.py --problem si --si-dim 8 \
  --trs Exact_RepMat --batch 64 --cpu-budget 0 --steps 6 > $O/prof.json 2> $O/prof.log || exit 1
RIPTRM_SI_CACHE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof0 -o p -- python bench.py --problem si --si-dim 8 \
  --trs Exact_RepMat --batch 64 --cpu-budget 0 --steps 6 > $O/prof0.json 2> $O/prof0.log || exit 1
find $O -name "*kernel_trace.csv" -delete
echo done
