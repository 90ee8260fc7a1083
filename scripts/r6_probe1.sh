# round 6 first measurements: rocprofv3 of the Exact n=1000 line and the
# configs[1] persistent pass trace (item 6 baseline)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6p1}; mkdir -p $O
export TMPDIR=/tmp
OUT=$(basename $O) bash scripts/prof_exact1000.sh > $O/prof_exact1000.txt 2>&1 || { cat $O/prof_exact1000.txt; exit 1; }
cat $O/prof_exact1000.txt
timeout -k 10 200 python scripts/persist_trace.py 1000 1 > $O/persist_trace.txt 2>&1 || { tail $O/persist_trace.txt; exit 1; }
tail -15 $O/persist_trace.txt
