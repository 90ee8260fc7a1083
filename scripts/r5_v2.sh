# eigensolver: one launch (stamps) vs the split launches (timing), then the Exact tests and benches
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5v}
mkdir -p $O
export TMPDIR=/tmp
for m in 100 199; do
  RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
  timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/split.txt 2>&1 || { tail $O/split.txt; exit 1; }
done
echo "one launch:"; grep "compact:\|values:" $O/stamps.txt | awk 'NR%3==0'
echo "split:"; grep "compact:\|values:" $O/split.txt | awk 'NR%3==0'
OUT=${OUT:-r5v} bash scripts/r5_p4.sh
