# eigensolver phase clocks (one launch, RIPTRM_EIG_STAMPS=1) at m = 100 and 199
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-eigclk}
mkdir -p $O
for m in 100 199; do
  RIPTRM_EIG_STAMPS=1 timeout -k 10 120 python scripts/eig_stamps.py $m 64 >> $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
done
grep "eig stamps" $O/stamps.txt | awk 'NR==4 || NR==13'
