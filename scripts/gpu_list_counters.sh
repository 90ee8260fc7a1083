# List the PMC counters rocprofv3 offers on this box (for choosing a pass).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; rc=$?
grep -oE "\b(SQC?_[A-Z0-9_]+|TA_[A-Z0-9_]+|TCP_[A-Z0-9_]+)" gpurun_out/counters.txt | sort -u | tr '\n' ' ' | head -c 6000
exit $rc
