set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_bench.hip -o /tmp/mfma_bench > gpurun_out/mfma_build.log 2>&1 || { echo build failed; cat gpurun_out/mfma_build.log; exit 3; }
timeout -k 10 300 /tmp/mfma_bench 4000 128 > gpurun_out/mfma_bench.jsonl 2>&1; rc=$?
cat gpurun_out/mfma_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 /tmp/mfma_bench 1000 64 >> gpurun_out/mfma_bench.jsonl 2>&1; rc=$?
tail -11 gpurun_out/mfma_bench.jsonl
exit $rc
