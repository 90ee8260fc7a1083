# Round 3: fp64 MFMA tile sweep (tools/mfma_bench.hip: peak probes with 1-16 chains, the solver's
# tile family over wave grids / stages / K slices) at n = 4000, 128 right-hand sides.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3mmb}
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_bench.hip -o /tmp/mfma_bench > $O/build.log 2>&1 || { cat $O/build.log; exit 3; }
timeout -k 10 300 /tmp/mfma_bench 4000 128 > $O/mfma_bench.jsonl 2> $O/mfma_bench.err; rc=$?
cat $O/mfma_bench.jsonl
exit $rc
