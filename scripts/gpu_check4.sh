set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spass_bench.hip -o /tmp/spass_bench > gpurun_out/spass_build.log 2>&1 || { echo tool build failed; exit 3; }
timeout -k 10 300 /tmp/spass_bench 4000 128 20 > gpurun_out/spass_bench.jsonl 2>&1; rc=$?
echo "spass_bench rc=$rc"; cat gpurun_out/spass_bench.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
exit 0
