set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_gpu_si.py -q -x -m gpu > gpurun_out/gpu_si.log 2>&1; rc=$?
echo "pytest si rc=$rc"; tail -40 gpurun_out/gpu_si.log
exit $rc
