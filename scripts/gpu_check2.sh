set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/window_profile.py 1000 1 20 > gpurun_out/win_1000_1.jsonl 2>&1; rc=$?
echo "win1000 rc=$rc"; tail -2 gpurun_out/win_1000_1.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/window_profile.py 4000 1 20 > gpurun_out/win_4000_1.jsonl 2>&1; rc=$?
echo "win4000x1 rc=$rc"; tail -2 gpurun_out/win_4000_1.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python scripts/window_profile.py 4000 128 20 > gpurun_out/win_4000_128.jsonl 2>&1; rc=$?
echo "win4000x128 rc=$rc"; tail -3 gpurun_out/win_4000_128.jsonl
exit $rc
