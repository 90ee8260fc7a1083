set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dim 1000 --batch 8 --steps 6 --warmup 1 --backend gloo --same-device > gpurun_out/bench_ddp_rehearsal.json 2> gpurun_out/bench_ddp_rehearsal.err; rc=$?
echo "ddp rehearsal rc=$rc"; cat gpurun_out/bench_ddp_rehearsal.json; tail -5 gpurun_out/bench_ddp_rehearsal.err
exit $rc
