# Round-2 gate g: the re-calibrated / new GPU tests, then the 2-rank same-device bench rehearsal.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_n4000.py tests/test_gpu_si.py tests/test_gpu_distributed.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|classified flips" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dim 1000 --batch 8 --steps 6 --warmup 1 --backend gloo --same-device --cpu-budget 0 > $O/bench_2rank_same_device.json 2> $O/bench_2rank.err; rc=$?
echo "2-rank rc=$rc"; head -c 300 $O/bench_2rank_same_device.json; echo
exit $rc
