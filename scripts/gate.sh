# GPU gate on the prebuilt tree (run through gpurun; builds nothing but the tools/ probes).
#
#   OUT=r4a STEPS="smoke tests headline" bash scripts/gate.sh [pytest selectors for 'tests'...]
#
# Every step has its own time limit, the steps are chained fail-fast, and everything lands in
# gpurun_out/$OUT.  Steps:
#   smoke            __graft_entry__.smoke()
#   tests            pytest -m gpu (selectors from the command line, default tests/)
#   headline         bench.py defaults (BASELINE configs[2])            -> bench_headline.json
#   headline_prof    rocprofv3 --kernel-trace --stats of the same        -> head/ (stats csv)
#   pmc_spass        FETCH_SIZE / WRITE_SIZE passes of k_spass_sup (separate rocprofv3 --pmc runs)
#                    -> r4_pmc_spass_sup.json + the traffic json bench.py reads
#   cfg1             bench.py --dim 1000 --batch 1 (configs[1])          -> bench_cfg1.json
#   cfg1_trace       scripts/persist_trace.py (k_persist phase stamps at configs[1])
#   shared           bench.py --layout shared (multi-start, MFMA S-pass), 128 and 256 starts -> bench_shared*.json
#   shared_prof      rocprofv3 stats of the shared bench (256 starts)
#   si               bench.py --problem si --batch 256                   -> bench_si_b256.json
#   stiefel          bench.py --problem stiefel at (200,50) x 256 and x 2048
#   stiefel_prof     rocprofv3 stats of the 256 and 2048 Stiefel benches
#   stiefel_pmc      FETCH_SIZE / WRITE_SIZE of the Stiefel kernels (tools/stiefel_stamps)
#   stiefel_stamps   in-kernel phase stamps of the Stiefel kernels (tools/stiefel_stamps)
#   exact            bench.py --trs Exact_RepMat --dim 200 --batch 64    -> bench_exact_200.json
#   exact_prof       rocprofv3 stats of the same
#   exact1000        bench.py --trs Exact_RepMat --dim 1000 --batch 1 with its (sampled) CPU baseline
#   si_pmc           issue-rate PMC pass of k_si (SQ_*) -> profiles/r5_si_pmc.json, read by the si step
#   si_prof          rocprofv3 stats of the SI bench
#   si_d8_pmc        issue-rate PMC pass of k_si at d = 8 (Exact) -> profiles/r5_si_pmc_d8.json, read by si_d8_exact
#   si_d8_exact      bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 with its CPU baseline
#   si_d8_exact_prof rocprofv3 stats of the same
#   (XB: extra bench.py arguments for the cfg1, shared and si steps, e.g. smaller CPU budgets)
#   dist2            bench.py --gpus 2 --same-device --backend gloo at the configs[3] per-rank shape
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-gate}
mkdir -p $O
export TMPDIR=/tmp
C=riemannian-interior-point-trust-region-method_amd/csrc
STEPS=${STEPS:-"smoke tests headline"}

note() { echo "[gate $(date +%H:%M:%S)] $*"; }
val() { python -c "import json,sys; d=json.load(open('$1')); print(sys.argv[1], d['value'], (d.get('roofline') or {}).get('frac'), ((d.get('cpu_baseline') or {}).get('value')))" "$2"; }

stamps_tool() {
  [ -x /tmp/stamps ] && return 0
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps \
    > $O/stamps_build.log 2>&1 || { cat $O/stamps_build.log; return 3; }
}

step() {
  case "$1" in
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; return 1; }
    tail -1 $O/smoke.log ;;
  tests)
    timeout -k 10 1050 python -u -m pytest ${SEL:-tests} -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1 \
      || { tail -40 $O/gpu_tests.log; return 1; }
    tail -1 $O/gpu_tests.log ;;
  headline)
    timeout -k 10 420 python bench.py ${BENCH_ARGS:-} > $O/bench_headline.json 2> $O/bench_headline.err || { tail $O/bench_headline.err; return 1; }
    val $O/bench_headline.json headline ;;
  headline_prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o head -- python bench.py --cpu-budget 0 \
      > $O/bench_headline_rocprof.json 2> $O/head_rocprof.log || return 1
    note "headline rocprof ok" ;;
  pmc_spass)
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/spmc_$c -o p -- python bench.py --cpu-budget 0 --warmup 1 --steps 2 \
        > $O/spmc_$c.log 2>&1 || { tail $O/spmc_$c.log; return 1; }
      note "spass pmc $c ok"
    done
    python scripts/pmc_summarize.py $(find $O/spmc_FETCH_SIZE -name "*counter_collection.csv" | head -1) \
      $(find $O/spmc_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/r4_pmc_spass_sup.json $O/r4_traffic_spass_sup.json \
      --n 4000 --batch 128 --instances 64 \
      --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, of python bench.py --cpu-budget 0 --warmup 1 --steps 2 ($O)" \
      && cp $O/r4_traffic_spass_sup.json profiles/ ;;   # the later headline step in this call reads it (bench.py --traffic-json)
  cfg1)
    timeout -k 10 400 python bench.py --dim 1000 --batch 1 ${XB:-} > $O/bench_cfg1.json 2> $O/bench_cfg1.err || { tail $O/bench_cfg1.err; return 1; }
    val $O/bench_cfg1.json cfg1 ;;
  cfg1_trace)
    timeout -k 10 120 python scripts/persist_trace.py 1000 > $O/cfg1_trace.txt 2>&1 || { tail $O/cfg1_trace.txt; return 1; }
    tail -5 $O/cfg1_trace.txt ;;
  shared)
    timeout -k 10 300 python bench.py --layout shared ${XB:-} > $O/bench_shared.json 2> $O/bench_shared.err || { tail $O/bench_shared.err; return 1; }
    val $O/bench_shared.json shared
    timeout -k 10 300 python bench.py --layout shared --batch 256 ${XB:-} > $O/bench_shared_b256.json 2> $O/bench_shared_b256.err \
      || { tail $O/bench_shared_b256.err; return 1; }
    val $O/bench_shared_b256.json shared256 ;;
  shared_prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shared -o shared -- python bench.py --layout shared \
      --batch 256 --cpu-budget 0 > $O/bench_shared_rocprof.json 2> $O/shared_rocprof.log || return 1
    note "shared rocprof ok" ;;
  si)
    timeout -k 10 400 python bench.py --problem si --batch 256 ${XB:-} > $O/bench_si_b256.json 2> $O/bench_si.err || { tail $O/bench_si.err; return 1; }
    val $O/bench_si_b256.json si ;;
  stiefel)
    timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 256 > $O/bench_stiefel_b256.json 2> $O/st256.err || return 1
    timeout -k 10 180 python bench.py --problem stiefel --dim 200 --batch 2048 > $O/bench_stiefel_b2048.json 2> $O/st2048.err || return 1
    python -c "
import json
for b in (256, 2048):
    d = json.load(open('$O/bench_stiefel_b%d.json' % b))
    print('stiefel', b, 'proj us', d['ms_per_step'] * 1e3, 'frac', d['roofline']['frac'], 'retr us', d['detail']['retraction_ms'] * 1e3,
          'frac', d['detail']['retraction_roofline']['frac'])" ;;
  stiefel_prof)
    for b in 256 2048; do
      timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st$b -o st -- python bench.py --problem stiefel \
        --dim 200 --batch $b --cpu-budget 0 > $O/bench_stiefel_rocprof_b$b.json 2> $O/st_rocprof_b$b.log || return 1
    done
    note "stiefel rocprof ok" ;;
  stiefel_pmc)
    stamps_tool || return 3
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/stpmc_$c -o p -- /tmp/stamps 200 50 ${ST_B:-2048} \
        > $O/stpmc_$c.log 2>&1 || return 1
      note "stiefel pmc $c ok"
    done
    python scripts/stiefel_pmc_summary.py $(find $O/stpmc_FETCH_SIZE -name "*counter_collection.csv" | head -1) \
      $(find $O/stpmc_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/stiefel_pmc.json --batch ${ST_B:-2048} ;;
  stiefel_stamps)
    stamps_tool || return 3
    timeout -k 10 60 /tmp/stamps 200 50 ${ST_B:-256} > $O/stiefel_stamps.txt 2>&1 || return 1
    tail -20 $O/stiefel_stamps.txt ;;
  exact)
    timeout -k 10 420 python bench.py --trs Exact_RepMat --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 60 \
      > $O/bench_exact_200.json 2> $O/bench_exact.err || { tail $O/bench_exact.err; return 1; }
    val $O/bench_exact_200.json exact200 ;;
  exact1000)
    timeout -k 10 900 python bench.py --trs Exact_RepMat --dim 1000 --batch ${EX_B:-1} --steps 3 --warmup 1 --cpu-budget 120 \
      --cpu-pool-budget 150 > $O/bench_exact_1000.json 2> $O/bench_exact1000.err || { tail $O/bench_exact1000.err; return 1; }
    val $O/bench_exact_1000.json exact1000 ;;
  si_pmc)
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
      --output-format csv -d $O/sipmc -o p -- python bench.py --problem si --batch 256 --cpu-budget 0 > $O/sipmc.log 2>&1 \
      || { tail $O/sipmc.log; return 1; }
    python scripts/si_pmc_summary.py $(find $O/sipmc -name "*counter_collection.csv" | head -1) $O/r5_si_pmc.json --d 5 \
      --source "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -- python bench.py --problem si --batch 256 --cpu-budget 0 ($O)" \
      && cp $O/r5_si_pmc.json profiles/ ;;   # the later si step in this call reads it (bench.py --si-pmc-json)
  si_prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/si -o si -- python bench.py --problem si \
      --batch 256 --cpu-budget 0 > $O/bench_si_rocprof.json 2> $O/si_rocprof.log || return 1
    note "si rocprof ok" ;;
  si_d8_pmc)
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
      --output-format csv -d $O/sid8pmc -o p -- python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 \
      --cpu-budget 0 --steps 4 > $O/sid8pmc.log 2>&1 || { tail $O/sid8pmc.log; return 1; }
    python scripts/si_pmc_summary.py $(find $O/sid8pmc -name "*counter_collection.csv" | head -1) $O/r5_si_pmc_d8.json --d 8 \
      --source "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -- python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 --steps 4 ($O)" \
      && cp $O/r5_si_pmc_d8.json profiles/ ;;
  si_d8_exact)
    timeout -k 10 900 python bench.py --problem si --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 100 --cpu-pool-budget 150 \
      --si-pmc-json profiles/r5_si_pmc_d8.json \
      > $O/bench_si_d8_exact.json 2> $O/bench_si_d8_exact.err || { tail $O/bench_si_d8_exact.err; return 1; }
    val $O/bench_si_d8_exact.json si_d8_exact ;;
  si_d8_exact_prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sid8 -o sid8 -- python bench.py --problem si \
      --si-dim 8 --trs Exact_RepMat --batch 64 --cpu-budget 0 > $O/bench_si_d8_rocprof.json 2> $O/sid8_rocprof.log || return 1
    note "si d8 exact rocprof ok" ;;
  exact_prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact -o exact -- python bench.py --trs Exact_RepMat \
      --dim 200 --batch 64 --steps 4 --warmup 1 --cpu-budget 0 > $O/bench_exact_rocprof.json 2> $O/exact_rocprof.log || return 1
    note "exact rocprof ok" ;;
  dist2)
    timeout -k 10 500 python bench.py --gpus 2 --same-device --backend gloo --batch 128 --warmup 1 --steps 2 --cpu-budget 0 \
      > $O/bench_dist2.json 2> $O/bench_dist2.err || { tail $O/bench_dist2.err; return 1; }
    val $O/bench_dist2.json dist2 ;;
  *)
    echo "unknown step $1"; return 2 ;;
  esac
}

# gpurun copies gpurun_out/ back only under 64 MiB: keep the rocprofv3 summaries (stats, PMC
# summaries), drop the per-dispatch traces and raw counter rows once the steps have read them
prune() {
  find $O \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*memory_copy_trace.csv" \
    -o -name "*.db" \) -delete 2>/dev/null
  du -sh $O 2>/dev/null | tail -1
}
trap prune EXIT

SEL="$*"
for s in $STEPS; do
  note "step $s"
  step "$s" || { note "step $s FAILED"; exit 1; }
done
note "all steps ok"
exit 0
