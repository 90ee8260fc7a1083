# round-6 final measurement gate, in three calls (each under gpurun's 1200 s):
#   OUT=r6f1 PART=1 bash scripts/r6_final.sh   headline (+ rocprofv3), configs[1], SI fixture (+ rocprofv3)
#   OUT=r6f2 PART=2 bash scripts/r6_final.sh   shared-Z, Exact n=200 (+ rocprofv3), SI d=8 Exact (+ rocprofv3)
#   OUT=r6f2b PART=2b                           SI d=8 Exact (+ rocprofv3) (exact_prof's rocprofv3 segfaults at exit
#                                               after writing its stats: the gate reads that as a failure)
#   OUT=r6f3 PART=3 bash scripts/r6_final.sh   Exact n=1000 one instance (sampled CPU), Stiefel (+ rocprofv3), smoke,
#                                               the new tridiagonal-path tests
set -u
cd "$GRAFT_REPO_ROOT"
case "${PART:-1}" in
  1) STEPS="headline headline_prof" bash scripts/gate.sh && XB="--cpu-pool-budget 100" STEPS="cfg1 si si_prof" bash scripts/gate.sh ;;
  2) XB="--cpu-budget 30 --cpu-pool-budget 60" STEPS="shared" bash scripts/gate.sh && STEPS="exact exact_prof si_d8_exact si_d8_exact_prof" bash scripts/gate.sh ;;
  2b) STEPS="si_d8_exact si_d8_exact_prof" bash scripts/gate.sh ;;
  3) STEPS="exact1000 stiefel stiefel_prof smoke" bash scripts/gate.sh &&
     timeout -k 10 600 python -u -m pytest tests/test_gpu_trs.py -m gpu -v --timeout 500 --timeout-method thread \
       -k "tri_wave_solves_match_one_lane_solves or above_lds_size_matches_oracle or hard_case_above" \
       > gpurun_out/${OUT:-gate}/trs_tests.log 2>&1 && tail -1 gpurun_out/${OUT:-gate}/trs_tests.log ;;
esac
