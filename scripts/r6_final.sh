# round-6 final measurement gate, in three calls (each under gpurun's 1200 s):
#   OUT=r6f1 PART=1 bash scripts/r5_final.sh   headline (+ rocprofv3), configs[1], SI fixture (+ PMC, rocprofv3)
#   OUT=r6f2 PART=2 bash scripts/r5_final.sh   shared-Z, Exact n=200 (+ rocprofv3), SI d=8 Exact (+ rocprofv3)
#   OUT=r6f3 PART=3 bash scripts/r5_final.sh   Exact n=1000 one instance (sampled CPU), Stiefel (+ rocprofv3)
#   OUT=r6f4 PART=4 bash scripts/r5_final.sh   the Exact lines again with the eigensolver roofline + the d=8 k_si PMC
#   OUT=r6f5 PART=5 bash scripts/r5_final.sh   the SI fixture line again (+ PMC, rocprofv3)
set -u
cd "$GRAFT_REPO_ROOT"
case "${PART:-1}" in
  1) STEPS="headline headline_prof" bash scripts/gate.sh && XB="--cpu-pool-budget 100" STEPS="cfg1 si_pmc si si_prof" bash scripts/gate.sh ;;
  2) XB="--cpu-budget 30 --cpu-pool-budget 60" STEPS="shared" bash scripts/gate.sh && STEPS="exact exact_prof si_d8_exact si_d8_exact_prof" bash scripts/gate.sh ;;
  3) STEPS="exact1000 stiefel stiefel_prof" bash scripts/gate.sh ;;
  4) STEPS="exact exact_prof si_d8_pmc si_d8_exact si_d8_exact_prof" bash scripts/gate.sh ;;
  5) XB="--cpu-pool-budget 100" STEPS="si_pmc si si_prof" bash scripts/gate.sh ;;
esac
