# Stiefel kernel phase stamps (diagnostic build of csrc/riptrm_stiefel.hip, tools/stiefel_stamps.hip).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-stst}
mkdir -p $O
C=riemannian-interior-point-trust-region-method_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I$C -Iinclude tools/stiefel_stamps.hip -o /tmp/stamps > $O/build.log 2>&1 || { cat $O/build.log; exit 3; }
timeout -k 10 120 /tmp/stamps 200 50 256 > $O/stamps.jsonl 2>&1; rc=$?
cat $O/stamps.jsonl
exit $rc
