#!/bin/bash
# Build libriptrm_hip.so with riptrm_stiefel.hip compiled under extra flags, for same-box A/B through
# RIPTRM_LIB (riptrm_native.load).  Needs the other objects from __graft_entry__.build() in build/obj.
# usage: tools/build_stiefel_variant.sh NAME [hipcc flags...]  ->  tools/bin/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=riemannian-interior-point-trust-region-method_amd/csrc
mkdir -p tools/bin build/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" -c $C/riptrm_stiefel.hip -o build/obj/st_$name.o
objs=$(ls build/obj/*.hip.o | grep -v riptrm_stiefel)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/obj/st_$name.o -ldl -o tools/bin/lib_$name.so
