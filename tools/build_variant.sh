# Build a libgbm variant on the CPU host (cross-compiled for gfx950) into build/var/<name>/libgbm.so;
# the .so travels to the GPU box with the tree. Usage: tools/build_variant.sh NAME "-DX=1 -DY=2"
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2
C=genomicbreedingmodels.jl_amd/csrc; D=build/var/$NAME; mkdir -p $D
for f in stats grm chol chol_flow effects gibbs; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $C/$f.hip -o $D/$f.o &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $C/capi.cpp -o $D/capi.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $C/session.cpp -o $D/session.o &
wait; for o in $D/*.o; do :; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -lrocprofiler-sdk-roctx -o $D/libgbm.so
echo built $D/libgbm.so
