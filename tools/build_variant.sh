# Build a libgbm variant on the CPU host (cross-compiled for gfx950) into build/var/<name>/libgbm.so;
# the .so travels to the GPU box with the tree. Usage: tools/build_variant.sh NAME "-DX=1 -DY=2" [gibbs-source]
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2; GIBBS=${3:-}
C=genomicbreedingmodels.jl_amd/csrc; D=build/var/$NAME; mkdir -p $D
pids=()
for f in stats grm chol chol_flow effects gibbs; do
  src=$C/$f.hip
  if [ "$f" = gibbs ] && [ -n "$GIBBS" ]; then cp "$GIBBS" $C/_variant_gibbs.hip; src=$C/_variant_gibbs.hip; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $src -o $D/$f.o & pids+=($!)
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $C/capi.cpp -o $D/capi.o & pids+=($!)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -c $C/session.cpp -o $D/session.o & pids+=($!)
for pid in "${pids[@]}"; do wait $pid; done
rm -f $C/_variant_gibbs.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -lrocprofiler-sdk-roctx -o $D/libgbm.so
echo built $D/libgbm.so
