# Timing variants of the marker-effects kernel (compile-time knobs of csrc/effects.hip: rows per wave of the
# byte and fp64 variants, unroll of the individuals loop): each links the in-tree objects of the other sources
# with an effects.o built with -D flags into variants/libgbm_<name>.so (load with GBM_LIBGBM=...).
# Run after __graft_entry__.build(); every variant sums each row in the same order (bit-identical B).
# Round 6 (C2, exact / fp64 effects stage, ms): R_I8 x R_F64 x unroll 4x2x1 0.261 / 0.366, 2x1x1 0.188 / 0.367,
# 4x2x2 0.309 / 0.367, 2x1x4 0.323 / 0.373, 8x4x1 0.434 / 0.364, 1x1x2 0.210 / 0.377 (profiles/r06_effects_variants.txt).
set -e
cd "$(dirname "$0")/.."
B=genomicbreedingmodels.jl_amd/csrc/build
mkdir -p variants
OBJS="$B/stats.hip.o $B/grm.hip.o $B/grm_exact.hip.o $B/chol.hip.o $B/chol_flow.hip.o $B/gibbs.hip.o $B/capi.cpp.o $B/session.cpp.o $B/knobs.cpp.o $B/hostpack.cpp.o"
build() {  # name flags...
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c genomicbreedingmodels.jl_amd/csrc/effects.hip -o variants/effects_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS variants/effects_$name.o -lrccl -lrocprofiler-sdk-roctx -o variants/libgbm_$name.so
}
for spec in ${VARIANTS:-"2 1 1" "2 1 2" "1 1 1" "3 1 1"}; do
  set -- $spec
  build e_r$1_r$2_u$3 -DGBM_EFF_R_I8=$1 -DGBM_EFF_R_F64=$2 -DGBM_EFF_UNROLL=$3 &
done
wait
