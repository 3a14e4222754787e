# Timing variants of the marker-effects kernel (compile-time knobs of csrc/effects.hip: rows per wave of the
# byte and fp64 variants, unroll of the individuals loop): each links the in-tree objects of the other sources
# with an effects.o built with -D flags into variants/libgbm_<name>.so (load with GBM_LIBGBM=...).
# Run after __graft_entry__.build(); every variant sums each row in the same order (bit-identical B).
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
build e_r4_r2_u1 -DGBM_EFF_R_I8=4 -DGBM_EFF_R_F64=2 -DGBM_EFF_UNROLL=1 &
build e_r2_r1_u1 -DGBM_EFF_R_I8=2 -DGBM_EFF_R_F64=1 -DGBM_EFF_UNROLL=1 &
build e_r4_r2_u2 -DGBM_EFF_R_I8=4 -DGBM_EFF_R_F64=2 -DGBM_EFF_UNROLL=2 &
build e_r2_r1_u4 -DGBM_EFF_R_I8=2 -DGBM_EFF_R_F64=1 -DGBM_EFF_UNROLL=4 &
build e_r8_r4_u1 -DGBM_EFF_R_I8=8 -DGBM_EFF_R_F64=4 -DGBM_EFF_UNROLL=1 &
build e_r1_r1_u2 -DGBM_EFF_R_I8=1 -DGBM_EFF_R_F64=1 -DGBM_EFF_UNROLL=2 &
wait
