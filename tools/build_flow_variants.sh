# Timing variants of the dataflow Cholesky (compile-time knobs of csrc/chol_flow.hip): each links the
# in-tree objects of the other sources with a chol_flow.o built with -D flags into variants/libgbm_<name>.so
# (loaded with GBM_LIBGBM=...). Run after __graft_entry__.build().
set -e
cd "$(dirname "$0")/.."
B=genomicbreedingmodels.jl_amd/csrc/build
mkdir -p variants
OBJS="$B/stats.hip.o $B/grm.hip.o $B/grm_exact.hip.o $B/chol.hip.o $B/effects.hip.o $B/gibbs.hip.o $B/capi.cpp.o $B/session.cpp.o $B/knobs.cpp.o $B/hostpack.cpp.o"
build() {  # name flags...
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c genomicbreedingmodels.jl_amd/csrc/chol_flow.hip -o variants/chol_flow_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS variants/chol_flow_$name.o -lrccl -lrocprofiler-sdk-roctx -o variants/libgbm_$name.so
}
# the workers' k-loop without operand loads / without MFMAs (timing only: the factorisation is of the
# un-updated tiles)
build base &
build noload -DGBM_FLOW_TIMING_NOLOAD &
build nomfma -DGBM_FLOW_TIMING_NOMFMA &
build noy -DGBM_FLOW_TIMING_NOY &
wait
