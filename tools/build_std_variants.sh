# Timing variants of the standardisation (compile-time knobs of csrc/stats.hip): each links the in-tree objects
# of the other sources with a stats.o built with -D flags into variants/libgbm_<name>.so (GBM_LIBGBM=...).
# Run after __graft_entry__.build().
set -e
cd "$(dirname "$0")/.."
B=genomicbreedingmodels.jl_amd/csrc/build
mkdir -p variants
OBJS="$B/grm.hip.o $B/grm_exact.hip.o $B/chol.hip.o $B/chol_flow.hip.o $B/effects.hip.o $B/gibbs.hip.o $B/capi.cpp.o $B/session.cpp.o $B/knobs.cpp.o $B/hostpack.cpp.o"
build() {  # name flags...
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c genomicbreedingmodels.jl_amd/csrc/stats.hip -o variants/stats_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS variants/stats_$name.o -lrccl -lrocprofiler-sdk-roctx -o variants/libgbm_std_$name.so
}
build plain -DGBM_STD_NT=0 &
build ntld -DGBM_STD_NT=2 &
build ntst -DGBM_STD_NT=3 &
wait
