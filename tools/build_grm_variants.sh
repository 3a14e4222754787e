# Timing variants of the GRM SYRK (compile-time knobs of csrc/grm.hip): each links the in-tree objects of the
# other sources with a grm.o built with -D flags into variants/libgbm_<name>.so (loaded with GBM_LIBGBM=...).
# Run after __graft_entry__.build(). Timing only: GBM_SYRK_TIMING_NOLOAD computes on stale LDS.
set -e
cd "$(dirname "$0")/.."
B=genomicbreedingmodels.jl_amd/csrc/build
mkdir -p variants
OBJS="$B/stats.hip.o $B/grm_exact.hip.o $B/chol.hip.o $B/chol_flow.hip.o $B/effects.hip.o $B/gibbs.hip.o $B/capi.cpp.o $B/session.cpp.o $B/knobs.cpp.o $B/hostpack.cpp.o"
build() {  # name flags...
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c genomicbreedingmodels.jl_amd/csrc/grm.hip -o variants/grm_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS variants/grm_$name.o -lrccl -lrocprofiler-sdk-roctx -o variants/libgbm_$name.so
}
build g_base &
build g_noload -DGBM_SYRK_TIMING_NOLOAD &
wait
