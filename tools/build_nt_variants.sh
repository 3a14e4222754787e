# Plain-load builds of the streams that read with the nontemporal hint (GBM_STD_NT, GBM_GRM_RED_NT, GBM_XG_TP_NT):
# each links the in-tree objects of the other sources with one object rebuilt with the hint off, into
# variants/libgbm_<name>.so (GBM_LIBGBM=...). Run after __graft_entry__.build().
set -e
cd "$(dirname "$0")/.."
B=genomicbreedingmodels.jl_amd/csrc/build
ALL="stats.hip grm.hip grm_exact.hip chol.hip chol_flow.hip effects.hip gibbs.hip capi.cpp session.cpp knobs.cpp hostpack.cpp"
mkdir -p variants
build() {  # name source flags...
  name=$1; src=$2; shift 2
  objs=""
  for f in $ALL; do [ "$f" = "$src" ] || objs="$objs $B/$f.o"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c genomicbreedingmodels.jl_amd/csrc/$src -o variants/$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs variants/$name.o -lrccl -lrocprofiler-sdk-roctx -o variants/libgbm_$name.so
}
build red_plain grm.hip -DGBM_GRM_RED_NT=0 &
build xtp_plain grm_exact.hip -DGBM_XG_TP_NT=0 &
wait
