# AddressSanitizer + UndefinedBehaviorSanitizer build of libgbm's HOST code (the C-ABI shim
# capi.cpp / session.cpp and the host launchers in the .hip files; device code is built as usual:
# GPU sanitizers are not used on this pool) linked into tests/native/asan_driver.cpp, then run.
# CPU only: the driver exercises argument validation, the no-device paths and thread-local errors.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CSRC="$ROOT/genomicbreedingmodels.jl_amd/csrc"
OUT="${ASAN_OUT:-$ROOT/genomicbreedingmodels.jl_amd/csrc/build/asan}"
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
objs=()
pids=()
for f in stats.hip grm.hip grm_exact.hip chol.hip chol_flow.hip effects.hip gibbs.hip capi.cpp session.cpp knobs.cpp hostpack.cpp; do
  o="$OUT/$f.o"
  objs+=("$o")
  HO=""
  [ "$f" = hostpack.cpp ] && HO="--offload-host-only"
  $HIPCC --offload-arch=gfx950 $HO -O1 -g -fno-omit-frame-pointer -fPIC -std=c++17 $SAN -c "$CSRC/$f" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC -O1 -g -std=c++17 $SAN -c "$ROOT/tests/native/asan_driver.cpp" -o "$OUT/asan_driver.o"
$HIPCC --offload-arch=gfx950 -fno-gpu-sanitize -fsanitize=address,undefined "$OUT/asan_driver.o" "${objs[@]}" -lrccl \
  -lrocprofiler-sdk-roctx -o "$OUT/asan_driver"
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 "$OUT/asan_driver"
