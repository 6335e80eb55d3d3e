#!/bin/bash
# Host-sanitized build of the C ABI's host code (capi.cpp, dit.cpp, vae_engine.cpp) + the validation driver,
# linked against the product kernels' objects (f-lite_amd/build/*.o, device code unchanged). CPU-only: the
# driver never touches a GPU. Output: tests/native/_build/capi_validation
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
CSRC="$ROOT/f-lite_amd/csrc"
OUT="$HERE/_build"
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fno-omit-frame-pointer -I$ROOT/include -I$CSRC"
python3 "$ROOT/f-lite_amd/build_native.py" >/dev/null   # the kernels' objects
objs=()
for f in capi.cpp dit.cpp vae_engine.cpp; do
  "$HIPCC" $FLAGS $SAN -c "$CSRC/$f" -o "$OUT/${f%.cpp}.asan.o"
  objs+=("$OUT/${f%.cpp}.asan.o")
done
"$HIPCC" $FLAGS $SAN -c "$HERE/capi_validation.cpp" -o "$OUT/capi_validation.o"
kern=()
for f in "$ROOT"/f-lite_amd/build/*.o; do
  case "$(basename "$f")" in capi.o|dit.o|vae_engine.o) ;; *) kern+=("$f") ;; esac
done
"$HIPCC" --offload-arch=gfx950 -fsanitize=address,undefined -o "$OUT/capi_validation" "$OUT/capi_validation.o" \
  "${objs[@]}" "${kern[@]}" -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$OUT/capi_validation"
