#!/bin/bash
# the library with HZ_DIAG_STAMPS in the stationary engine's units -> huygens_amd/lib/diag/ (HZ_LIB_PATH)
cd "$(dirname "$0")/.." || exit 2
mkdir -p build/diag huygens_amd/lib/diag
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-pass-failed -munsafe-fp-atomics"
objs=""
for f in huygens_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  case $b in hz_fb_resp|hz_fb_state) /opt/rocm/bin/hipcc $F -DHZ_DIAG_STAMPS -c "$f" -o build/diag/$b.o || exit 1; objs="$objs build/diag/$b.o";;
  *) objs="$objs build/obj/$b.o";; esac
done
/opt/rocm/bin/hipcc $F -shared -o huygens_amd/lib/diag/libhuygens_hip.so $objs
