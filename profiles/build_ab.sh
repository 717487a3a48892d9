#!/bin/bash
# A/B builds of libcvd.so: cvd_kernels.hip compiled with extra -D flags, linked with the
# in-tree objects of the other sources, into lib/libcvd_<name>.so
#   bash profiles/build_ab.sh <name> -DFLAG=V ...
set -euo pipefail
name=$1; shift
C=$(cd "$(dirname "$0")/../detecting-convolutional-codes-via-markovian-statistics_amd/csrc" && pwd)
make -s -C "$C" >/dev/null
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -ffp-contract=off \
  -munsafe-fp-atomics "$@" -c "$C/cvd_kernels.hip" -o "$T/cvd_kernels.o"
objs=""
for o in cvd_host cvd_parity cvd_exponent cvd_rtc cvd_comm cvd_learn cvd_bfs; do objs="$objs $C/$o.o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$C/../lib/libcvd_$name.so" "$T/cvd_kernels.o" $objs -lhiprtc -ldl
rm -rf "$T"
echo "$C/../lib/libcvd_$name.so"
