#!/bin/bash
# Builds an A/B variant of the C-ABI library with extra -D flags into
# tools/ablib/<name>/libugofec.so (gitignored; it travels to the GPU box) (select it with UGO_FEC_LIB=...).  Not product.
# usage: tools/build_variant.sh <name> -DMACRO=value ...
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$ROOT/tools/ablib/$name
mkdir -p "$out/host"
cd "$ROOT/ugo_amd/csrc"
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result $*"
for k in fec_kernels rx_kernels tx_kernels pkt_kernels; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $k.hip -o "$out/$k.o" &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c ugo_fec.cpp -o "$out/ugo_fec.o" &
for k in reedsolomon fec conn_abi; do /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c host/$k.cpp -o "$out/host/$k.o" & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libugofec.so" "$out"/*.o "$out"/host/*.o
echo "$out/libugofec.so"
