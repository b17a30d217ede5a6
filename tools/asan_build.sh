#!/bin/bash
# Builds tools/asan_driver: every library source plus tools/asan_driver.cpp in
# one executable, HOST code instrumented with AddressSanitizer and UBSan
# (device code is not: -Xarch_host puts each -fsanitize= on the host side
# only).  Run it on the GPU box as
#   ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 ./tools/asan_driver
set -eu
cd "$(dirname "$0")/.."
OUT=build/asan
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950"
objs=()
for f in ugo_amd/csrc/fec_kernels.hip ugo_amd/csrc/rx_kernels.hip ugo_amd/csrc/tx_kernels.hip \
         ugo_amd/csrc/pkt_kernels.hip; do
  o=$OUT/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc $FLAGS $SAN -c "$f" -o "$o" &
  objs+=("$o")
done
for f in ugo_amd/csrc/ugo_fec.cpp ugo_amd/csrc/host/reedsolomon.cpp ugo_amd/csrc/host/fec.cpp \
         ugo_amd/csrc/host/conn_abi.cpp tools/asan_driver.cpp; do
  o=$OUT/$(basename "$f" .cpp).o
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC $SAN -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN -o tools/asan_driver "${objs[@]}"
echo "built tools/asan_driver"
