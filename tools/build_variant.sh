#!/bin/bash
# Builds libkc_hip.so with extra device-compile flags into
# kmer-counter_amd/variants/<name>/ (tuning experiments; select with KC_LIB).
# usage: tools/build_variant.sh <name> "<hipcc flags>"
set -e
R=/root/repo/kmer-counter_amd
make -C $R -s ARCH=gfx950 >/dev/null
mkdir -p $R/variants/$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -Wno-unused-function $2 \
  -c $R/csrc/kc_kernels.hip -o $R/variants/$1/kc_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/variants/$1/libkc_hip.so $R/variants/$1/kc_kernels.o \
  $R/build/kc_api.o $R/build/kc_io.o -pthread
rm -f $R/variants/$1/kc_kernels.o
echo built $R/variants/$1/libkc_hip.so
