#!/bin/bash
# Builds libkc_hip.so with extra device-compile flags into
# kmer-counter_amd/variants/<name>/ (tuning experiments; select with KC_LIB).
# Variants are experiment builds (-DKC_EXPERIMENTS): they honour the timing
# ablation variables (KC_F_SKIP, KC_P2_SKIP, KC_P5_SKIP, KC_SEG_SKIP,
# KC_SKM_MMIN) that the release library ignores.
# usage: tools/build_variant.sh <name> "<hipcc flags>"
set -e
R=/root/repo/kmer-counter_amd
[ -n "$NO_MAKE" ] || make -C $R -s ARCH=gfx950 >/dev/null
mkdir -p $R/variants/$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -Wno-unused-function \
  -DKC_EXPERIMENTS $2 -c $R/csrc/kc_kernels.hip -o $R/variants/$1/kc_kernels.o
g++ -O2 -std=c++17 -fPIC -I$R/../include -I$R/csrc -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -pthread \
  -DKC_EXPERIMENTS -c $R/csrc/kc_api.cpp -o $R/variants/$1/kc_api.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/variants/$1/libkc_hip.so $R/variants/$1/kc_kernels.o \
  $R/variants/$1/kc_api.o $R/build/kc_io.o $R/build/kc_stage.o -pthread
rm -f $R/variants/$1/kc_kernels.o $R/variants/$1/kc_api.o
echo built $R/variants/$1/libkc_hip.so
