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
D=${VARIANT_DIR:-$R/variants}/$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -Wno-unused-function \
  -DKC_EXPERIMENTS $2 -c $R/csrc/kc_kernels.hip -o $D/kc_kernels.o
g++ -O2 -std=c++17 -fPIC -I$R/../include -I$R/csrc -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -pthread \
  -DKC_EXPERIMENTS -c $R/csrc/kc_api.cpp -o $D/kc_api.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libkc_hip.so $D/kc_kernels.o \
  $D/kc_api.o $R/build/kc_io.o $R/build/kc_stage.o -pthread
rm -f $D/kc_kernels.o $D/kc_api.o
echo built $D/libkc_hip.so
