#!/bin/bash
# A/B builds: tools/build_variant.sh NAME "-DFLAG ..." -> llmvox_amd/libllmvox_hip_NAME.so
# (load with LVX_LIB_PATH=llmvox_amd/libllmvox_hip_NAME.so; git-ignored, travels with gpurun)
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../llmvox_amd/csrc"
O=build/var_$NAME; mkdir -p $O
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function $FLAGS"
$CXX -c ar_kernels.hip -o $O/ar.o &
$CXX -c codec_kernels.hip -o $O/codec.o &
$CXX -c encoder_kernels.hip -o $O/enc.o &
$CXX -x hip -c lvx_api.cpp -o $O/api.o &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libllmvox_hip_$NAME.so $O/ar.o $O/codec.o $O/enc.o $O/api.o
echo built ../libllmvox_hip_$NAME.so
