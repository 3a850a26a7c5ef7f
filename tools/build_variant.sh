#!/bin/bash
# dev: build libsanta_hip.so from a given santa_hip.hip (default: the working
# tree) into abl/<name>.so for A/B runs (tools/ab_libs.sh, SANTA_HIP_LIB).
#   tools/build_variant.sh NAME [SRC.hip] [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=${1:-mpi-hungarian-method_amd/csrc/santa_hip.hip}; shift || true
mkdir -p abl
D=mpi-hungarian-method_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Iinclude -I$D \
  -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -shared -o abl/$NAME.so "$SRC" $D/santa_host.cpp
echo abl/$NAME.so
