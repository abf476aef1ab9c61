#!/bin/bash
# Build a diagnostic / A-B variant of libswrt.so with extra compile flags into
# build/var/<name>.so (git-ignored, but shipped to the GPU box by gpurun);
# select it at run time with SWRT_LIB_PATH=build/var/<name>.so.
#   tools/build_variant.sh phase -DSWRT_PHASE_TIMING
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall "$@" \
  -o "build/var/$name.so" swraytracing_amd/csrc/swrt_api.hip -x none build/obj/*.o  # host TUs (build() made them)
echo "built build/var/$name.so"
