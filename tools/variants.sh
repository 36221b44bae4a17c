#!/bin/bash
# Builds A/B variants of libcrimp_hip.so into build/variants/<name>.so: tools/variants.sh "name:-DFLAG ..." ...
cd "$(dirname "$0")/../crimp_amd/csrc"
mkdir -p ../../build/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags -shared \
      -o ../../build/variants/$name.so crimp_hip.hip &
done
wait
ls -la ../../build/variants/
