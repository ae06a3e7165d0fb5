#!/bin/bash
# Build an experiment variant of the library: tools/build_variant.sh <name> <extra hipcc flags...>
# -> tools/variants/lib<name>.so (git-ignored), used via FV3NET_AMD_LIB=...
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tools/variants
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC -shared --offload-arch=gfx950 -I include "$@" \
    -o tools/variants/lib$NAME.so fv3net_amd/csrc/*.hip fv3net_amd/csrc/*.cpp
echo tools/variants/lib$NAME.so
