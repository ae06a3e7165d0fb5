#!/bin/bash
# An experiment build of csrc/dense.hip only, linked with the product's cached objects:
#   tools/build_dense_variant.sh <name> <extra hipcc flags...>  -> tools/variants/lib<name>.so
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tools/variants/obj
OBJ=tools/variants/obj/dense_$NAME.o
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -I include "$@" \
    -c fv3net_amd/csrc/dense.hip -o $OBJ
OTHERS=$(ls fv3net_amd/_lib/obj/*.o | grep -v '/dense\.')
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC -shared --offload-arch=gfx950 -o tools/variants/lib$NAME.so $OBJ $OTHERS
echo tools/variants/lib$NAME.so
