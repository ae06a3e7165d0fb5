#!/bin/bash
# Experiment build of csrc/dense_b3.hip only, linked with the cached objects of every other
# source: tools/build_b3_variant.sh <name> <extra hipcc flags...> -> tools/variants/lib<name>.so
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tools/variants
python3 -c "from fv3net_amd import build; build.build()" >/dev/null
OBJS=$(ls fv3net_amd/_lib/obj/*.o | grep -v '/dense_b3\.')
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -I include "$@" \
    -c fv3net_amd/csrc/dense_b3.hip -o tools/variants/$NAME.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/variants/lib$NAME.so $OBJS tools/variants/$NAME.o
rm -f tools/variants/$NAME.o
echo tools/variants/lib$NAME.so
