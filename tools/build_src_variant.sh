#!/bin/bash
# Experiment build of ONE source, linked with the cached objects of every other source:
#   tools/build_src_variant.sh <source stem, e.g. mappm> <name> <extra hipcc flags...>
#   -> tools/variants/lib<name>.so (git-ignored), used via FV3NET_AMD_LIB=...
set -euo pipefail
cd "$(dirname "$0")/.."
SRC=$1; NAME=$2; shift 2
mkdir -p tools/variants
python3 -c "from fv3net_amd import build; build.build()" >/dev/null
OBJS=$(ls fv3net_amd/_lib/obj/*.o | grep -v "/$SRC\.")
EXT=hip; [ -f fv3net_amd/csrc/$SRC.hip ] || EXT=cpp
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -I include "$@" \
    -c fv3net_amd/csrc/$SRC.$EXT -o tools/variants/$NAME.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/variants/lib$NAME.so $OBJS tools/variants/$NAME.o
rm -f tools/variants/$NAME.o
echo tools/variants/lib$NAME.so
