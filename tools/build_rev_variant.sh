#!/bin/bash
# Experiment build: one source file as it was at a git revision (its headers too), linked
# with the current objects of every other source:
#   tools/build_rev_variant.sh <name> <rev> <csrc file> [headers...] -> tools/variants/lib<name>.so
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; REV=$2; SRC=$3; shift 3
T=$(mktemp -d)
mkdir -p $T/fv3net_amd/csrc tools/variants
ln -s "$PWD/include" $T/include
cp fv3net_amd/csrc/*.h $T/fv3net_amd/csrc/
for f in $SRC "$@"; do git show $REV:fv3net_amd/csrc/$f > $T/fv3net_amd/csrc/$f; done
python3 -c "from fv3net_amd import build; build.build()" >/dev/null
BASE=${SRC%.hip}
OBJS=$(ls fv3net_amd/_lib/obj/*.o | grep -v "/$BASE\.")
/opt/rocm/bin/hipcc -DFV3_EXPERIMENT_BUILD -O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -I include \
    -c $T/fv3net_amd/csrc/$SRC -o $T/v.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/variants/lib$NAME.so $OBJS $T/v.o
rm -rf $T
echo tools/variants/lib$NAME.so
