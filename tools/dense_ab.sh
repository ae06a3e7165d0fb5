#!/bin/bash
# A/B of runtime knobs for the dense kernel: mean launch time at C48 and C384
# (each line: the env it ran under, then dense_time.py's figures)
set -o pipefail
export FV3_VARIANTS=1  # A/B tool: the library reads kernel-variant selectors only with this set
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/dense_time.py 2>&1 | grep -v amdgpu.ids; }
if [ $# -gt 0 ]; then
    for cfg in "$@"; do run $cfg || exit $?; done
else
    run X=1 && run FV3_DENSE_NC=1 && run FV3_DENSE_NC=1 FV3_DENSE_CFG=4,2 && run FV3_DENSE_NC=1 FV3_DENSE_CFG=2,3
fi
