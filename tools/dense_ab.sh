#!/bin/bash
# A/B of runtime knobs for the dense kernel: mean launch time at C48 and C384
set -o pipefail
run() { env "$@" timeout -k 10 120 python tools/dense_time.py 2>&1 | grep -v amdgpu.ids; }
run X=1 && run FV3_DENSE_NC=1 && run FV3_DENSE_NC=1 FV3_DENSE_CFG=4,2 && run FV3_DENSE_NC=1 FV3_DENSE_CFG=2,3 && run FV3_DENSE_NC=1 FV3_DENSE_GRID=100000000
