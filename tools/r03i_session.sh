#!/usr/bin/env bash
# Round-3 profile session: kernel trace of the bench + the headline's FETCH/WRITE passes,
# then the per-kernel PMC passes of the bf16x6 legs (with the calibration leg).
set -uo pipefail
bash tools/profile.sh r03i || exit $?
bash tools/pmc_all.sh r03i calib dense_c48_bf16x6 dense_c384_bf16x6 emulator_c384_bf16x6 predict_mappm_c384_bf16x6
