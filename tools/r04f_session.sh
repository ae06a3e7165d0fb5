#!/usr/bin/env bash
# Round-4 PMC passes: one rank's share of the 8-GPU configs, the kord-10 mappm, the stepper
# (bound launches), then the bench's kernel trace + the headline's FETCH/WRITE passes.
set -uo pipefail
bash tools/pmc_all.sh r04f calib stepper_c96_r8 emulator_c384_r8 emulator_c384_f32_r8 predict_mappm_c384_r8 \
    predict_mappm_c384_bf16x6_r8 mappm_c384_k10 stepper_c96 || exit $?
