#!/usr/bin/env bash
# Round-4 PMC passes of the legs changed since r04f: kord-10 mappm, the stepper (full and
# one rank's share), coarsen, the split kernel (emulator, 2x256 C384), with the calibration.
set -uo pipefail
bash tools/pmc_all.sh r04y calib mappm_c384_k10 mappm_c384_k1 stepper_c96 stepper_c96_r8 coarsen_1f coarsen_4f \
    emulator_c384 dense_c384_bf16x3 emulator_c384_r8 || exit $?
echo done
