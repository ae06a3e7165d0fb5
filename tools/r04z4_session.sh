#!/usr/bin/env bash
# Closing profile of the final kernels (after the prologue-barrier fix): the bench under
# rocprofv3 --kernel-trace --stats, then the FETCH_SIZE / WRITE_SIZE passes.
set -uo pipefail
bash tools/profile.sh r04z4 || exit $?
echo done
