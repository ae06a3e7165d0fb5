// TEMPORARY: placeholder until coarsen.hip lands (same commit series).
#include "common.h"
extern "C" {
int fv3_regrid_coarsen(const float*, const float*, const float* const*, float* const*, int, float*, int, int, int, int, int, int, int, double, void*) { fv3::set_error("not yet"); return FV3_ERR_UNSUPPORTED; }
}
