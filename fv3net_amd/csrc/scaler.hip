// fv3net_amd — fv3fit StandardScaler on device (external/fv3fit/fv3fit/_shared/scaler.py:
// 36-100), as the PytorchPredictor uses it around its model
// (external/fv3fit/fv3fit/pytorch/predict.py:299-387):
//
//   pack      normalized = (x - mean) / std      float64 numpy arithmetic (x float32 or
//             -> torch.as_tensor(...).float()   float64, mean/std float64), rounded to
//                                                float32 once (_pack_to_tensor :371-375)
//   unpack    out = y * std + mean               y the model's float32 output, promoted
//                                                to float64 (_unpack_tensor :378-399)
//
// Bit-identical to numpy: the same IEEE double operations in the same order (the library
// is built with -ffp-contract=off, so y * std + mean stays two roundings as in numpy).
// mean/std hold one value per level, or a single value for a 2-D variable.
//
// Mapping: one thread per (column, level) element; blockIdx.y is the level, so each
// wave reads one level of 64 consecutive columns (coalesced on the [level][column] layout
// of the state; a [column][level] array still works, with strided reads).  HBM-bound:
// (4 or 8) + 4 bytes per element.
#include "common.h"

namespace fv3 {
namespace {

constexpr int kScaleBlock = 256;

template <typename T, typename TO>
__global__ __launch_bounds__(kScaleBlock) void standard_normalize_kernel(const T* __restrict__ x, fv3_layout xl,
                                                                         const double* __restrict__ mean,
                                                                         const double* __restrict__ std_,
                                                                         int per_level, TO* __restrict__ out,
                                                                         fv3_layout ol, int64_t ncol)
{
    const int64_t c = (int64_t)blockIdx.x * kScaleBlock + threadIdx.x;
    const int k = blockIdx.y;
    if (c >= ncol) return;
    const int p = per_level ? k : 0;
    const double v = (double)x[col_offset(xl, c) + (int64_t)k * xl.ld];
    const double n = (v - mean[p]) / std_[p];
    out[col_offset(ol, c) + (int64_t)k * ol.ld] = (TO)n;
}

template <typename T>
__global__ __launch_bounds__(kScaleBlock) void standard_denormalize_kernel(const T* __restrict__ y,
                                                                           fv3_layout yl,
                                                                           const double* __restrict__ mean,
                                                                           const double* __restrict__ std_,
                                                                           int per_level, double* __restrict__ out,
                                                                           fv3_layout ol, int64_t ncol)
{
    const int64_t c = (int64_t)blockIdx.x * kScaleBlock + threadIdx.x;
    const int k = blockIdx.y;
    if (c >= ncol) return;
    const int p = per_level ? k : 0;
    const double v = (double)y[col_offset(yl, c) + (int64_t)k * yl.ld];
    const double s = v * std_[p];
    out[col_offset(ol, c) + (int64_t)k * ol.ld] = s + mean[p];
}

int check_scale_args(const void* x, fv3_layout xl, const double* mean, const double* std_, int n_params,
                     const void* out, fv3_layout ol, int64_t ncol, int nz, const char* what)
{
    FV3_REQUIRE(ncol >= 0 && nz >= 1 && nz <= 65535, "%s: bad sizes ncol=%lld nz=%d", what, (long long)ncol, nz);
    FV3_REQUIRE(n_params == nz || n_params == 1, "%s: %d scaler values for %d levels", what, n_params, nz);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(x && mean && std_ && out, "%s: NULL array", what);
    FV3_REQUIRE(layout_ok(xl, ncol) && layout_ok(ol, ncol), "%s: bad layout", what);
    return FV3_OK;
}

template <typename TO>
int normalize_impl(const void* x, int x_f64, fv3_layout x_l, const double* mean, const double* std_, int n_params,
                   TO* out, fv3_layout out_l, int64_t ncol, int nz, void* stream)
{
    clear_error();
    if (int st = check_scale_args(x, x_l, mean, std_, n_params, out, out_l, ncol, nz, "standard_normalize")) return st;
    if (ncol == 0) return FV3_OK;
    const dim3 grid((unsigned)((ncol + kScaleBlock - 1) / kScaleBlock), (unsigned)nz);
    if (x_f64)
        hipLaunchKernelGGL((standard_normalize_kernel<double, TO>), grid, dim3(kScaleBlock), 0, (hipStream_t)stream,
                           (const double*)x, x_l, mean, std_, n_params == nz ? 1 : 0, out, out_l, ncol);
    else
        hipLaunchKernelGGL((standard_normalize_kernel<float, TO>), grid, dim3(kScaleBlock), 0, (hipStream_t)stream,
                           (const float*)x, x_l, mean, std_, n_params == nz ? 1 : 0, out, out_l, ncol);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

template <typename T>
int denormalize_impl(const T* y, fv3_layout y_l, const double* mean, const double* std_, int n_params, double* out,
                     fv3_layout out_l, int64_t ncol, int nz, void* stream)
{
    clear_error();
    if (int st = check_scale_args(y, y_l, mean, std_, n_params, out, out_l, ncol, nz, "standard_denormalize"))
        return st;
    if (ncol == 0) return FV3_OK;
    const dim3 grid((unsigned)((ncol + kScaleBlock - 1) / kScaleBlock), (unsigned)nz);
    hipLaunchKernelGGL(standard_denormalize_kernel<T>, grid, dim3(kScaleBlock), 0, (hipStream_t)stream, y, y_l, mean,
                       std_, n_params == nz ? 1 : 0, out, out_l, ncol);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_standard_normalize(const void* x, int x_f64, fv3_layout x_l, const double* mean,
                                      const double* std_, int n_params, float* out, fv3_layout out_l, int64_t ncol,
                                      int nz, void* stream)
{
    return fv3::normalize_impl<float>(x, x_f64, x_l, mean, std_, n_params, out, out_l, ncol, nz, stream);
}

extern "C" int fv3_standard_normalize_f64(const void* x, int x_f64, fv3_layout x_l, const double* mean,
                                          const double* std_, int n_params, double* out, fv3_layout out_l,
                                          int64_t ncol, int nz, void* stream)
{
    return fv3::normalize_impl<double>(x, x_f64, x_l, mean, std_, n_params, out, out_l, ncol, nz, stream);
}

extern "C" int fv3_standard_denormalize(const float* y, fv3_layout y_l, const double* mean, const double* std_,
                                        int n_params, double* out, fv3_layout out_l, int64_t ncol, int nz,
                                        void* stream)
{
    return fv3::denormalize_impl<float>(y, y_l, mean, std_, n_params, out, out_l, ncol, nz, stream);
}

extern "C" int fv3_standard_denormalize_f64(const double* y, fv3_layout y_l, const double* mean, const double* std_,
                                            int n_params, double* out, fv3_layout out_l, int64_t ncol, int nz,
                                            void* stream)
{
    return fv3::denormalize_impl<double>(y, y_l, mean, std_, n_params, out, out_l, ncol, nz, stream);
}
