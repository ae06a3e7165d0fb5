// fv3net_amd — a launch plan: a fixed sequence of this library's launches over fixed
// device buffers, recorded once and issued by one C-ABI call per timestep.
//
// The prognostic run applies the same state buffers every step
// (workflows/prognostic_c48_run/runtime/loop.py:604-628 around
// runtime/steppers/machine_learning.py:239-309), and one rank's step at C96 over 8 GPUs
// (6,912 columns) is five short kernels (~50 us together).  Issued one by one from
// Python, the per-call host work (argument conversion, stream lookup, one foreign call
// each) took longer than the kernels; a HIP graph of the same step was slower still on
// the full grid.  A plan holds each launch's arguments in C++ and
// replays them on the caller's stream: the host cost of a step is one foreign call plus
// the launches themselves.
//
// Buffers named when an op is added must stay allocated while the plan is used, and the
// dense model (fv3_plan_add_dense_forward) must outlive the plan.
#include <functional>
#include <new>
#include <vector>

#include "common.h"
#include "dense_model.h"

struct fv3_plan {
    std::vector<std::function<int(void*)>> ops;
};

namespace {
// dst[t][i] = src[i], t < times, over 4-byte words (one launch for every copy)
__global__ __launch_bounds__(256) void repeat_words_kernel(const unsigned* __restrict__ src, int64_t n, int times,
                                                           unsigned* __restrict__ dst)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned v = src[i];
    for (int t = 0; t < times; ++t) dst[(int64_t)t * n + i] = v;
}
}  // namespace

extern "C" int fv3_plan_create(fv3_plan** out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(out, "plan_create: NULL output");
    *out = new (std::nothrow) fv3_plan();
    FV3_REQUIRE(*out, "plan_create: out of host memory");
    return FV3_OK;
}

extern "C" int fv3_plan_destroy(fv3_plan* plan)
{
    delete plan;
    return FV3_OK;
}

extern "C" int fv3_plan_size(const fv3_plan* plan) { return plan ? (int)plan->ops.size() : 0; }

// every op in order on `stream`; the first failing op's status (and its error text)
extern "C" int fv3_plan_run(const fv3_plan* plan, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan, "plan_run: NULL plan");
    for (const auto& op : plan->ops) {
        const int st = op(stream);
        if (st != FV3_OK) return st;
    }
    return FV3_OK;
}

// fv3_dense_forward_f64in (inputs_f64) or fv3_dense_forward_ex (float32 inputs at
// `precision`); the pointer and layout arrays are copied
extern "C" int fv3_plan_add_dense_forward(fv3_plan* plan, const fv3_dense_model* m, const void* const* inputs,
                                          const fv3_layout* in_l, float* const* outputs, const fv3_layout* out_l,
                                          int64_t ncol, int precision, int inputs_f64)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && m && inputs && in_l && outputs && out_l, "plan_add_dense_forward: NULL argument");
    std::vector<const void*> in(inputs, inputs + m->n_in);
    std::vector<fv3_layout> inl(in_l, in_l + m->n_in);
    std::vector<float*> out(outputs, outputs + m->n_out);
    std::vector<fv3_layout> outl(out_l, out_l + m->n_out);
    if (inputs_f64) {
        plan->ops.push_back([=](void* s) {
            return fv3_dense_forward_f64in(m, reinterpret_cast<const double* const*>(in.data()), inl.data(),
                                           out.data(), outl.data(), ncol, s);
        });
    } else {
        plan->ops.push_back([=](void* s) {
            return fv3_dense_forward_ex(m, reinterpret_cast<const float* const*>(in.data()), inl.data(), out.data(),
                                        outl.data(), ncol, precision, s);
        });
    }
    return FV3_OK;
}

extern "C" int fv3_plan_add_ml_epilogue(fv3_plan* plan, const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol,
                                        int nz, int state_f64, double dt, int mse_conserving, int hydrostatic,
                                        int flags)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && io, "plan_add_ml_epilogue: NULL argument");
    const fv3_epilogue_io cp = *io;
    plan->ops.push_back([=](void* s) {
        return fv3_ml_epilogue_ex(&cp, lay, ncol, nz, state_f64, dt, mse_conserving, hydrostatic, flags, s);
    });
    return FV3_OK;
}

extern "C" int fv3_plan_add_area_weighted_sums_f64(fv3_plan* plan, const double* const* diags, int n_diag,
                                                   const double* area, int64_t n, double* out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && diags && n_diag >= 0, "plan_add_area_weighted_sums_f64: bad argument");
    std::vector<const double*> d(diags, diags + n_diag);
    plan->ops.push_back([=](void* s) { return fv3_area_weighted_sums_f64(d.data(), n_diag, area, n, out, s); });
    return FV3_OK;
}

extern "C" int fv3_plan_add_area_weighted_row_sums_f64(fv3_plan* plan, const double* const* diags, int n_diag,
                                                       const double* area, int64_t nrows, int row_len,
                                                       double* partial, int64_t partial_ld)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && diags && n_diag >= 0, "plan_add_area_weighted_row_sums_f64: bad argument");
    std::vector<const double*> d(diags, diags + n_diag);
    plan->ops.push_back([=](void* s) {
        return fv3_area_weighted_row_sums_f64(d.data(), n_diag, area, nrows, row_len, partial, partial_ld, s);
    });
    return FV3_OK;
}

extern "C" int fv3_plan_add_level_sums_u8(fv3_plan* plan, const unsigned char* x, fv3_layout x_l, int64_t ncol,
                                          int nz, double* out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan, "plan_add_level_sums_u8: NULL plan");
    plan->ops.push_back([=](void* s) { return fv3_level_sums_u8(x, x_l, ncol, nz, out, s); });
    return FV3_OK;
}

extern "C" int fv3_plan_add_fold_rows(fv3_plan* plan, const double* rows, int64_t nrows, int width, double* out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan, "plan_add_fold_rows: NULL plan");
    plan->ops.push_back([=](void* s) { return fv3_fold_rows(rows, nrows, width, out, s); });
    return FV3_OK;
}

extern "C" int fv3_plan_add_step_partials_f64(fv3_plan* plan, const double* const* diags, int n_diag,
                                              const double* area, int64_t nrows, int row_len, double* partial,
                                              int64_t partial_ld, const unsigned char* limiter, fv3_layout lim_l,
                                              int64_t ncol, int nz, double* level_out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && diags && n_diag >= 0, "plan_add_step_partials_f64: bad argument");
    std::vector<const double*> d(diags, diags + n_diag);
    plan->ops.push_back([=](void* s) {
        return fv3_step_partials_f64(d.data(), n_diag, area, nrows, row_len, partial, partial_ld, limiter, lim_l,
                                     ncol, nz, level_out, s);
    });
    return FV3_OK;
}

extern "C" int fv3_plan_add_fold_rows_repeat(fv3_plan* plan, const double* rows, int64_t nrows, int width,
                                             int times, double* rep, double* out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan, "plan_add_fold_rows_repeat: NULL plan");
    plan->ops.push_back([=](void* s) { return fv3_fold_rows_repeat(rows, nrows, width, times, rep, out, s); });
    return FV3_OK;
}

// device-to-device copy of `bytes` (hipMemcpyAsync on the plan's stream)
extern "C" int fv3_plan_add_copy(fv3_plan* plan, void* dst, const void* src, size_t bytes)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && (bytes == 0 || (dst && src)), "plan_add_copy: bad argument");
    plan->ops.push_back([=](void* s) -> int {
        if (bytes) FV3_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s));
        return FV3_OK;
    });
    return FV3_OK;
}

// `times` back-to-back copies of `bytes` (a multiple of 4) into dst, one launch
extern "C" int fv3_plan_add_repeat(fv3_plan* plan, void* dst, const void* src, size_t bytes, int times)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(plan && times >= 0 && bytes % 4 == 0, "plan_add_repeat: bad argument (bytes must be a multiple of 4)");
    FV3_REQUIRE(bytes == 0 || times == 0 || (dst && src), "plan_add_repeat: NULL array");
    const int64_t n = (int64_t)(bytes / 4);
    plan->ops.push_back([=](void* s) -> int {
        if (n == 0 || times == 0) return FV3_OK;
        hipLaunchKernelGGL(repeat_words_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s,
                           (const unsigned*)src, n, times, (unsigned*)dst);
        FV3_LAUNCH_CHECK();
        return FV3_OK;
    });
    return FV3_OK;
}
