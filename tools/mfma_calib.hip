// f32 MFMA issue rates on gfx950 (tools only): cycles per instruction on one SIMD,
// back-to-back with 4 independent accumulators, one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/mfma_calib.hip -o tools/variants/libmfma_calib.so
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int OP>
__global__ __launch_bounds__(256) void mfma_kernel(int iters, float a, float b, float* out, uint64_t* clk)
{
    const uint64_t t0 = clock64();
    if constexpr (OP == 0 || OP == 1) {
        f4 c[4] = {};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (OP == 0) c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
                    else c[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[j], 0, 0, 0);
                }
        }
        float s = 0;
        for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
        if (s == 1234.5f) out[threadIdx.x] = s;
    } else {
        f16v c[4] = {};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[j], 0, 0, 0);
        }
        float s = 0;
        for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][15];
        if (s == 1234.5f) out[threadIdx.x] = s;
    }
    const uint64_t t1 = clock64();
    if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

extern "C" int mfma_calib_run(int op, int blocks, int iters, float* out, uint64_t* clk, void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (op == 0) mfma_kernel<0><<<blocks, 256, 0, s>>>(iters, 1.0f, 1e-7f, out, clk);
    else if (op == 1) mfma_kernel<1><<<blocks, 256, 0, s>>>(iters, 1.0f, 1e-7f, out, clk);
    else mfma_kernel<2><<<blocks, 256, 0, s>>>(iters, 1.0f, 1e-7f, out, clk);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
