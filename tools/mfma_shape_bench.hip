// Microbenchmark (tools only): the split kernel's hidden-layer inner loop on the two bf16
// MFMA shapes, to price the shape before building a kernel on it.
//   S16: 8 waves (2 per SIMD), 16 columns per wave, v_mfma_f32_16x16x32_bf16, 16 unit tiles
//        of 16 per 32-deep chunk, A fragments (hi, lo) from LDS, B (hi, lo) in registers:
//        the shape dense_b3_kernel runs today.
//   S32: 4 waves (1 per SIMD), 32 columns per wave, v_mfma_f32_32x32x16_bf16, 8 unit
//        tiles of 32 per 16-deep chunk.
// Both: three MFMAs per (A, B) fragment pair (bf16x3), one barrier per chunk, FILL
// independent v_fma_f32 per MFMA (the splits / epilogue arithmetic), and the same FLOPs
// per launch.  Results are meaningless numbers; only the time is read.
#include <hip/hip_runtime.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int FILL>
__device__ __forceinline__ void fill(float (&x)[4])
{
#pragma unroll
    for (int i = 0; i < FILL; ++i) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x[i & 3]));
}

template <int FILL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void s16_kernel(int nch, float* out)
{
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x & 63;
    bf16x8 B[8][2];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        for (int h = 0; h < 2; ++h)
            for (int j = 0; j < 8; ++j) B[c][h][j] = (__bf16)(float)(lane + j + c + h);
    f4 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = f4{0, 0, 0, 0};
    float x[4] = {1, 2, 3, 4};
    for (int c = 0; c < nch; ++c) {
        __syncthreads();
        const char* slot = lds + (c & 1) * 32768;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(slot + t * 2048 + lane * 16);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(slot + t * 2048 + 1024 + lane * 16);
            const bf16x8(&b)[2] = B[c & 7];
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b[0], acc[t], 0, 0, 0);
            fill<FILL>(x);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b[0], acc[t], 0, 0, 0);
            fill<FILL>(x);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b[1], acc[t], 0, 0, 0);
            fill<FILL>(x);
        }
    }
    float s = x[0] + x[1] + x[2] + x[3];
#pragma unroll
    for (int t = 0; t < 16; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    if (s == 1234.5f) out[blockIdx.x] = s;
}

template <int FILL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void s32_kernel(int nch, float* out)
{
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x & 63;
    bf16x8 B[16][2];
#pragma unroll
    for (int c = 0; c < 16; ++c)
        for (int h = 0; h < 2; ++h)
            for (int j = 0; j < 8; ++j) B[c][h][j] = (__bf16)(float)(lane + j + c + h);
    f16v acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    float x[4] = {1, 2, 3, 4};
    for (int c = 0; c < nch; ++c) {
        __syncthreads();
        const char* slot = lds + (c & 1) * 16384;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(slot + t * 2048 + lane * 16);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(slot + t * 2048 + 1024 + lane * 16);
            const bf16x8(&b)[2] = B[c & 15];
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b[0], acc[t], 0, 0, 0);
            fill<FILL>(x);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b[0], acc[t], 0, 0, 0);
            fill<FILL>(x);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b[1], acc[t], 0, 0, 0);
            fill<FILL>(x);
        }
    }
    float s = x[0] + x[1] + x[2] + x[3];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        for (int r = 0; r < 16; ++r) s += acc[t][r];
    if (s == 1234.5f) out[blockIdx.x] = s;
}

// shape 16 / 32, fill 0 / 2 / 4 / 8: mean ms per launch of `reps` launches on `blocks`
// blocks (`lds` dynamic bytes per block, sized to one block per CU), `nch` chunks each
extern "C" int mfma_shape_run(int shape, int fillv, int blocks, int nch, int reps, int lds, float* out, float* ms)
{
    const void* k = nullptr;
#define PICK(S, F) k = (const void*)S##_kernel<F>
    if (shape == 16) {
        if (fillv == 0) PICK(s16, 0); else if (fillv == 2) PICK(s16, 2); else if (fillv == 4) PICK(s16, 4); else PICK(s16, 8);
    } else {
        if (fillv == 0) PICK(s32, 0); else if (fillv == 2) PICK(s32, 2); else if (fillv == 4) PICK(s32, 4); else PICK(s32, 8);
    }
#undef PICK
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 1;
    const int threads = shape == 16 ? 512 : 256;
    void* args[] = {&nch, &out};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernel(k, dim3(blocks), dim3(threads), args, lds, 0);
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernel(k, dim3(blocks), dim3(threads), args, lds, 0);
    hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return 2;
    float t = 0;
    hipEventElapsedTime(&t, e0, e1);
    *ms = t / reps;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
