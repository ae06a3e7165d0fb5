#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void layout(float* out, float* aval, float* bval)
{
    int l = threadIdx.x;
    float a = aval[l], b = bval[l];
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}
template <int NACC>
__global__ __launch_bounds__(256) void thr(float* out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    f4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b + j, acc[j], 0, 0, 0);
    }
    float s = 0;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void thr16(float* out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    f4 acc[NACC];
    for (int j = 0; j < NACC; ++j) acc[j] = f4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b + j, acc[j], 0, 0, 0);
    }
    float s = 0;
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main()
{
    float *out, *a, *b;
    hipMalloc(&out, 1 << 26);
    hipMalloc(&a, 256);
    hipMalloc(&b, 256);
    float ha[64], hb[64], ho[256];
    // A: lane l -> 1 + l (distinct); B: unit  -> find which lanes contribute
    for (int l = 0; l < 64; ++l) { ha[l] = (float)(l + 1); hb[l] = (float)(1000 * (l + 1)); }
    // probe 1: a = l+1, b = 1 only at lane j -> D = a_i * 1 where block/col matches
    for (int j : {0, 1, 2, 3, 4, 5}) {
        for (int l = 0; l < 64; ++l) hb[l] = (l == j) ? 1.0f : 0.0f;
        hipMemcpy(a, ha, 256, hipMemcpyHostToDevice);
        hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
        layout<<<1, 64>>>(out, a, b);
        hipMemcpy(ho, out, 1024, hipMemcpyDeviceToHost);
        printf("B one-hot at lane %d: nonzero D (lane,reg)=A-lane:", j);
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 4; ++i)
                if (ho[l * 4 + i] != 0) printf(" (%d,%d)=%g", l, i, ho[l * 4 + i]);
        printf("\n");
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int iters = 4096, blocks = 256 * 8;
    for (int rep = 0; rep < 2; ++rep) {
        thr<16><<<blocks, 256>>>(out, 64);
        hipEventRecord(e0);
        thr<16><<<blocks, 256>>>(out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double fl = 2.0 * 4 * 4 * 1 * 16 * 16.0 * iters * (blocks * 4.0);
        printf("4x4x1_16b  16 acc: %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
        thr16<16><<<blocks, 256>>>(out, 64);
        hipEventRecord(e0);
        thr16<16><<<blocks, 256>>>(out, iters / 4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        fl = 2.0 * 16 * 16 * 4 * 16.0 * (iters / 4) * (blocks * 4.0);
        printf("16x16x4    16 acc: %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
    }
    return 0;
}
