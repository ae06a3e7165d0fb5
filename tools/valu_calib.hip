// VALU issue-rate calibration on gfx950 (tools only, never part of the product).
//
// Each kernel runs 8 independent dependency chains per lane of one pinned VALU opcode
// (inline asm, so the instruction stream is exactly the named opcode plus the loop
// counter), at 1..8 waves per SIMD.  The measured rate, in wave-instructions per CU per
// shader clock, is the peak the bench's valu_issue_frac divides by.  The shader clock is
// read in-kernel (s_memtime against the 100 MHz s_memrealtime), so clock throttling does
// not bias the per-cycle rate.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/valu_calib.hip -o tools/variants/libvalu_calib.so
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f2 __attribute__((ext_vector_type(2)));

enum Op {
    ADD = 0, FMA = 1, MUL = 2, RCP = 3, CND = 4, PK_ADD = 5, PK_FMA = 6, ADD_RCP = 7, EXP = 8, DIV = 9,
    CND32 = 10, CMP = 11, MAX = 12, MOV = 13, DSCALE = 14, DFMAS = 15, DFIXUP = 16, IADD = 17, BFE = 18
};

template <int OP>
__device__ __forceinline__ void step(float& x, f2& p, float a, float b, uint64_t m)
{
    if constexpr (OP == ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
    if constexpr (OP == EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(x));
    if constexpr (OP == CND) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "s"(m));
    if constexpr (OP == PK_ADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p) : "v"(f2{a, b}));
    if constexpr (OP == PK_FMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p) : "v"(f2{a, a}), "v"(f2{b, b}));
    if constexpr (OP == ADD_RCP) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
        asm volatile("v_rcp_f32 %0, %0" : "+v"(p.x));
    }
    if constexpr (OP == DIV) x = __fdiv_rn(x, a);  // the correctly rounded IEEE division sequence
    if constexpr (OP == CND32) asm volatile("v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(x) : "v"(a));
    if constexpr (OP == CMP) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" : : "v"(x), "v"(a) : "vcc");
    if constexpr (OP == MAX) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(a));
    if constexpr (OP == DSCALE) asm volatile("v_div_scale_f32 %0, vcc, %0, %1, %0" : "+v"(x) : "v"(a) : "vcc");
    if constexpr (OP == DFMAS) asm volatile("v_div_fmas_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == DFIXUP) asm volatile("v_div_fixup_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == IADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == BFE) asm volatile("v_bfe_u32 %0, %0, 23, 8" : "+v"(x));
}

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(int iters, float a, float b, float* out, uint64_t* clk)
{
    float x[8];
    f2 p[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        x[c] = 1.0f + 1e-3f * (threadIdx.x + c);
        p[c] = f2{x[c], -x[c]};
    }
    const uint64_t m = 0x5555555555555555ull;
    const uint64_t t0 = clock64(), r0 = wall_clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 8; ++c) step<OP>(x[c], p[c], a, b, m);
    }
    const uint64_t t1 = clock64(), r1 = wall_clock64();
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c] + p[c].x + p[c].y;
    if (s == 1234.5f) out[threadIdx.x] = s;  // keeps the chains alive; never true here
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

// instructions per wave per loop iteration (the opcode under test)
extern "C" int valu_calib_insts_per_iter(int op) { return op == ADD_RCP ? 64 : 32; }

extern "C" int valu_calib_run(int op, int blocks, int iters, float* out, uint64_t* clk, void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(blocks), b(256);
    switch (op) {
    case ADD: valu_kernel<ADD><<<g, b, 0, s>>>(iters, 1e-7f, 0.5f, out, clk); break;
    case FMA: valu_kernel<FMA><<<g, b, 0, s>>>(iters, 0.999f, 1e-7f, out, clk); break;
    case MUL: valu_kernel<MUL><<<g, b, 0, s>>>(iters, 0.9999f, 0.0f, out, clk); break;
    case RCP: valu_kernel<RCP><<<g, b, 0, s>>>(iters, 0.0f, 0.0f, out, clk); break;
    case CND: valu_kernel<CND><<<g, b, 0, s>>>(iters, 2.0f, 0.0f, out, clk); break;
    case PK_ADD: valu_kernel<PK_ADD><<<g, b, 0, s>>>(iters, 1e-7f, 1e-7f, out, clk); break;
    case PK_FMA: valu_kernel<PK_FMA><<<g, b, 0, s>>>(iters, 0.999f, 1e-7f, out, clk); break;
    case ADD_RCP: valu_kernel<ADD_RCP><<<g, b, 0, s>>>(iters, 1e-7f, 0.0f, out, clk); break;
    case EXP: valu_kernel<EXP><<<g, b, 0, s>>>(iters, 0.0f, 0.0f, out, clk); break;
    case DIV: valu_kernel<DIV><<<g, b, 0, s>>>(iters, 1.0001f, 0.0f, out, clk); break;
    case CND32: valu_kernel<CND32><<<g, b, 0, s>>>(iters, 2.0f, 0.0f, out, clk); break;
    case CMP: valu_kernel<CMP><<<g, b, 0, s>>>(iters, 2.0f, 0.0f, out, clk); break;
    case MAX: valu_kernel<MAX><<<g, b, 0, s>>>(iters, 2.0f, 0.0f, out, clk); break;
    case MOV: valu_kernel<MOV><<<g, b, 0, s>>>(iters, 2.0f, 0.0f, out, clk); break;
    case DSCALE: valu_kernel<DSCALE><<<g, b, 0, s>>>(iters, 1.5f, 0.0f, out, clk); break;
    case DFMAS: valu_kernel<DFMAS><<<g, b, 0, s>>>(iters, 0.999f, 1e-7f, out, clk); break;
    case DFIXUP: valu_kernel<DFIXUP><<<g, b, 0, s>>>(iters, 1.5f, 2.0f, out, clk); break;
    case IADD: valu_kernel<IADD><<<g, b, 0, s>>>(iters, 1.0f, 0.0f, out, clk); break;
    case BFE: valu_kernel<BFE><<<g, b, 0, s>>>(iters, 0.0f, 0.0f, out, clk); break;
    default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
