// VALU issue-rate microbenchmark (gfx950): wave64 VALU instructions per
// SIMD-cycle for independent fp32 FMA / add chains and a compare+select mix,
// at 8 waves per SIMD.  Prints instructions/s and cycles per instruction per
// SIMD at the measured clock-free rate (assumes 2.4 GHz for the cycle figure).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int kMode>
__global__ __launch_bounds__(256) void valu_kernel(float *out, int iters, float a, float b)
{
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
          x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters; ++i) {
        if constexpr (kMode == 0) {   // 8 independent FMAs
            x0 = __builtin_fmaf(x0, a, b); x1 = __builtin_fmaf(x1, a, b); x2 = __builtin_fmaf(x2, a, b);
            x3 = __builtin_fmaf(x3, a, b); x4 = __builtin_fmaf(x4, a, b); x5 = __builtin_fmaf(x5, a, b);
            x6 = __builtin_fmaf(x6, a, b); x7 = __builtin_fmaf(x7, a, b);
        } else if constexpr (kMode == 1) {   // 8 independent adds
            x0 += a; x1 += b; x2 += a; x3 += b; x4 += a; x5 += b; x6 += a; x7 += b;
        } else if constexpr (kMode == 3) {   // 4 independent packed FMAs (2 fp32 lanes each)
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p0 = {x0, x1}, p1 = {x2, x3}, p2 = {x4, x5}, p3 = {x6, x7};
            const f2 va = {a, a}, vb = {b, b};
            p0 = __builtin_elementwise_fma(p0, va, vb); p1 = __builtin_elementwise_fma(p1, va, vb);
            p2 = __builtin_elementwise_fma(p2, va, vb); p3 = __builtin_elementwise_fma(p3, va, vb);
            x0 = p0.x; x1 = p0.y; x2 = p1.x; x3 = p1.y; x4 = p2.x; x5 = p2.y; x6 = p3.x; x7 = p3.y;
        } else if constexpr (kMode == 4) {   // 8 independent reciprocals (transcendental)
            x0 = __builtin_amdgcn_rcpf(x0); x1 = __builtin_amdgcn_rcpf(x1); x2 = __builtin_amdgcn_rcpf(x2);
            x3 = __builtin_amdgcn_rcpf(x3); x4 = __builtin_amdgcn_rcpf(x4); x5 = __builtin_amdgcn_rcpf(x5);
            x6 = __builtin_amdgcn_rcpf(x6); x7 = __builtin_amdgcn_rcpf(x7);
        } else if constexpr (kMode == 5) {   // 6 FMAs + 2 reciprocals (do they overlap?)
            x0 = __builtin_fmaf(x0, a, b); x1 = __builtin_fmaf(x1, a, b); x2 = __builtin_amdgcn_rcpf(x2);
            x3 = __builtin_fmaf(x3, a, b); x4 = __builtin_fmaf(x4, a, b); x5 = __builtin_fmaf(x5, a, b);
            x6 = __builtin_amdgcn_rcpf(x6); x7 = __builtin_fmaf(x7, a, b);
        } else if constexpr (kMode == 6) {   // 8 independent square roots
            x0 = __builtin_amdgcn_sqrtf(x0); x1 = __builtin_amdgcn_sqrtf(x1); x2 = __builtin_amdgcn_sqrtf(x2);
            x3 = __builtin_amdgcn_sqrtf(x3); x4 = __builtin_amdgcn_sqrtf(x4); x5 = __builtin_amdgcn_sqrtf(x5);
            x6 = __builtin_amdgcn_sqrtf(x6); x7 = __builtin_amdgcn_sqrtf(x7);
        } else if constexpr (kMode == 7) {   // 8 independent multiplies
            x0 *= a; x1 *= b; x2 *= a; x3 *= b; x4 *= a; x5 *= b; x6 *= a; x7 *= b;
        } else if constexpr (kMode == 8) {   // 4 independent packed f16 FMAs (2 halves each)
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            h2 p0 = {(_Float16)x0, (_Float16)x1}, p1 = {(_Float16)x2, (_Float16)x3};
            h2 p2 = {(_Float16)x4, (_Float16)x5}, p3 = {(_Float16)x6, (_Float16)x7};
            const h2 va = {(_Float16)a, (_Float16)a}, vb = {(_Float16)b, (_Float16)b};
            for (int k = 0; k < 4; ++k) {
                p0 = __builtin_elementwise_fma(p0, va, vb); p1 = __builtin_elementwise_fma(p1, va, vb);
                p2 = __builtin_elementwise_fma(p2, va, vb); p3 = __builtin_elementwise_fma(p3, va, vb);
            }
            x0 = (float)p0.x; x1 = (float)p0.y; x2 = (float)p1.x; x3 = (float)p1.y;
            x4 = (float)p2.x; x5 = (float)p2.y; x6 = (float)p3.x; x7 = (float)p3.y;
        } else if constexpr (kMode == 9) {   // 8 independent f32 compares to lane masks, OR-combined
            uint64_t m = 0;
            m |= __builtin_amdgcn_fcmpf(x0, a, 5); m |= __builtin_amdgcn_fcmpf(x1, b, 5);
            m |= __builtin_amdgcn_fcmpf(x2, a, 5); m |= __builtin_amdgcn_fcmpf(x3, b, 5);
            m |= __builtin_amdgcn_fcmpf(x4, a, 5); m |= __builtin_amdgcn_fcmpf(x5, b, 5);
            m |= __builtin_amdgcn_fcmpf(x6, a, 5); m |= __builtin_amdgcn_fcmpf(x7, b, 5);
            x0 += (float)(m & 1u);
        } else {   // compare + select pairs (VOPC to vcc / SGPR + v_cndmask)
            x0 = x0 < a ? x0 + b : x0 - b; x1 = x1 < a ? x1 + b : x1 - b;
            x2 = x2 < a ? x2 + b : x2 - b; x3 = x3 < a ? x3 + b : x3 - b;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

template <int kMode>
void run(const char *name, int instr_per_iter, float *out)
{
    const int blocks = 256 * 8, iters = 4096;   // 8 blocks of 4 waves per CU = 8 waves / SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(valu_kernel<kMode>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(valu_kernel<kMode>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)blocks * 4 * iters * instr_per_iter;   // wave-instructions
    const double rate = instr / (ms * 1e-3);
    printf("{\"mode\": \"%s\", \"ms\": %.4f, \"wave_instr_per_s\": %.4g, \"cycles_per_instr_per_simd_at_2.4GHz\": %.3f}\n",
           name, ms, rate, 1024 * 2.4e9 / rate);
}

int main()
{
    float *out; hipMalloc(&out, 256 * 8 * 256 * 4);
    run<0>("fma x8", 8, out);
    run<1>("add x8", 8, out);
    run<2>("cmp+cndmask+add x4", 12, out);
    run<3>("pk_fma x4 (8 fp32 FMAs)", 4, out);
    run<4>("rcp x8", 8, out);
    run<5>("fma x6 + rcp x2", 8, out);
    run<6>("sqrt x8", 8, out);
    run<7>("mul x8", 8, out);   // per pair: v_cmp, v_add, v_sub, v_cndmask ~ 3 VALU
    run<8>("pk_fma_f16 x16 (32 f16 FMAs; + 8 cvt in / 8 out per 4 iters)", 16, out);
    run<9>("cmp-to-mask x8 (+1 add)", 9, out);
    hipFree(out);
    return 0;
}
