// Microbenchmark: wave-instruction issue rate of common VALU forms on gfx950 (cycles per
// wave64 instruction per SIMD with many waves resident).  Build with -fno-slp-vectorize so the
// scalar forms stay scalar.  usage: pk_fma
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N 16
#define ITERS 2048

__global__ void __launch_bounds__(256) k_fma(float* out, float a, float b)
{
    float x[N];
    for (int i = 0; i < N; i++) x[i] = threadIdx.x * 1e-3f + i;
    const float bv = b + threadIdx.x * 1e-9f; // keep b in a VGPR (one SGPR operand per VOP3)
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = fmaf(x[i], a, bv);
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_pkfma(float* out, float a, float b)
{
    f2 x[N];
    for (int i = 0; i < N; i++) x[i] = f2{threadIdx.x * 1e-3f + i, 1.0f + i};
    const f2 av = {a, a}, bv = {b + threadIdx.x * 1e-9f, b};
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = __builtin_elementwise_fma(x[i], av, bv);
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_add(float* out, float a, float b)
{
    float x[N];
    for (int i = 0; i < N; i++) x[i] = threadIdx.x * 1e-3f + i;
    const float bv = b + threadIdx.x * 1e-9f;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = x[i] + bv;
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_iadd(float* out, float a, float b)
{
    unsigned x[N];
    for (int i = 0; i < N; i++) x[i] = threadIdx.x * 7u + i;
    const unsigned bv = threadIdx.x * 3u + 1u;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = (x[i] ^ bv) + 0x9E3779B9u; // 2 VALU
    unsigned s = 0;
    for (int i = 0; i < N; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}
__global__ void __launch_bounds__(256) k_max(float* out, float a, float b)
{
    float x[N];
    for (int i = 0; i < N; i++) x[i] = threadIdx.x * 1e-3f + i;
    const float bv = b + threadIdx.x * 1e-9f;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = fmaxf(x[i], bv) - a; // max + sub
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


#define KSCALAR(NAME, T, INIT, BODY)                                                      \
    __global__ void __launch_bounds__(256) NAME(float* out, float a, float b)             \
    {                                                                                     \
        T x[N];                                                                           \
        for (int i = 0; i < N; i++) x[i] = INIT;                                          \
        const float bv = b + threadIdx.x * 1e-9f, cv = a + threadIdx.x * 1e-9f;           \
        for (int it = 0; it < ITERS; it++)                                                \
            _Pragma("unroll") for (int i = 0; i < N; i++) { BODY; }                       \
        float s = 0;                                                                      \
        for (int i = 0; i < N; i++) s += (float)x[i];                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
    }
KSCALAR(k_mul, float, threadIdx.x * 1e-3f + i, x[i] = x[i] * bv)
KSCALAR(k_fmavv, float, threadIdx.x * 1e-3f + i, x[i] = fmaf(x[i], cv, bv))
KSCALAR(k_cmpsel, float, threadIdx.x * 1e-3f + i, x[i] = x[i] < bv ? cv : x[i])
KSCALAR(k_max3, float, threadIdx.x * 1e-3f + i, x[i] = fmaxf(fmaxf(x[i], bv), cv))
KSCALAR(k_rcp, float, threadIdx.x * 1e-3f + i, x[i] = __builtin_amdgcn_rcpf(x[i]))
KSCALAR(k_mulu, unsigned, threadIdx.x * 7u + i, x[i] = x[i] * 0x7FEB352Du)
__global__ void __launch_bounds__(256) k_pkmul(float* out, float a, float b)
{
    f2 x[N];
    for (int i = 0; i < N; i++) x[i] = f2{threadIdx.x * 1e-3f + i, 1.0f + i};
    const f2 bv = {b + threadIdx.x * 1e-9f, b};
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = x[i] * bv;
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_pkadd(float* out, float a, float b)
{
    f2 x[N];
    for (int i = 0; i < N; i++) x[i] = f2{threadIdx.x * 1e-3f + i, 1.0f + i};
    const f2 bv = {b + threadIdx.x * 1e-9f, b};
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < N; i++) x[i] = x[i] + bv;
    float s = 0;
    for (int i = 0; i < N; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, float, float);
static void run(const char* name, kfn k, double valu_per_lane_iter, float* out)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 8192;
    float ms = 0;
    for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        k<<<blocks, 256>>>(out, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const double waves = blocks * 4.0;
    const double winstr = waves * ITERS * valu_per_lane_iter; // wave-instructions
    const double cyc_per_simd = ms * 1e-3 * 2.4e9;
    printf("%-8s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms,
           cyc_per_simd / (winstr / 1024.0));
}
int main()
{
    float* out;
    hipMalloc(&out, 256 * 8192 * 4);
    run("fma", k_fma, N, out);
    run("pk_fma", k_pkfma, N, out);
    run("add", k_add, N, out);
    run("iadd", k_iadd, 2 * N, out);
    run("max", k_max, 2 * N, out);
    run("mul", k_mul, N, out);
    run("fma_vv", k_fmavv, N, out);
    run("cmpsel", k_cmpsel, 2 * N, out);
    run("max3", k_max3, N, out);
    run("rcp", k_rcp, N, out);
    run("mul_u32", k_mulu, N, out);
    run("pk_mul", k_pkmul, N, out);
    run("pk_add", k_pkadd, N, out);
    return 0;
}
