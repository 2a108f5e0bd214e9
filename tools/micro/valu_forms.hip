// Microbenchmark: issue cost (cycles per wave64 instruction per SIMD, many waves resident) of
// VALU encodings on gfx950, isolating SGPR operands, VOP2 accumulate forms and compares.
// Vector instructions only.  usage: valu_forms
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 16
#define ITERS 1024

#define KASM(NAME, INSTR, ...)                                                             \
    __global__ void __launch_bounds__(256) NAME(float* out, float a, float b)              \
    {                                                                                      \
        float x[N];                                                                        \
        for (int i = 0; i < N; i++) x[i] = threadIdx.x * 1e-3f + i;                        \
        float bv = b + threadIdx.x * 1e-9f, cv = a + threadIdx.x * 1e-9f;                  \
        for (int it = 0; it < ITERS; it++)                                                 \
            _Pragma("unroll") for (int i = 0; i < N; i++) asm volatile(INSTR : __VA_ARGS__);\
        float s = 0;                                                                       \
        for (int i = 0; i < N; i++) s += x[i];                                             \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s + bv + cv;                          \
    }

KASM(k_fma_vvv, "v_fma_f32 %0, %1, %2, %0", "+v"(x[i]) : "v"(cv), "v"(bv))
KASM(k_fma_svv, "v_fma_f32 %0, %1, %2, %0", "+v"(x[i]) : "s"(a), "v"(bv))
KASM(k_fmac_vv, "v_fmac_f32_e32 %0, %1, %2", "+v"(x[i]) : "v"(cv), "v"(bv))
KASM(k_fmac_sv, "v_fmac_f32_e32 %0, %1, %2", "+v"(x[i]) : "s"(a), "v"(bv))
KASM(k_add_vv, "v_add_f32_e32 %0, %1, %0", "+v"(x[i]) : "v"(bv))
KASM(k_add_sv, "v_add_f32_e32 %0, %1, %0", "+v"(x[i]) : "s"(a))
KASM(k_add_e64_sv, "v_add_f32_e64 %0, %1, %0", "+v"(x[i]) : "s"(a))
KASM(k_mul_sv, "v_mul_f32_e32 %0, %1, %0", "+v"(x[i]) : "s"(a))
KASM(k_sub_abs_v, "v_sub_f32_e64 %0, |%0|, %1", "+v"(x[i]) : "v"(bv))
KASM(k_cmp_vcc, "v_cmp_lt_f32_e32 vcc, %0, %1", "+v"(x[i]) : "v"(bv) : "vcc")
KASM(k_cmp_e64, "v_cmp_lt_f32_e64 s[40:41], %0, %1", "+v"(x[i]) : "v"(bv) : "s40", "s41")
KASM(k_cmp_e64_s, "v_cmp_lt_f32_e64 s[40:41], %0, %1", "+v"(x[i]) : "s"(a) : "s40", "s41")
KASM(k_cnd_e64, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]", "+v"(x[i]) : "v"(bv) : "s40", "s41")
KASM(k_cnd_vcc, "v_cndmask_b32_e32 %0, %0, %1, vcc", "+v"(x[i]) : "v"(bv) : "vcc")
KASM(k_xor_vv, "v_xor_b32_e32 %0, %1, %0", "+v"(x[i]) : "v"(bv))
KASM(k_xor_sv, "v_xor_b32_e32 %0, %1, %0", "+v"(x[i]) : "s"(a))
KASM(k_max_vv, "v_max_f32_e32 %0, %1, %0", "+v"(x[i]) : "v"(bv))
KASM(k_max3_vvv, "v_max3_f32 %0, %1, %2, %0", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_med3_vvv, "v_med3_f32 %0, %1, %2, %0", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_pkfma_vvv, "v_pk_fma_f32 %0, %1, %2, %0", "+v"(*(double*)&x[i & ~1]) : "v"(*(double*)&x[(i + 2) & 15]), "v"(*(double*)&x[(i + 4) & 15]))
KASM(k_pkadd_vv, "v_pk_add_f32 %0, %1, %0", "+v"(*(double*)&x[i & ~1]) : "v"(*(double*)&x[(i + 2) & 15]))
KASM(k_mov_sv, "v_mov_b32_e32 %0, %1", "=v"(x[i]) : "s"(a))
// round 6: forms a quantised-node slab test could use instead of v_cvt_f32_ubyte + v_fma
KASM(k_cvt_ubyte1, "v_cvt_f32_ubyte1_e32 %0, %0", "+v"(x[i]))
KASM(k_mov_sdwa_byte, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2", "+v"(x[i]) : "v"(bv))
KASM(k_mul_u24_sdwa, "v_mul_u32_u24_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD", "+v"(x[i]) : "v"(bv))
KASM(k_fma_mix, "v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_fma_mix_hi, "v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_pk_fma_f16, "v_pk_fma_f16 %0, %1, %2, %0", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_perm, "v_perm_b32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_max_u32, "v_max_u32_e32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_max3_u32, "v_max3_u32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_cvt_pk_fp8, "v_cvt_pk_f32_fp8_e32 %0, %1", "+v"(*(double*)&x[i & ~1]) : "v"(bv))
KASM(k_bfi, "v_bfi_b32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_and_vv, "v_and_b32_e32 %0, 3, %0", "+v"(x[i]))

KASM(k_mullo_u32, "v_mul_lo_u32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_mulhi_u32, "v_mul_hi_u32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_mul_u24, "v_mul_u32_u24_e32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_xad_u32, "v_xad_u32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1", "+v"(x[i]) : "v"(bv))
KASM(k_lshr_b32, "v_lshrrev_b32_e32 %0, 16, %0", "+v"(x[i]))
KASM(k_alignbit, "v_alignbit_b32 %0, %0, %1, 13", "+v"(x[i]) : "v"(bv))
KASM(k_bfe_u32, "v_bfe_u32 %0, %0, 8, 8", "+v"(x[i]))
KASM(k_cvt_f32_u32, "v_cvt_f32_u32_e32 %0, %0", "+v"(x[i]))
KASM(k_sin, "v_sin_f32_e32 %0, %0", "+v"(x[i]))
KASM(k_exp, "v_exp_f32_e32 %0, %0", "+v"(x[i]))
KASM(k_sqrt, "v_sqrt_f32_e32 %0, %0", "+v"(x[i]))
KASM(k_fma_lit, "v_fmaak_f32 %0, %0, %1, 0x3f000000", "+v"(x[i]) : "v"(bv))
KASM(k_add_inl, "v_add_f32_e32 %0, 0.5, %0", "+v"(x[i]))
KASM(k_cnd_sgpr_pair, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]", "+v"(x[i]) : "v"(bv) : "s40", "s41")
KASM(k_readlane, "v_readlane_b32 s40, %0, 3", "+v"(x[i]) :: "s40")
KASM(k_and_or, "v_and_or_b32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_min_f32, "v_min_f32_e32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_med3_i32, "v_med3_i32 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_min_u32, "v_min_u32_e32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_sub_u32, "v_sub_u32_e32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_ldexp, "v_ldexp_f32 %0, %0, %1", "+v"(x[i]) : "v"(bv))
KASM(k_dot2, "v_dot2_f32_f16 %0, %0, %1, %2", "+v"(x[i]) : "v"(bv), "v"(cv))
KASM(k_cmpx, "v_cmp_class_f32_e64 s[40:41], %0, %1", "+v"(x[i]) : "v"(bv) : "s40", "s41")

typedef void (*kfn)(float*, float, float);
static void run(const char* name, kfn k, float* out)
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
    const double winstr = blocks * 4.0 * ITERS * N;
    printf("%-14s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms,
           ms * 1e-3 * 2.4e9 / (winstr / 1024.0));
}
#define RUN(k) run(#k, k, out)
int main()
{
    float* out;
    hipMalloc(&out, 256 * 8192 * 4);
    RUN(k_fma_vvv);
    RUN(k_fma_svv);
    RUN(k_fmac_vv);
    RUN(k_fmac_sv);
    RUN(k_add_vv);
    RUN(k_add_sv);
    RUN(k_add_e64_sv);
    RUN(k_mul_sv);
    RUN(k_sub_abs_v);
    RUN(k_cmp_vcc);
    RUN(k_cmp_e64);
    RUN(k_cmp_e64_s);
    RUN(k_cnd_e64);
    RUN(k_cnd_vcc);
    RUN(k_xor_vv);
    RUN(k_xor_sv);
    RUN(k_max_vv);
    RUN(k_max3_vvv);
    RUN(k_med3_vvv);
    RUN(k_mullo_u32);
    RUN(k_mulhi_u32);
    RUN(k_mul_u24);
    RUN(k_mad_u24);
    RUN(k_xad_u32);
    RUN(k_lshl_add);
    RUN(k_lshr_b32);
    RUN(k_alignbit);
    RUN(k_bfe_u32);
    RUN(k_cvt_f32_u32);
    RUN(k_sin);
    RUN(k_exp);
    RUN(k_sqrt);
    RUN(k_fma_lit);
    RUN(k_add_inl);
    RUN(k_cnd_sgpr_pair);
    RUN(k_readlane);
    RUN(k_and_or);
    RUN(k_min_f32);
    RUN(k_med3_i32);
    RUN(k_min_u32);
    RUN(k_sub_u32);
    RUN(k_ldexp);
    RUN(k_dot2);
    RUN(k_cmpx);
    RUN(k_mov_sv);
    RUN(k_cvt_ubyte1);
    RUN(k_mov_sdwa_byte);
    RUN(k_mul_u24_sdwa);
    RUN(k_fma_mix);
    RUN(k_fma_mix_hi);
    RUN(k_pk_fma_f16);
    RUN(k_perm);
    RUN(k_max_u32);
    RUN(k_max3_u32);
    RUN(k_cvt_pk_fp8);
    RUN(k_bfi);
    RUN(k_and_vv);
    return 0;
}
