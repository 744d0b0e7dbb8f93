// Issue cost of single VALU instructions on gfx950 (diagnostic).  Each kernel runs 8
// independent chains of one instruction per thread in a loop; full-chip instruction rate
// -> cycles per wave-instruction per SIMD at the measured clock.
//
//   hipcc --offload-arch=gfx950 -O3 tools/isa_rates.hip -o /tmp/isa_rates && /tmp/isa_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

#define KERNEL(NAME, T, INIT, ASM)                                                             \
    __global__ __launch_bounds__(256) void NAME(T* out, uint32_t seed) {                       \
        T v0 = INIT(0), v1 = INIT(1), v2 = INIT(2), v3 = INIT(3), v4 = INIT(4), v5 = INIT(5), \
          v6 = INIT(6), v7 = INIT(7);                                                          \
        for (int i = 0; i < ITERS; ++i) {                                                      \
            ASM(v0); ASM(v1); ASM(v2); ASM(v3); ASM(v4); ASM(v5); ASM(v6); ASM(v7);            \
        }                                                                                      \
        out[blockIdx.x * 256 + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;            \
    }

typedef float f2 __attribute__((ext_vector_type(2)));
#define IU(k) (seed + threadIdx.x * 7u + (k))
#define IF(k) ((float)(threadIdx.x + (k)) * 1e-3f + 0.5f)
#define IU64(k) ((uint64_t)(seed + threadIdx.x + (k)))
#define IF2(k) (f2{IF(k), IF(k + 9)})

#define A_ADD(v) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_FMA(v) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v))
#define A_PKFMA(v) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(v))
#define A_PKFMA_SW(v) asm volatile("v_pk_fma_f32 %0, %0, %0, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "+v"(v))
#define A_MULHI(v) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_MULLO(v) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_MUL24(v) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_MAD64(v) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v) : "v"((uint32_t)v) : "vcc")
#define A_SIN(v) asm volatile("v_sin_f32 %0, %0" : "+v"(v))
#define A_LOG(v) asm volatile("v_log_f32 %0, %0" : "+v"(v))
#define A_SQRT(v) asm volatile("v_sqrt_f32 %0, %0" : "+v"(v))
#define A_CVT(v) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(v))
#define A_PERM(v) asm volatile("v_perm_b32 %0, %0, %1, %0" : "+v"(v) : "v"(seed))
#define A_ALIGN(v) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(v) : "v"(seed))
#define A_MED3(v) asm volatile("v_med3_i32 %0, %0, %1, %0" : "+v"(v) : "v"(seed))
#define A_BCNT(v) asm volatile("v_bcnt_u32_b32 %0, %0, %0" : "+v"(v))
#define A_XOR3(v) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(v) : "v"(seed))
#define A_ADD3(v) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(v) : "v"(seed))
#define A_ADDF(v) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v) : "v"((float)seed))
#define A_MULF(v) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v) : "v"((float)seed))
#define A_FMA3(v) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"((float)seed), "v"((float)threadIdx.x))
#define A_PKADD(v) asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(v))
#define A_PKMUL(v) asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(v))
#define A_XOR(v) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_LSHR(v) asm volatile("v_lshrrev_b32 %0, 9, %0" : "+v"(v))
#define A_LSHLADD(v) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(v) : "v"(seed))
#define A_LSHLOR(v) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(v) : "v"(seed))
#define A_BFE(v) asm volatile("v_bfe_u32 %0, %0, %1, 6" : "+v"(v) : "v"(seed))
#define A_MAXF(v) asm volatile("v_max_f32 %0, %0, %1" : "+v"(v) : "v"((float)seed))
#define A_MAX3F(v) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(v) : "v"((float)seed))
#define A_CNDMASK(v) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v) : "v"(seed))
#define A_MOV(v) asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(v + seed))
#define A_CVTI(v) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(v))
#define A_FLOOR(v) asm volatile("v_floor_f32 %0, %0" : "+v"(v))
#define A_MAD24(v) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(v) : "v"(seed))
#define A_RCP(v) asm volatile("v_rcp_f32 %0, %0" : "+v"(v))
#define A_AND_OR(v) asm volatile("v_and_or_b32 %0, %0, %1, %0" : "+v"(v) : "v"(seed))
#define A_SUB(v) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v) : "v"(seed))
#define A_LSHL64(v) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(v))
#define A_PKADD2(v) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v) : "v"(f2{(float)seed, 1.f}))
#define A_PKFMA3(v) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(f2{(float)seed, 1.f}), "v"(f2{2.f, (float)threadIdx.x}))
#define A_PKFMA2S(v) asm volatile("v_pk_fma_f32 %0, %0, %1, %0 op_sel_hi:[1,0,1]" : "+v"(v) : "s"(f2{(float)seed, 1.f}))
#define A_PKMUL2(v) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v) : "v"(f2{(float)seed, 1.f}))
#define A_FMAS(v) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v) : "s"((float)seed), "v"((float)threadIdx.x))
#define A_FMAC(v) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v) : "v"((float)seed), "v"((float)threadIdx.x))
#define A_CNDS(v) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(v) : "v"(seed), "s"((uint64_t)seed))
#define ID(k) ((double)(threadIdx.x + (k)) * 1e-3 + 0.5)
#define A_ADDD(v) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v) : "v"((double)seed))
#define A_MULD(v) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v) : "v"((double)seed))
#define A_FMAD(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"((double)seed), "v"((double)threadIdx.x))
#define A_FMACD(v) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(v) : "v"((double)seed), "v"((double)threadIdx.x))
#define A_CVTD(v) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(v) : "v"((float)v))
#define A_MOVD(v) asm volatile("v_mov_b64 %0, %1" : "=v"(v) : "v"(v + 1.0))
#define A_RCPD(v) asm volatile("v_rcp_f64 %0, %0" : "+v"(v))
#define A_CMP(v) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(v) : "v"(seed) : "vcc")

KERNEL(k_add, uint32_t, IU, A_ADD)
KERNEL(k_fma, float, IF, A_FMA)
KERNEL(k_pkfma, f2, IF2, A_PKFMA)
KERNEL(k_pkfma_sw, f2, IF2, A_PKFMA_SW)
KERNEL(k_mulhi, uint32_t, IU, A_MULHI)
KERNEL(k_mullo, uint32_t, IU, A_MULLO)
KERNEL(k_mul24, uint32_t, IU, A_MUL24)
KERNEL(k_mad64, uint64_t, IU64, A_MAD64)
KERNEL(k_sin, float, IF, A_SIN)
KERNEL(k_log, float, IF, A_LOG)
KERNEL(k_sqrt, float, IF, A_SQRT)
KERNEL(k_cvt, uint32_t, IU, A_CVT)
KERNEL(k_perm, uint32_t, IU, A_PERM)
KERNEL(k_align, uint32_t, IU, A_ALIGN)
KERNEL(k_med3, uint32_t, IU, A_MED3)
KERNEL(k_bcnt, uint32_t, IU, A_BCNT)
KERNEL(k_xor3, uint32_t, IU, A_XOR3)
KERNEL(k_add3, uint32_t, IU, A_ADD3)
KERNEL(k_addf, float, IF, A_ADDF)
KERNEL(k_mulf, float, IF, A_MULF)
KERNEL(k_fma3, float, IF, A_FMA3)
KERNEL(k_pkadd, f2, IF2, A_PKADD)
KERNEL(k_pkmul, f2, IF2, A_PKMUL)
KERNEL(k_xor, uint32_t, IU, A_XOR)
KERNEL(k_lshr, uint32_t, IU, A_LSHR)
KERNEL(k_lshladd, uint32_t, IU, A_LSHLADD)
KERNEL(k_lshlor, uint32_t, IU, A_LSHLOR)
KERNEL(k_bfe, uint32_t, IU, A_BFE)
KERNEL(k_maxf, float, IF, A_MAXF)
KERNEL(k_max3f, float, IF, A_MAX3F)
KERNEL(k_cndmask, uint32_t, IU, A_CNDMASK)
KERNEL(k_mov, uint32_t, IU, A_MOV)
KERNEL(k_cvti, float, IF, A_CVTI)
KERNEL(k_floor, float, IF, A_FLOOR)
KERNEL(k_mad24, uint32_t, IU, A_MAD24)
KERNEL(k_rcp, float, IF, A_RCP)
KERNEL(k_andor, uint32_t, IU, A_AND_OR)
KERNEL(k_sub, uint32_t, IU, A_SUB)
KERNEL(k_lshl64, uint64_t, IU64, A_LSHL64)
KERNEL(k_cmp, uint32_t, IU, A_CMP)
KERNEL(k_pkadd2, f2, IF2, A_PKADD2)
KERNEL(k_pkfma3, f2, IF2, A_PKFMA3)
KERNEL(k_pkfma2s, f2, IF2, A_PKFMA2S)
KERNEL(k_pkmul2, f2, IF2, A_PKMUL2)
KERNEL(k_fmas, float, IF, A_FMAS)
KERNEL(k_fmac, float, IF, A_FMAC)
KERNEL(k_cnds, uint32_t, IU, A_CNDS)
KERNEL(k_addd, double, ID, A_ADDD)
KERNEL(k_muld, double, ID, A_MULD)
KERNEL(k_fmad, double, ID, A_FMAD)
KERNEL(k_fmacd, double, ID, A_FMACD)
KERNEL(k_cvtd, double, ID, A_CVTD)
KERNEL(k_movd, double, ID, A_MOVD)
KERNEL(k_rcpd, double, ID, A_RCPD)

template <typename T>
static double run(void (*k)(T*, uint32_t), const char* name, double ref_ms) {
    const int blocks = 256 * 8 * 4;  // 8 waves per SIMD worth of work, many rounds
    T* out;
    hipMalloc(&out, sizeof(T) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    hipFree(out);
    const double waves = blocks * 4.0, insts = waves * ITERS * 8;
    const double per_simd = insts / 1024.0;
    printf("%-12s %8.3f ms  %6.2f x v_add_u32  (%.1f Ginst/s per SIMD)\n", name, ms, ref_ms > 0 ? ms / ref_ms : 1.0,
           per_simd / (ms * 1e-3) / 1e9);
    return ms;
}

int main() {
    const double r = run(k_add, "v_add_u32", 0);
    run(k_add3, "v_add3_u32", r);
    run(k_xor3, "v_bitop3", r);
    run(k_fma, "v_fma_f32", r);
    run(k_pkfma, "v_pk_fma", r);
    run(k_pkfma_sw, "v_pk_fma_sw", r);
    run(k_mul24, "v_mul_u24", r);
    run(k_mullo, "v_mul_lo", r);
    run(k_mulhi, "v_mul_hi", r);
    run(k_mad64, "v_mad_u64", r);
    run(k_cvt, "v_cvt_f32", r);
    run(k_sin, "v_sin_f32", r);
    run(k_log, "v_log_f32", r);
    run(k_sqrt, "v_sqrt_f32", r);
    run(k_perm, "v_perm_b32", r);
    run(k_align, "v_alignbit", r);
    run(k_med3, "v_med3_i32", r);
    run(k_bcnt, "v_bcnt", r);
    run(k_addf, "v_add_f32", r);
    run(k_mulf, "v_mul_f32", r);
    run(k_fma3, "v_fma_f32(3r)", r);
    run(k_pkadd, "v_pk_add", r);
    run(k_pkmul, "v_pk_mul", r);
    run(k_xor, "v_xor_b32", r);
    run(k_lshr, "v_lshrrev", r);
    run(k_lshladd, "v_lshl_add", r);
    run(k_lshlor, "v_lshl_or", r);
    run(k_bfe, "v_bfe_u32", r);
    run(k_maxf, "v_max_f32", r);
    run(k_max3f, "v_max3_f32", r);
    run(k_cndmask, "v_cndmask", r);
    run(k_mov, "v_mov_b32", r);
    run(k_cvti, "v_cvt_i32_f32", r);
    run(k_floor, "v_floor_f32", r);
    run(k_mad24, "v_mad_u32_u24", r);
    run(k_rcp, "v_rcp_f32", r);
    run(k_andor, "v_and_or_b32", r);
    run(k_sub, "v_sub_u32", r);
    run(k_lshl64, "v_lshlrev_b64", r);
    run(k_cmp, "v_cmp+addc", r);
    run(k_pkadd2, "pk_add(2 pairs)", r);
    run(k_pkmul2, "pk_mul(2 pairs)", r);
    run(k_pkfma3, "pk_fma(3 pairs)", r);
    run(k_pkfma2s, "pk_fma(sgpr)", r);
    run(k_fmas, "fma(sgpr,2v)", r);
    run(k_fmac, "v_fmac(3v)", r);
    run(k_cnds, "cndmask(sgpr)", r);
    run(k_addd, "v_add_f64", r);
    run(k_muld, "v_mul_f64", r);
    run(k_fmad, "v_fma_f64", r);
    run(k_fmacd, "v_fmac_f64", r);
    run(k_cvtd, "v_cvt_f64_f32", r);
    run(k_movd, "v_mov_b64", r);
    run(k_rcpd, "v_rcp_f64", r);
    return 0;
}
