// ofdm_device.hpp -- device building blocks for the gfx950 OFDM modem kernels.
//
//  * cpx<R>           interleaved complex in the plan precision (float / double)
//  * dft<RAD>         radix-2/4/8/16 DFTs held entirely in registers
//  * fft_passes<>     LDS-staged mixed-radix Stockham FFT: radix-16 passes, then
//                     one radix-2/4/8 pass; each thread owns E = min(16, N)
//                     elements, a symbol is handled by TPS = N/E threads, a
//                     256-thread workgroup holds SPB = 256/TPS symbols.  LDS rows
//                     are padded by one element per 16 (pad()) so the stride-16
//                     Stockham writes of the first pass do not serialise on banks.
//  * philox4x32_10    counter-based RNG (Salmon et al., SC'11) for throughput mode
//  * slicer           per-axis nearest-point decision for the separable QAM LUTs
//                     built by QAMConstellationMapper.generate_constellation
//                     (constellation/models.py:180-218).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace ofdm {

constexpr int kBlock = 256;

template <typename R>
struct cpx {
    R re, im;
};

template <typename R>
__device__ __forceinline__ cpx<R> mk(R a, R b) {
    cpx<R> c;
    c.re = a;
    c.im = b;
    return c;
}
template <typename R>
__device__ __forceinline__ cpx<R> operator+(cpx<R> a, cpx<R> b) { return mk<R>(a.re + b.re, a.im + b.im); }
template <typename R>
__device__ __forceinline__ cpx<R> operator-(cpx<R> a, cpx<R> b) { return mk<R>(a.re - b.re, a.im - b.im); }
template <typename R>
__device__ __forceinline__ cpx<R> cmul(cpx<R> a, cpx<R> b) {
    return mk<R>(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
template <typename R>
__device__ __forceinline__ cpx<R> cscale(cpx<R> a, R s) { return mk<R>(a.re * s, a.im * s); }
template <typename R>
__device__ __forceinline__ cpx<R> conjc(cpx<R> a) { return mk<R>(a.re, -a.im); }
// multiply by -i (forward) or +i (inverse)
template <typename R, bool INV>
__device__ __forceinline__ cpx<R> rot90(cpx<R> a) {
    return INV ? mk<R>(-a.im, a.re) : mk<R>(a.im, -a.re);
}
template <typename R>
__device__ __forceinline__ R norm2(cpx<R> a) { return a.re * a.re + a.im * a.im; }
// max of two arithmetic results (the PAPR peak): v_max_* directly.  fmax() in IEEE mode quiets an
// operand the compiler cannot prove canonical first -- a second v_max_f64 x, x per element of the
// complex128 flat transmitter's peak scan.  Same result for every non-signalling input.
template <typename R>
__device__ __forceinline__ R peak_max(R a, R b) {
    R r;
    if constexpr (sizeof(R) == 8)
        asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    else
        asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// complex64 on the packed-f32 VALU: v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 do both
// components in one issue slot (the f32 vector peak of CDNA4 is only reached packed);
// swizzles and negations fold into the op_sel / neg_lo / neg_hi operand modifiers.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
template <>
struct cpx<float> {
    union {
        f32x2 v;
        struct {
            float re, im;
        };
    };
};
__device__ __forceinline__ cpx<float> pk(f32x2 v) {
    cpx<float> c;
    c.v = v;
    return c;
}
template <>
__device__ __forceinline__ cpx<float> mk<float>(float a, float b) { return pk(f32x2{a, b}); }
template <>
__device__ __forceinline__ cpx<float> operator+<float>(cpx<float> a, cpx<float> b) { return pk(a.v + b.v); }
template <>
__device__ __forceinline__ cpx<float> operator-<float>(cpx<float> a, cpx<float> b) { return pk(a.v - b.v); }
template <>
__device__ __forceinline__ cpx<float> cmul<float>(cpx<float> a, cpx<float> b) {
    // (ar br, ar bi) + (ai, ai) * (-bi, br): the swizzle and negation of b fold into
    // op_sel / neg_lo when b has one use, so pass the twiddle as a (splatted) and the data as b
    return pk(__builtin_elementwise_fma(a.v.yy, f32x2{-b.v.y, b.v.x}, a.v.xx * b.v));
}
template <>
__device__ __forceinline__ cpx<float> cscale<float>(cpx<float> a, float s) { return pk(a.v * s); }

// a * b for two run-time values: 2 packed instructions.  The compiler materialises the
// swizzled, negated b with a v_xor + v_mov pair whenever b has another use, so the fma
// is spelt out: lo = a.y * -b.y + t.x, hi = a.y * b.x + t.y.
template <typename R>
__device__ __forceinline__ cpx<R> cmulv(cpx<R> a, cpx<R> b) {
    if constexpr (sizeof(R) == 4) {
        const f32x2 t = a.v.xx * b.v;
        f32x2 r;
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
            : "=v"(r)
            : "v"(a.v), "v"(b.v), "v"(t));
        return pk(r);
    } else {
        return cmul(a, b);
    }
}

// ------------------------------------------------------------------ small DFTs
template <typename R, bool INV>
__device__ __forceinline__ void dft2(cpx<R>& a, cpx<R>& b) {
    cpx<R> t = a - b;
    a = a + b;
    b = t;
}

// a + rot90(d) (SGN = +1) or a - rot90(d) (SGN = -1).  complex64: one v_pk_fma_f32 on
// the swizzled operand, so the rotation is never materialised.
template <typename R, bool INV, int SGN>
__device__ __forceinline__ cpx<R> add_rot(cpx<R> a, cpx<R> d) {
    if constexpr (sizeof(R) == 4) {
        constexpr float s = (INV ? -1.f : 1.f) * SGN;
        return pk(__builtin_elementwise_fma(d.v.yx, f32x2{s, -s}, a.v));
    } else {
        const cpx<R> r = rot90<R, INV>(d);
        return SGN > 0 ? a + r : a - r;
    }
}

// ROT2: v2 enters multiplied by -i (forward) / +i (inverse)
template <typename R, bool INV, bool ROT2 = false>
__device__ __forceinline__ void dft4(cpx<R>& v0, cpx<R>& v1, cpx<R>& v2, cpx<R>& v3) {
    cpx<R> t0, t1;
    if constexpr (ROT2) {
        t0 = add_rot<R, INV, 1>(v0, v2);
        t1 = add_rot<R, INV, -1>(v0, v2);
    } else {
        t0 = v0 + v2;
        t1 = v0 - v2;
    }
    const cpx<R> t2 = v1 + v3, d = v1 - v3;
    v0 = t0 + t2;
    v2 = t0 - t2;
    v1 = add_rot<R, INV, 1>(t1, d);
    v3 = add_rot<R, INV, -1>(t1, d);
}

// W_n^k = exp(-+2 pi i k / n), compile-time constants for n = 8, 16
template <typename R, bool INV>
__device__ __forceinline__ cpx<R> w16(int k) {
    // cos/sin(2*pi*k/16), k in [0, 9]
    constexpr double c[10] = {1.0,
                              0.92387953251128673848,
                              0.70710678118654752440,
                              0.38268343236508977173,
                              0.0,
                              -0.38268343236508977173,
                              -0.70710678118654752440,
                              -0.92387953251128673848,
                              -1.0,
                              -0.92387953251128673848};
    constexpr double s[10] = {0.0,
                              0.38268343236508977173,
                              0.70710678118654752440,
                              0.92387953251128673848,
                              1.0,
                              0.92387953251128673848,
                              0.70710678118654752440,
                              0.38268343236508977173,
                              0.0,
                              -0.38268343236508977173};
    return mk<R>((R)c[k], INV ? (R)s[k] : (R)-s[k]);
}

template <typename R, int RAD, bool INV>
__device__ __forceinline__ void dft(cpx<R>* v) {
    if constexpr (RAD == 1) {
    } else if constexpr (RAD == 2) {
        dft2<R, INV>(v[0], v[1]);
    } else if constexpr (RAD == 4) {
        dft4<R, INV>(v[0], v[1], v[2], v[3]);
    } else if constexpr (RAD == 8) {
        // n = 2 n1 + n2, k = k1 + 4 k2
        cpx<R> a[2][4];
#pragma unroll
        for (int n2 = 0; n2 < 2; ++n2) {
            a[n2][0] = v[n2];
            a[n2][1] = v[n2 + 2];
            a[n2][2] = v[n2 + 4];
            a[n2][3] = v[n2 + 6];
            dft4<R, INV>(a[n2][0], a[n2][1], a[n2][2], a[n2][3]);
        }
        a[1][1] = cmul(a[1][1], w16<R, INV>(2));
        a[1][3] = cmul(a[1][3], w16<R, INV>(6));
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            cpx<R> p = a[0][k1], q = a[1][k1];
            if (k1 == 2) {  // q * W8^2 = rot90(q)
                v[k1] = add_rot<R, INV, 1>(p, q);
                v[k1 + 4] = add_rot<R, INV, -1>(p, q);
            } else {
                v[k1] = p + q;
                v[k1 + 4] = p - q;
            }
        }
    } else if constexpr (RAD == 16) {
        // n = 4 n1 + n2, k = k1 + 4 k2
        cpx<R> a[4][4];
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) {
            a[n2][0] = v[n2];
            a[n2][1] = v[n2 + 4];
            a[n2][2] = v[n2 + 8];
            a[n2][3] = v[n2 + 12];
            dft4<R, INV>(a[n2][0], a[n2][1], a[n2][2], a[n2][3]);
        }
#pragma unroll
        for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
            for (int k1 = 1; k1 < 4; ++k1) {
                const int e = n2 * k1;
                if (e != 4) a[n2][k1] = cmul(a[n2][k1], w16<R, INV>(e));  // e = 4: ROT2 below
            }
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            cpx<R> b0 = a[0][k1], b1 = a[1][k1], b2 = a[2][k1], b3 = a[3][k1];
            if (k1 == 2)
                dft4<R, INV, true>(b0, b1, b2, b3);
            else
                dft4<R, INV>(b0, b1, b2, b3);
            v[k1] = b0;
            v[k1 + 4] = b1;
            v[k1 + 8] = b2;
            v[k1 + 12] = b3;
        }
    }
}

template <int I, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, E>(f);
    }
}

// ------------------------------------------------------------------ FFT geometry
template <int LOGN, int BLK = kBlock>
struct Geo {
    static constexpr int N = 1 << LOGN;
    static constexpr int LOGE = LOGN < 4 ? LOGN : 4;
    static constexpr int E = 1 << LOGE;   // elements per thread
    static constexpr int TPS = N / E;     // threads per symbol
    static constexpr int SPB = BLK / TPS;  // symbols per workgroup
    static constexpr int PADN = N + (N >> 4);  // padded LDS row (complex elements); with pad()
                                                // conflict-free row spacing (tools/lds_banks.py)
};

__device__ __forceinline__ int pad(int i) { return i + (i >> 4); }
// pad(b + c) for a constant c that is a multiple of 16: pad(b) + pad(c), so every such
// access is one base register plus an instruction offset (written as pad(b + c), the
// compiler materialises and keeps a separate address register per constant)
template <int C>
__device__ __forceinline__ int pad_plus(int padded_b) {
    static_assert(C % 16 == 0, "pad(b + c) = pad(b) + pad(c) needs c = 0 mod 16");
    return padded_b + C + (C >> 4);
}

// Per-pass twiddle tables (throughput kernels).  Pass (LOGR, LOGNS > 0) multiplies input r
// of butterfly k = j mod NS by W^(k r), W = exp(-+2 pi i / (NS RAD)); the tables hold
// T[(r - 1) NS + k] for 0 < r < RAD, k < NS, pass after pass, computed on the host in
// double.  One LDS read per twiddle instead of the two-level lookup and the recurrence.
// Compact passes (NS >= 256 at N >= 2^OFDM_TT_COMPACT_MIN_LOGN: the last pass of N = 2048 / 4096)
// hold only W^k for k < NS: the butterfly reads w = W^k and forms W^(k r) by recurrence (RAD - 2
// complex products; <= 14 roundings, ~1e-6 in f32).  The full tables of those passes are 7/8 of
// the total (28.7 of 32.6 KB at N = 4096 in complex64), which would otherwise cap a CU at two
// workgroups.
#ifndef OFDM_TT_COMPACT_MIN_LOGN
#define OFDM_TT_COMPACT_MIN_LOGN 11
#endif
constexpr bool tt_compact(int logn, int logns) { return logn >= OFDM_TT_COMPACT_MIN_LOGN && logns >= 8; }
constexpr int tt_from(int logn, int logns) {
    if (logns >= logn) return 0;
    const int logr = logn - logns >= 4 ? 4 : logn - logns;
    const int here = logns > 0 ? (tt_compact(logn, logns) ? 1 : (1 << logr) - 1) << logns : 0;
    return here + tt_from(logn, logns + logr);
}
constexpr int tt_size(int logn) { return logn <= 4 ? 0 : tt_from(logn, 0); }

// Twiddle W_N^m = exp(-2 pi i m / N) (conjugated for the inverse) from a two-level
// table held in LDS: lo[m & 63] * hi[m >> 6].  Both tables are computed on the host
// in double precision.
template <typename R, int LOGN, bool INV>
__device__ __forceinline__ cpx<R> twiddle(int m, const cpx<R>* lo, const cpx<R>* hi) {
    cpx<R> w;
    if constexpr (LOGN <= 6) {
        w = lo[m];
    } else {
        w = cmul(lo[m & 63], hi[m >> 6]);
    }
    return INV ? conjc(w) : w;
}

// Barrier between FFT passes.  A symbol's TPS threads sit inside one wavefront when
// TPS <= 64, but every kernel runs whole-workgroup loops, so a workgroup barrier is
// always correct; it is cheap at 4 waves per workgroup.
__device__ __forceinline__ void group_sync() { __syncthreads(); }

template <typename R, int LOGN, int LOGR, int LOGNS, bool INV>
__device__ __forceinline__ void stockham_pass(cpx<R>* buf, const cpx<R>* lo, const cpx<R>* hi,
                                              int t) {
    using G = Geo<LOGN>;
    constexpr int RAD = 1 << LOGR;
    constexpr int NS = 1 << LOGNS;
    constexpr int NB = G::E / RAD;  // butterflies per thread
    constexpr int STRIDE = G::N / RAD;
    cpx<R> v[NB][RAD];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int j = t + q * G::TPS;
#pragma unroll
        for (int r = 0; r < RAD; ++r) v[q][r] = buf[pad(j + r * STRIDE)];
    }
    group_sync();
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int j = t + q * G::TPS;
        const int k = j & (NS - 1);
        if constexpr (LOGNS > 0) {
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                const int m = (r * k) << (LOGN - LOGNS - LOGR);
                v[q][r] = cmul(v[q][r], twiddle<R, LOGN, INV>(m, lo, hi));
            }
        }
        dft<R, RAD, INV>(v[q]);
        const int idx = ((j >> LOGNS) << (LOGNS + LOGR)) + k;
#pragma unroll
        for (int r = 0; r < RAD; ++r) buf[pad(idx + r * NS)] = v[q][r];
    }
    group_sync();
}

// Full FFT of one symbol resident (padded, natural order) in buf; result in natural
// order in buf.  Unnormalised (callers fold the ortho 1/sqrt(N) into a load or store).
// Requires a group_sync() between the writes that filled buf and this call.
template <typename R, int LOGN, int LOGNS, bool INV>
__device__ __forceinline__ void fft_passes(cpx<R>* buf, const cpx<R>* lo, const cpx<R>* hi, int t) {
    if constexpr (LOGNS < LOGN) {
        constexpr int REM = LOGN - LOGNS;
        constexpr int LOGR = REM >= 4 ? 4 : REM;
        stockham_pass<R, LOGN, LOGR, LOGNS, INV>(buf, lo, hi, t);
        fft_passes<R, LOGN, LOGNS + LOGR, INV>(buf, lo, hi, t);
    }
}

// Load the 2 x 64-entry twiddle table into LDS (caller syncs).
template <typename R>
__device__ __forceinline__ void load_twiddles(cpx<R>* lds, const cpx<R>* g) {
    if (threadIdx.x < 128) lds[threadIdx.x] = g[threadIdx.x];
}

// Per-LUT decision info for the separable square-QAM LUTs: LUT[i] = lev[ki] + j lev[kq]
// with i = (qpat[kq] << hbits) | ipat[ki]; levels sorted ascending, uniform step.
struct AxisInfo {
    double lev0;      // most negative level
    double inv_step;  // 1 / level spacing
    int32_t side;     // sqrt(M)
    int32_t hbits;    // b / 2
    int32_t lut_off;  // offset of this LUT in the pool
    int32_t bits;     // b
    uint8_t ipat[16];
    uint8_t qpat[16];
};

// Per-subcarrier table for adaptive bit loading.
struct ScInfo {
    int16_t lut;     // AxisInfo index, -1 = inactive
    int16_t bits;    // b_k
    int32_t bitoff;  // bit offset of subcarrier k inside one OFDM symbol's bit stream
};

// ------------------------------------------------------------------ register-resident FFT
// Synchronisation of one symbol group.  When a symbol's TPS threads sit in one
// wavefront (TPS <= 64) and every LDS region they touch is private to that symbol,
// a wavefront-scope fence is enough: a wave's LDS operations execute in program
// order, the fence only stops the compiler from moving them.  Larger groups span
// waves and need the workgroup barrier (then every thread of the block calls it).
template <int TPS>
__device__ __forceinline__ void sym_sync() {
    if constexpr (TPS <= 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        // LDS writes issued as inline assembly (OFDM_SPLIT_WRITE_B64) are not
        // tracked by the compiler's wait-count pass, which drops the barrier's lgkmcnt(0) when it
        // sees no LDS operation of its own in flight: wait here, so the other waves read them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// OFDM_SPLIT_READ_B64: the split exchange's reads as single ds_read_b64 (inline assembly) instead of
// the compiler's ds_read2_b64 pairs
#ifndef OFDM_SPLIT_READ_B64
#define OFDM_SPLIT_READ_B64 1
#endif
// OFDM_SPLIT_WRITE_B64: the exchange's writes as single ds_write_b64 (inline assembly) instead of the
// compiler's ds_write2_b64 pairs (c 1.196 -> 1.218e8, d 5.43 -> 5.51e7 symbols/s,
// profiles/r04l_ab_orderparams_writeb64.txt)
#ifndef OFDM_SPLIT_WRITE_B64
#define OFDM_SPLIT_WRITE_B64 1
#endif
#ifndef OFDM_SPLIT_XL
#define OFDM_SPLIT_XL 1
#endif
// OFDM_SPLIT_PERMLANE: the second exchange of the N = 1024 complex128 FFT in registers
// (v_permlane32_swap / v_permlane16_swap, reg_pass_split) instead of through the LDS row
#ifndef OFDM_SPLIT_PERMLANE
#define OFDM_SPLIT_PERMLANE 1
#endif
// 32-bit LDS address of a pointer into __shared__ memory
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(const T* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) T*)p;
}
template <int OFF>
__device__ __forceinline__ void ds_write_b64_at(uint32_t la, double d) {
    asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(la), "v"(d), "i"(OFF) : "memory");
}
// 16 ds_read_b64 at LDS byte addresses la + O_m and their s_waitcnt lgkmcnt(0) as ONE inline-assembly
// statement: the compiler's wait-count pass does not track inline-assembly LDS loads, so with the
// reads and the wait in separate statements nothing would stop it from copying (or spilling) a
// destination register between a read and the wait -- a stale value without any error.  Inside
// one statement no instruction can be placed between them; the destinations are early-clobber, so
// none of them shares a register with the address.
template <int... O>
__device__ __forceinline__ void ds_read16_b64(double (&u)[16], uint32_t la) {
    static_assert(sizeof...(O) == 16, "16 offsets");
    constexpr int o[16] = {O...};
    asm volatile(
        "ds_read_b64 %0, %16 offset:%17\n\tds_read_b64 %1, %16 offset:%18\n\t"
        "ds_read_b64 %2, %16 offset:%19\n\tds_read_b64 %3, %16 offset:%20\n\t"
        "ds_read_b64 %4, %16 offset:%21\n\tds_read_b64 %5, %16 offset:%22\n\t"
        "ds_read_b64 %6, %16 offset:%23\n\tds_read_b64 %7, %16 offset:%24\n\t"
        "ds_read_b64 %8, %16 offset:%25\n\tds_read_b64 %9, %16 offset:%26\n\t"
        "ds_read_b64 %10, %16 offset:%27\n\tds_read_b64 %11, %16 offset:%28\n\t"
        "ds_read_b64 %12, %16 offset:%29\n\tds_read_b64 %13, %16 offset:%30\n\t"
        "ds_read_b64 %14, %16 offset:%31\n\tds_read_b64 %15, %16 offset:%32\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(u[0]), "=&v"(u[1]), "=&v"(u[2]), "=&v"(u[3]), "=&v"(u[4]), "=&v"(u[5]), "=&v"(u[6]), "=&v"(u[7]),
          "=&v"(u[8]), "=&v"(u[9]), "=&v"(u[10]), "=&v"(u[11]), "=&v"(u[12]), "=&v"(u[13]), "=&v"(u[14]),
          "=&v"(u[15])
        : "v"(la), "i"(o[0]), "i"(o[1]), "i"(o[2]), "i"(o[3]), "i"(o[4]), "i"(o[5]), "i"(o[6]), "i"(o[7]),
          "i"(o[8]), "i"(o[9]), "i"(o[10]), "i"(o[11]), "i"(o[12]), "i"(o[13]), "i"(o[14]), "i"(o[15])
        : "memory");
}
// the same with byte offsets Off::at(m), m = 0..15 (Off: a class with a static constexpr at(int))
template <class Off, int... M>
__device__ __forceinline__ void ds_read16_b64_seq(double (&u)[16], uint32_t la, std::integer_sequence<int, M...>) {
    ds_read16_b64<Off::at(M)...>(u, la);
}
template <class Off>
__device__ __forceinline__ void ds_read16_b64(double (&u)[16], uint32_t la) {
    ds_read16_b64_seq<Off>(u, la, std::make_integer_sequence<int, 16>{});
}

// One Stockham pass with the data distribution "thread t owns elements t + i*TPS".
// FIRST: inputs come from x[] (valid because the first pass has RAD = E, STRIDE = TPS);
// LAST: outputs stay in x[] (the last pass writes j + r*NS with j = t + q*TPS and
// NS = TPS*E/RAD, i.e. element t + (q + r*NB)*TPS); otherwise through the LDS row.
template <typename R, int LOGN, int LOGR, int LOGNS, bool INV, bool FIRST, bool LAST, bool TT>
__device__ __forceinline__ void reg_pass(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                         const cpx<R>* hi, const cpx<R>* tt, int t) {
    using G = Geo<LOGN>;
    constexpr int RAD = 1 << LOGR;
    constexpr int NS = 1 << LOGNS;
    constexpr int NB = G::E / RAD;
    constexpr int STRIDE = G::N / RAD;
    cpx<R> v[NB][RAD];
    // complex64 rows at N = 1024..4096 (8-byte elements): the exchanges as single ds_read_b64 /
    // ds_write_b64 in the conflict-free layouts of the split complex128 exchange (reg_pass_split):
    // after pass 1 element e = 16 t + r at (TPS + 2) r + t, after pass 2 at e
    constexpr bool XLC = sizeof(cpx<R>) == 8 && OFDM_SPLIT_XL && OFDM_SPLIT_READ_B64 && OFDM_SPLIT_WRITE_B64 &&
                         LOGN >= 10 && LOGN <= 12 && G::E == 16 && (LOGNS == 0 || LOGNS == 4 || LOGNS == 8);
    if constexpr (FIRST) {
        static_assert(NB == 1 && STRIDE == G::TPS, "first pass consumes the register layout");
#pragma unroll
        for (int r = 0; r < RAD; ++r) v[0][r] = x[r];
    } else if constexpr (XLC) {
        static_assert(NB * RAD == 16, "one read per element");
        const uint32_t la = lds_addr(buf + (LOGNS == 4 ? (G::TPS + 2) * (t & 15) + (t >> 4) : t));
        double u[16];
        struct Off {  // element u[Q RAD + Rr]
            static constexpr int at(int m) {
                return 8 * (LOGNS == 4 ? (G::TPS / 16) * (m % RAD) : (m / RAD) * G::TPS + (m % RAD) * STRIDE);
            }
        };
        ds_read16_b64<Off>(u, la);
#pragma unroll
        for (int q = 0; q < NB; ++q)
#pragma unroll
            for (int r = 0; r < RAD; ++r) v[q][r] = __builtin_bit_cast(cpx<R>, u[q * RAD + r]);
        if constexpr (!LAST) sym_sync<G::TPS>();  // every read done before the rewrite
    } else if constexpr (G::TPS % 16 == 0 && STRIDE % 16 == 0) {
        const int pt = pad(t);  // every read is pad(t) + a constant
        static_for<0, NB>([&](auto Q) {
            static_for<0, RAD>([&](auto Rr) {
                v[Q][Rr] = buf[pad_plus<Q * G::TPS + Rr * STRIDE>(pt)];
            });
        });
        if constexpr (!LAST) sym_sync<G::TPS>();  // every read done before the rewrite
    } else {
#pragma unroll
        for (int q = 0; q < NB; ++q)
#pragma unroll
            for (int r = 0; r < RAD; ++r) v[q][r] = buf[pad(t + q * G::TPS + r * STRIDE)];
        if constexpr (!LAST) sym_sync<G::TPS>();  // every read done before the rewrite
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int j = t + q * G::TPS;
        const int k = j & (NS - 1);
        if constexpr (LOGNS > 0 && TT && tt_compact(LOGN, LOGNS)) {
            const cpx<R> w1 = tt[(tt_size(LOGN) - tt_from(LOGN, LOGNS)) + k];
            cpx<R> wr = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmulv(wr, v[q][r]);
                if (r + 1 < RAD) wr = cmulv(wr, w1);
            }
        } else if constexpr (LOGNS > 0 && TT) {
            const cpx<R>* T = tt + (tt_size(LOGN) - tt_from(LOGN, LOGNS)) + k;
#pragma unroll
            for (int r = 1; r < RAD; ++r) v[q][r] = cmulv(T[(r - 1) * NS], v[q][r]);
        } else if constexpr (LOGNS > 0) {
            // w^r by recurrence from one table lookup: 2 live registers instead of the
            // RAD-1 hoisted table loads (<= 15 roundings: ~1e-6 in f32, ~2e-15 in f64)
            const cpx<R> w1 = twiddle<R, LOGN, INV>(k << (LOGN - LOGNS - LOGR), lo, hi);
            cpx<R> wr = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmulv(wr, v[q][r]);
                if (r + 1 < RAD) wr = cmulv(wr, w1);
            }
        }
        dft<R, RAD, INV>(v[q]);
        if constexpr (LAST) {
#pragma unroll
            for (int r = 0; r < RAD; ++r) x[q + r * NB] = v[q][r];
        } else if constexpr (XLC) {
            // the per-radix offset 16 Rr below assumes NS = 16 whenever LOGNS != 0
            static_assert(LOGNS == 0 || (LOGNS == 4 && RAD == 16 && NB == 1), "XLC write layout");
            const int idx = ((j >> LOGNS) << (LOGNS + LOGR)) + k;
            const uint32_t la = lds_addr(buf + (LOGNS == 0 ? j : idx));
            static_for<0, RAD>([&](auto Rr) {
                constexpr int off = 8 * (LOGNS == 0 ? (G::TPS + 2) * Rr : 16 * Rr);
                ds_write_b64_at<off>(la, __builtin_bit_cast(double, v[q][Rr]));
            });
        } else if constexpr (NS % 16 == 0) {
            const int pi = pad(((j >> LOGNS) << (LOGNS + LOGR)) + k);
            static_for<0, RAD>([&](auto Rr) { buf[pad_plus<Rr * NS>(pi)] = v[q][Rr]; });
        } else {
            const int idx = ((j >> LOGNS) << (LOGNS + LOGR)) + k;
#pragma unroll
            for (int r = 0; r < RAD; ++r) buf[pad(idx + r * NS)] = v[q][r];
        }
    }
    if constexpr (!LAST) sym_sync<G::TPS>();
}

// complex128 throughput kernels: the transposes between passes go through a row of N doubles,
// real parts first, then imaginary parts -- half the LDS of a complex row per symbol, so twice
// as many symbols (waves) fit a CU at the register budget complex128 needs.  Every pass takes
// its inputs from x[] ("thread t owns elements t + i*TPS": element t + (q + r NB) TPS is input r
// of butterfly q, which holds for every radix) and, unless LAST, leaves the next pass's inputs
// there: its outputs go to the row at their Stockham positions, one component at a time, and
// elements t + m*TPS come back.  With TPS <= 64 the exchange is wave-local (sym_sync = fences: a
// wave's LDS operations execute in program order).
template <typename R, int LOGN, int LOGR, int LOGNS, bool INV, bool LAST, bool TT>
__device__ __forceinline__ void reg_pass_split(cpx<R> (&x)[Geo<LOGN>::E], R* rb, const cpx<R>* lo,
                                               const cpx<R>* hi, const cpx<R>* tt, int t) {
    using G = Geo<LOGN>;
    constexpr int RAD = 1 << LOGR;
    constexpr int NS = 1 << LOGNS;
    constexpr int NB = G::E / RAD;
    cpx<R> v[NB][RAD];
#pragma unroll
    for (int q = 0; q < NB; ++q)
#pragma unroll
        for (int r = 0; r < RAD; ++r) v[q][r] = x[q + r * NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const int j = t + q * G::TPS;
        const int k = j & (NS - 1);
        if constexpr (LOGNS > 0 && TT && tt_compact(LOGN, LOGNS)) {
            const cpx<R> w1 = tt[(tt_size(LOGN) - tt_from(LOGN, LOGNS)) + k];
            cpx<R> wr = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmul(wr, v[q][r]);
                if (r + 1 < RAD) wr = cmul(wr, w1);
            }
        } else if constexpr (LOGNS > 0 && TT) {
            const cpx<R>* T = tt + (tt_size(LOGN) - tt_from(LOGN, LOGNS)) + k;
#pragma unroll
            for (int r = 1; r < RAD; ++r) v[q][r] = cmul(T[(r - 1) * NS], v[q][r]);
        } else if constexpr (LOGNS > 0) {
            const cpx<R> w1 = twiddle<R, LOGN, INV>(k << (LOGN - LOGNS - LOGR), lo, hi);
            cpx<R> wr = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmul(wr, v[q][r]);
                if (r + 1 < RAD) wr = cmul(wr, w1);
            }
        }
        dft<R, RAD, INV>(v[q]);
    }
    // N = 1024 (a symbol per wave), the exchange after the second radix-16 pass: in registers with
    // the gfx950 cross-row swaps instead of through the LDS row.  Pass 2 leaves output r = 4 rh + rl
    // of lane t at Stockham position 256 (t >> 4) + (t & 15) + 16 r; the last pass (radix 4) reads
    // element t' + 64 m into x[m].  So the value moves to lane (t & 15) + 16 rl, register
    // 4 (t >> 4) + rh: for each rh, a 4 x 4 transpose of (16-lane row t >> 4, rl), which
    // v_permlane32_swap (rows {2,3} of one register <-> rows {0,1} of another) and
    // v_permlane16_swap (odd rows <-> even rows) do in four swaps per 4 dwords -- 64 VALU swaps
    // per symbol instead of 32 ds_write_b64 + 32 ds_read_b64 and their waits.
    constexpr bool XPERM = OFDM_SPLIT_PERMLANE && sizeof(R) == 8 && G::TPS == 64 && G::E == 16 && LOGN == 10 &&
                           LOGNS == 4 && RAD == 16 && NB == 1 && !LAST;
    if constexpr (LAST) {
#pragma unroll
        for (int q = 0; q < NB; ++q)
#pragma unroll
            for (int r = 0; r < RAD; ++r) x[q + r * NB] = v[q][r];
    } else if constexpr (XPERM) {
        typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
        static_for<0, 4>([&](auto RH) {
            u32x4v d[4];
#pragma unroll
            for (int rl = 0; rl < 4; ++rl) d[rl] = __builtin_bit_cast(u32x4v, v[0][4 * RH + rl]);
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                auto s02 = __builtin_amdgcn_permlane32_swap(d[0][w], d[2][w], false, false);
                auto s13 = __builtin_amdgcn_permlane32_swap(d[1][w], d[3][w], false, false);
                auto s01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
                auto s23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
                d[0][w] = s01[0];
                d[1][w] = s01[1];
                d[2][w] = s23[0];
                d[3][w] = s23[1];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) x[4 * k + RH] = __builtin_bit_cast(cpx<R>, d[k]);
        });
    } else {
        // Exchange layouts of the radix-16 passes at TPS >= 64 (N >= 1024), for the single 8-byte
        // accesses (ds_write_b64: 16-lane groups over 32 banks; ds_read_b64: 32-lane groups over
        // 64): after pass 1, element e = 16 t + r at (TPS + 2) r + t; after pass 2, at e itself.
        // Both are conflict-free for the writes (lane t, fixed r) and the reads (e = t + TPS m);
        // pad() costs the reads one conflict per 32 lanes (128 cycles per N = 1024 symbol,
        // SQ_LDS_BANK_CONFLICT 133 per symbol, profiles/r04n_counters_stall_c_f64.txt).  Rows fit: 16 TPS + 30 < PADN.
        constexpr bool XL = sizeof(R) == 8 && OFDM_SPLIT_XL && OFDM_SPLIT_READ_B64 && OFDM_SPLIT_WRITE_B64 && G::TPS >= 64 &&
                            RAD == 16 && NB == 1 && (LOGNS == 0 || LOGNS == 4);
        auto put = [&](bool im) {
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int j = t + q * G::TPS;
                const int idx = ((j >> LOGNS) << (LOGNS + LOGR)) + (j & (NS - 1));
                if constexpr (XL) {
                    const uint32_t la = lds_addr(rb + (LOGNS == 0 ? t : idx));
                    static_for<0, RAD>([&](auto Rr) {
                        constexpr int off = 8 * (LOGNS == 0 ? (G::TPS + 2) * Rr : 16 * Rr);
                        ds_write_b64_at<off>(la, im ? v[q][Rr].im : v[q][Rr].re);
                    });
                } else if constexpr (sizeof(R) == 8 && OFDM_SPLIT_WRITE_B64 && (NS % 16 == 0 || NS == 1)) {
                    // one ds_write_b64 per element (the compiler's ds_write2_b64 pairs cost 13 LDS
                    // cycles per KB against 12 for two single writes); NS = 1: idx = 0 mod 16, so
                    // pad(idx + r) = pad(idx) + r
                    const uint32_t la = lds_addr(rb + pad(idx));
                    static_for<0, RAD>([&](auto Rr) {
                        constexpr int C = Rr * NS;
                        constexpr int off = 8 * (NS == 1 ? C : C + (C >> 4));
                        ds_write_b64_at<off>(la, im ? v[q][Rr].im : v[q][Rr].re);
                    });
                } else if constexpr (NS % 16 == 0) {
                    const int pi = pad(idx);
                    static_for<0, RAD>([&](auto Rr) { rb[pad_plus<Rr * NS>(pi)] = im ? v[q][Rr].im : v[q][Rr].re; });
                } else {
#pragma unroll
                    for (int r = 0; r < RAD; ++r) rb[pad(idx + r * NS)] = im ? v[q][r].im : v[q][r].re;
                }
            }
        };
        auto get = [&](bool im) {
            if constexpr (G::TPS % 16 == 0 && sizeof(R) == 8 && OFDM_SPLIT_READ_B64) {
                // one ds_read_b64 per element: the compiler pairs the reads into ds_read2_b64,
                // which the LDS serves at half the rate (8 cycles per KB against 4 for two
                // ds_read_b64, MI355X_MICROARCH.md LDS table).  Issued with their lgkmcnt(0) as one
                // inline-assembly statement (ds_read16_b64).
                const uint32_t la =
                    lds_addr(rb + (!XL ? pad(t) : LOGNS == 0 ? (G::TPS + 2) * (t & 15) + (t >> 4) : t));
                static_assert(G::E == 16, "16 elements per lane");
                R u[G::E];
                struct Off {
                    static constexpr int at(int m) {
                        return 8 * (!XL ? m * G::TPS + ((m * G::TPS) >> 4)  // pad_plus<C>(0), C = 0 mod 16
                                        : LOGNS == 0 ? m * G::TPS / 16 : m * G::TPS);
                    }
                };
                ds_read16_b64<Off>(u, la);
                static_for<0, G::E>([&](auto M) {
                    if (im) x[M].im = u[M]; else x[M].re = u[M];
                });
            } else if constexpr (G::TPS % 16 == 0) {
                const int pt = pad(t);
                static_for<0, G::E>([&](auto M) {
                    const R u = rb[pad_plus<M * G::TPS>(pt)];
                    if (im) x[M].im = u; else x[M].re = u;
                });
            } else {
#pragma unroll
                for (int m = 0; m < G::E; ++m) {
                    const R u = rb[pad(t + m * G::TPS)];
                    if (im) x[m].im = u; else x[m].re = u;
                }
            }
        };
        put(false);
        sym_sync<G::TPS>();
        get(false);
        sym_sync<G::TPS>();
        put(true);
        sym_sync<G::TPS>();
        get(true);
        sym_sync<G::TPS>();  // every read done before the next pass rewrites the row
    }
}

template <typename R, int LOGN, int LOGNS, bool INV, bool TT>
__device__ __forceinline__ void reg_passes_split(cpx<R> (&x)[Geo<LOGN>::E], R* rb, const cpx<R>* lo,
                                                 const cpx<R>* hi, const cpx<R>* tt, int t) {
    if constexpr (LOGNS < LOGN) {
        constexpr int REM = LOGN - LOGNS;
        constexpr int LOGR = REM >= 4 ? 4 : REM;
        reg_pass_split<R, LOGN, LOGR, LOGNS, INV, LOGNS + LOGR == LOGN, TT>(x, rb, lo, hi, tt, t);
        reg_passes_split<R, LOGN, LOGNS + LOGR, INV, TT>(x, rb, lo, hi, tt, t);
    }
}

template <typename R, int LOGN, int LOGNS, bool INV, bool TT>
__device__ __forceinline__ void reg_passes(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                           const cpx<R>* hi, const cpx<R>* tt, int t) {
    if constexpr (LOGNS < LOGN) {
        constexpr int REM = LOGN - LOGNS;
        constexpr int LOGR = REM >= 4 ? 4 : REM;
        reg_pass<R, LOGN, LOGR, LOGNS, INV, LOGNS == 0, LOGNS + LOGR == LOGN, TT>(x, buf, lo, hi, tt, t);
        reg_passes<R, LOGN, LOGNS + LOGR, INV, TT>(x, buf, lo, hi, tt, t);
    }
}

// FFT of one symbol: on entry and exit thread t (of TPS) holds element t + i*TPS in
// x[i].  Unnormalised.  buf is the symbol's private padded LDS row; the caller must
// sym_sync() between an earlier use of buf and this call when TPS > 64.  Twiddles from the
// two-level table lo/hi (recurrence) or, TT, from the per-pass tables tt in LDS.
template <typename R, int LOGN, bool INV, bool TT = false>
__device__ __forceinline__ void fft_reg(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                        const cpx<R>* hi, int t, const cpx<R>* tt = nullptr) {
    if constexpr (LOGN <= 4) {
        dft<R, (1 << LOGN), INV>(x);  // one register-resident pass (TPS = 1)
    } else {
        reg_passes<R, LOGN, 0, INV, TT>(x, buf, lo, hi, tt, t);
    }
}

// The same FFT with the split (real / imaginary) exchange; rb: the symbol's row of PADN reals.
template <typename R, int LOGN, bool INV, bool TT>
__device__ __forceinline__ void fft_reg_split(cpx<R> (&x)[Geo<LOGN>::E], R* rb, const cpx<R>* lo,
                                              const cpx<R>* hi, int t, const cpx<R>* tt) {
    if constexpr (LOGN <= 4) {
        dft<R, (1 << LOGN), INV>(x);
    } else {
        reg_passes_split<R, LOGN, 0, INV, TT>(x, rb, lo, hi, tt, t);
    }
}

// Twiddle source of the throughput kernels: per-pass LDS tables (complex64 always; complex128
// while the table fits beside the rows, <= 16 KB: every N with the compact last passes) or the
// two-level table plus recurrence.
template <typename R, int LOGN>
constexpr bool fast_tt() { return sizeof(R) == 4 || tt_size(LOGN) * 2 * (int)sizeof(R) <= 16384; }

// b (<= 8) bits at bit offset o of a stream stored as 32-bit words, stream bit 32w+j
// = bit (31-j) of word w; one word of slack after the stream.
__device__ __forceinline__ uint32_t extract_w(const uint32_t* w, int o, int b) {
    const int q = o >> 5, s = o & 31;
    const uint64_t x = ((uint64_t)w[q] << 32) | (uint64_t)w[q + 1];
    return (uint32_t)(x >> (64 - s - b)) & ((1u << b) - 1u);
}

// Per-axis decision held in registers: ipat / qpat as 4-bit nibbles of a 64-bit word.
template <typename R>
struct Slicer {
    R lev0, inv_step;
    int smax, hbits;
    uint64_t ipat, qpat;
    __device__ void load(const AxisInfo& a) {
        lev0 = (R)a.lev0;
        inv_step = (R)a.inv_step;
        smax = a.side - 1;
        hbits = a.hbits;
        ipat = qpat = 0;
        for (int k = 0; k < a.side; ++k) {
            ipat |= (uint64_t)a.ipat[k] << (4 * k);
            qpat |= (uint64_t)a.qpat[k] << (4 * k);
        }
    }
    __device__ __forceinline__ int level(R u) const {
        int k = (int)floor((u - lev0) * inv_step + (R)0.5);
        return min(max(k, 0), smax);
    }
    __device__ __forceinline__ uint32_t operator()(cpx<R> z) const {
        const uint32_t i = (uint32_t)(ipat >> (4 * level(z.re))) & 15u;
        const uint32_t q = (uint32_t)(qpat >> (4 * level(z.im))) & 15u;
        return (q << hbits) | i;
    }
};

// Throughput-mode slicer (complex64, square QAM with b = FB <= 8 bits).  Both axes per
// packed op: y = z * inv_step - lev0 * inv_step is the level coordinate (offset (side-1)/2,
// a half-integer).  One v_pk_fma_f32 computes y / (side-1) of both axes with the instruction's
// clamp bit, i.e. clamped to [0, 1] (every point beyond the outer levels decides the outer
// level), and a second one v * (side-1) + 1.5*2^23 leaves round(y) in the low mantissa bits
// (round-to-nearest-even; a tie is a decision boundary, probability zero under noise) -- two
// packed ops per element, where clamping y + 1.5*2^23 on the raw bits took four.  The levels
// of four elements are gathered into one selector word (byte j = element j) and looked up
// with v_perm_b32 in byte tables: four rx indices per instruction, byte-aligned like the
// lane's tx bits (lane_bits).
template <int FB>
struct PermSlicer {
    static constexpr int SIDE = 1 << (FB / 2), HB = FB / 2;
    static constexpr uint32_t BYTE_MASK = 0x01010101u * ((1u << FB) - 1u);
    f32x2 mul, add, magic, smax;
    uint32_t ti[4], tq[4];  // byte k: ipat[k] / qpat[k] << HB (k < SIDE)

    // scale: factor between the slicer input and the constellation's scale (1/sqrt(N)
    // when the FFT output is left unnormalised)
    __device__ void load(const AxisInfo& a, float scale) {
        // clamp form: the level coordinate divided by side - 1 (QPSK: side - 1 = 1)
        const double span = (double)(SIDE - 1);
        const float is = (float)(a.inv_step * (double)scale / span);
        const float off = (float)(-a.lev0 * a.inv_step / span);
        mul = f32x2{is, is};
        add = f32x2{off, off};
        magic = f32x2{12582912.0f, 12582912.0f};
        smax = f32x2{(float)(SIDE - 1), (float)(SIDE - 1)};
        for (int w = 0; w < 4; ++w) ti[w] = tq[w] = 0u;
        for (int k = 0; k < SIDE; ++k) {
            ti[k >> 2] |= (uint32_t)a.ipat[k] << (8 * (k & 3));
            tq[k >> 2] |= ((uint32_t)a.qpat[k] << HB) << (8 * (k & 3));
        }
    }
    // byte j of the result = table[byte j of sel]
    __device__ __forceinline__ static uint32_t lookup(const uint32_t (&tb)[4], uint32_t sel) {
        if constexpr (SIDE <= 8) {
            return __builtin_amdgcn_perm(tb[1], tb[0], sel);
        } else {
            const uint32_t s7 = sel & 0x07070707u;
            const uint32_t lo = __builtin_amdgcn_perm(tb[1], tb[0], s7);
            const uint32_t hi = __builtin_amdgcn_perm(tb[3], tb[2], s7);
            // 0xff in byte j when bit 3 of byte j of sel is set: the perm sign selectors
            // 8..11 read bit 7 of bytes 1, 3 (S1) and 5, 7 (S0)
            const uint32_t m = __builtin_amdgcn_perm(sel << 12, sel << 4, 0x090B080Au);
            return (hi & m) | (lo & ~m);
        }
    }
    // (rx ^ tx) indices of four elements, one per byte; txw = the lane word (unmasked)
    __device__ __forceinline__ uint32_t diff(const cpx<float> (&z)[4], uint32_t txw) const {
        uint32_t li[4], lq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // both axes clamped to [0, 1] by the clamp bit of v_pk_fma_f32 (tools/clamp_probe.hip)
            f32x2 v;
            asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(v) : "v"(z[j].v), "v"(mul), "v"(add));
            // the rounded levels taken as a 64-bit integer: read back as a float2 whose lanes
            // are bit-cast, the compiler used lane 0 for both axes (as in adaptive_diff)
            uint64_t fb;
            asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(fb) : "v"(v), "v"(smax), "v"(magic));
            li[j] = (uint32_t)fb;  // level in the low byte
            lq[j] = (uint32_t)(fb >> 32);
        }
        const uint32_t si = __builtin_amdgcn_perm(__builtin_amdgcn_perm(li[3], li[2], 0x0c0c0400u),
                                                  __builtin_amdgcn_perm(li[1], li[0], 0x0c0c0400u), 0x05040100u);
        const uint32_t sq = __builtin_amdgcn_perm(__builtin_amdgcn_perm(lq[3], lq[2], 0x0c0c0400u),
                                                  __builtin_amdgcn_perm(lq[1], lq[0], 0x0c0c0400u), 0x05040100u);
        return (lookup(ti, si) | lookup(tq, sq)) ^ (txw & BYTE_MASK);
    }
    // number of non-zero bytes
    __device__ __forceinline__ static uint32_t nonzero_bytes(uint32_t d) {
        if constexpr (FB < 8)
            return __popc((d + 0x7F7F7F7Fu) & 0x80808080u);  // bytes < 0x80: no carry out
        else
            return __popc((((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u);
    }
};

// complex128 throughput slicer (same decisions and tables as PermSlicer): the level
// coordinate of each axis is one v_fma_f64 with the clamp bit (y / (side - 1) clamped to
// [0, 1]), and a second one v * (side - 1) + 1.5*2^52 leaves round(y) in the low mantissa word
// (round-to-nearest-even; a tie is a decision boundary, probability zero under noise) -- both
// in double precision, so a decision differs from the reference's float64 nearest-point search
// only for points within ~1e-16 of a boundary.
template <int FB>
struct PermSlicer64 {
    static constexpr int SIDE = 1 << (FB / 2), HB = FB / 2;
    static constexpr uint32_t BYTE_MASK = 0x01010101u * ((1u << FB) - 1u);
    double mul, add, smax, magic;
    uint32_t ti[4], tq[4];

    // the constants are workgroup-uniform: held in SGPR pairs (readfirstlane), so each v_fma_f64
    // takes one scalar operand instead of a VGPR copy
    __device__ static double uniform(double x) {
        const uint64_t u = __builtin_bit_cast(uint64_t, x);
        // readfirstlane returns a signed int: widen through uint32_t, or bit 31 of the low word
        // would sign-extend into the high word
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
        return __builtin_bit_cast(double, lo | (hi << 32));
    }
    __device__ void load(const AxisInfo& a, double scale) {
        const double span = (double)(SIDE - 1);
        mul = uniform(a.inv_step * scale / span);
        add = a.lev0 * a.inv_step / span;  // negated in the FMA (neg modifier)
        smax = span;
        magic = uniform(6755399441055744.0);  // 1.5 * 2^52
        for (int w = 0; w < 4; ++w) ti[w] = tq[w] = 0u;
        for (int k = 0; k < SIDE; ++k) {
            ti[k >> 2] |= (uint32_t)a.ipat[k] << (8 * (k & 3));
            tq[k >> 2] |= ((uint32_t)a.qpat[k] << HB) << (8 * (k & 3));
        }
    }
    // Both FMAs in asm: written in C the second became an in-place v_fmac_f64 whose addend (the
    // 1.5 * 2^52 constant) was rebuilt by two v_mov_b32 before every decision.
    __device__ __forceinline__ uint32_t level(double u) const {
        double v, f;
        asm("v_fma_f64 %0, %1, %2, -%3 clamp" : "=v"(v) : "v"(u), "s"(mul), "v"(add));
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(f) : "v"(v), "v"(smax), "s"(magic));
        return (uint32_t)__builtin_bit_cast(uint64_t, f);
    }
    // the same with a per-element level multiplier m = s mul (z s the point: the MMSE scale s folded in)
    __device__ __forceinline__ uint32_t level_m(double u, double m) const {
        double v, f;
        asm("v_fma_f64 %0, %1, %2, -%3 clamp" : "=v"(v) : "v"(u), "v"(m), "v"(add));
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(f) : "v"(v), "v"(smax), "s"(magic));
        return (uint32_t)__builtin_bit_cast(uint64_t, f);
    }
    __device__ __forceinline__ uint32_t diff(const cpx<double> (&z)[4], uint32_t txw) const {
        uint32_t li[4], lq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            li[j] = level(z[j].re);
            lq[j] = level(z[j].im);
        }
        return combine(li, lq, txw);
    }
    __device__ __forceinline__ uint32_t diff_scaled(const cpx<double> (&z)[4], const double (&s)[4], uint32_t txw) const {
        uint32_t li[4], lq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double m = s[j] * mul;
            li[j] = level_m(z[j].re, m);
            lq[j] = level_m(z[j].im, m);
        }
        return combine(li, lq, txw);
    }
    __device__ __forceinline__ uint32_t combine(const uint32_t (&li)[4], const uint32_t (&lq)[4], uint32_t txw) const {
        const uint32_t si = __builtin_amdgcn_perm(__builtin_amdgcn_perm(li[3], li[2], 0x0c0c0400u),
                                                  __builtin_amdgcn_perm(li[1], li[0], 0x0c0c0400u), 0x05040100u);
        const uint32_t sq = __builtin_amdgcn_perm(__builtin_amdgcn_perm(lq[3], lq[2], 0x0c0c0400u),
                                                  __builtin_amdgcn_perm(lq[1], lq[0], 0x0c0c0400u), 0x05040100u);
        return (PermSlicer<FB>::lookup(ti, si) | PermSlicer<FB>::lookup(tq, sq)) ^ (txw & BYTE_MASK);
    }
};

// ------------------------------------------------------------------ adaptive throughput slicer
// The reference's square-QAM LUTs (constellation/models.py:180-218) share one level -> index
// pattern for every order: ipat_M[k] is the first sqrt(M) entries of
// U = [0 1 3 2 7 6 4 5 15 14 12 13 8 9 11 10], and qpat_M[k] = U[sqrt(M) - 1 - k] (the Q
// levels run the other way; the plan checks both, ofdm_abi.hip:universal_patterns).  So a
// per-subcarrier order changes only the level scale, the clamp and the bit split: the Q level
// is taken on -Im z, both axes look up U, and the Q bits move up by b_k/2.
constexpr uint32_t kUPat[4] = {0x02030100u, 0x05040607u, 0x0D0C0E0Fu, 0x0A0B0908u};

// byte j of the result = U[byte j of sel] (bytes of sel < 16; SMALL: < 8, orders <= 64)
template <bool SMALL = false>
__device__ __forceinline__ uint32_t upat_lookup(uint32_t sel) {
    if constexpr (SMALL) return __builtin_amdgcn_perm(kUPat[1], kUPat[0], sel);
    const uint32_t s7 = sel & 0x07070707u;
    const uint32_t lo = __builtin_amdgcn_perm(kUPat[1], kUPat[0], s7);
    const uint32_t hi = __builtin_amdgcn_perm(kUPat[3], kUPat[2], s7);
    const uint32_t m = __builtin_amdgcn_perm(sel << 12, sel << 4, 0x090B080Au);  // 0xff where bit 3 set
    return (hi & m) | (lo & ~m);
}

// Per-order slicer constants in LDS (one entry per LUT of the plan, entry 7 = unused
// subcarrier): level coordinate y = z * mul + add divided by side - 1 (clamped to [0, 1]), smax
// = side - 1 as a float (0 for the unused entry), and meta = tx bit mask (1 << b) - 1 |
// (1 << b/2) << 8.
struct OrderParams {
    float mul, add;
    uint32_t smax, meta;
};
constexpr int kUnusedOrder = 7;

// (rx ^ tx) of four elements from their levels (li: I axis, lq: Q axis on -Im z, level in the low
// byte), per-order meta words and the lane word: U lookups, Q bits moved up by b_j / 2, tx mask
template <bool SMALL>
__device__ __forceinline__ uint32_t adaptive_combine(const uint32_t (&li)[4], const uint32_t (&lq)[4],
                                                     const uint32_t (&meta)[4], uint32_t txw) {
    const uint32_t si = __builtin_amdgcn_perm(__builtin_amdgcn_perm(li[3], li[2], 0x0c0c0400u),
                                              __builtin_amdgcn_perm(li[1], li[0], 0x0c0c0400u), 0x05040100u);
    const uint32_t sq = __builtin_amdgcn_perm(__builtin_amdgcn_perm(lq[3], lq[2], 0x0c0c0400u),
                                              __builtin_amdgcn_perm(lq[1], lq[0], 0x0c0c0400u), 0x05040100u);
    const uint32_t ib = upat_lookup<SMALL>(si), qb = upat_lookup<SMALL>(sq);
    // Q bits << b_j/2 per byte: bytes 0, 2 and 1, 3 as u16 pairs through v_pk_mul_lo_u16
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t w02 = __builtin_amdgcn_perm(0u, qb, 0x0c020c00u), w13 = __builtin_amdgcn_perm(0u, qb, 0x0c030c01u);
    const uint32_t f02 = __builtin_amdgcn_perm(meta[2], meta[0], 0x0c050c01u);
    const uint32_t f13 = __builtin_amdgcn_perm(meta[3], meta[1], 0x0c050c01u);
    const uint32_t p02 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, w02) * __builtin_bit_cast(u16x2, f02));
    const uint32_t p13 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, w13) * __builtin_bit_cast(u16x2, f13));
    const uint32_t qs = __builtin_amdgcn_perm(p13, p02, 0x06020400u);
    const uint32_t mw = __builtin_amdgcn_perm(__builtin_amdgcn_perm(meta[3], meta[2], 0x0c0c0400u),
                                              __builtin_amdgcn_perm(meta[1], meta[0], 0x0c0c0400u), 0x05040100u);
    return (ib | qs) ^ (txw & mw);
}

// (rx ^ tx) of four elements of possibly different orders, one per byte.  op[j] = the
// element's order entry, txw = the lane word; mask_out = the tx masks (byte j).  SMALL: every
// order of the plan is <= 64 (levels < 8: one v_perm per U lookup).
template <bool SMALL>
__device__ __forceinline__ uint32_t adaptive_diff(const cpx<float> (&z)[4], const OrderParams* const (&op)[4],
                                                  uint32_t txw) {
    const f32x2 magic2 = f32x2{12582912.0f, 12582912.0f};
    uint32_t li[4], lq[4], meta[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // level coordinates (Re z * mul + add, -Im z * mul + add) in one v_pk_fma_f32: (mul, add)
        // is one register pair, splatted / negated by the operand modifiers (written in C the
        // two axes' chains were merged -- the Q axis vanished from the ISA).
        // The result is taken as a 64-bit integer: read back as a float2 whose lanes are then
        // bit-cast, the compiler used lane 0 for both (reproduced in a 15-line kernel)
        const f32x2 ma = *(const f32x2*)&op[j]->mul;
        // (mul, add) hold the coordinate / (side - 1), clamped to [0, 1] by the clamp bit (as
        // PermSlicer); smax holds side - 1 as a float, splatted by op_sel_hi
        f32x2 v;
        asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1] neg_hi:[0,1,0] clamp"
            : "=v"(v)
            : "v"(z[j].v), "v"(ma));
        const f32x2 sm = *(const f32x2*)&op[j]->smax;
        uint64_t f;
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(f) : "v"(v), "v"(sm), "v"(magic2));
        li[j] = (uint32_t)f;
        lq[j] = (uint32_t)(f >> 32);
        // opaque to the v_perm byte-provider combine, which otherwise merges the Q gather
        // into the I gather (seen with run-time clamp bounds: the Q axis vanished)
        asm("" : "+v"(li[j]), "+v"(lq[j]));
        meta[j] = op[j]->meta;
    }
    return adaptive_combine<SMALL>(li, lq, meta, txw);
}

// ------------------------------------------------------------------ exact power sums
// The AWGN power is the whole-stream mean of |y|^2 (noise/models.py:14).  Summed in floating
// point, its last bits would depend on how symbols are batched, sharded over GPUs and reduced, and
// so would sigma.  Instead every lane's share of one OFDM symbol's sum |y|^2 -- a fixed set of
// samples, summed in a fixed order -- is rounded once to 2^-40 fixed point and accumulated as two
// 32-bit limbs in 64-bit integers: the total is exact integer arithmetic, independent of every
// grouping.  Value = limb1 2^-8 + limb0 2^-40 (kFxLo / kFxHi), limb0 < 2^32 after normalisation;
// a lane's share is < 2^24 (unit-power signals), so limb1 stays exact in a double.
constexpr double kFxHi = 0x1p-8, kFxLo = 0x1p-40;
__device__ __forceinline__ void fx_accum(double p, unsigned long long& l0, unsigned long long& l1) {
    const double a = p * 256.0;  // exact
    const double hi = floor(a);
    l1 += (unsigned long long)(uint32_t)hi;
    // (a - hi) exact; its rounded multiple of 2^-40 can be exactly 2^32 (a fraction within 2^-41 of
    // 1), so it is converted through 64 bits: the carry reaches l1 in fx_normalize
    l0 += (unsigned long long)rint((a - hi) * 4294967296.0);
}
// complex64: the same limbs from a float32 share in float32 arithmetic.  Every step is exact:
// p 2^8, its floor and its fraction are floats (Sterbenz), the fraction times 2^32 is a float below
// 2^32, and only when p < 2^-17 does it carry bits below 2^0, which v_rndne_f32 rounds as rint does
// in double -- so the limbs equal those of the double path (tests/test_fixed_point.py restates
// both), at ~10 full-rate VALU instead of ~10 f64 operations and conversions per lane and symbol.
__device__ __forceinline__ void fx_accum(float p, unsigned long long& l0, unsigned long long& l1) {
    const float a = p * 256.0f;
    const float hi = __builtin_floorf(a);
    l1 += (unsigned long long)(uint32_t)hi;
    l0 += (unsigned long long)(uint32_t)__builtin_rintf((a - hi) * 4294967296.0f);
}
__host__ __device__ inline void fx_normalize(unsigned long long& l0, unsigned long long& l1) {
    l1 += l0 >> 32;
    l0 &= 0xFFFFFFFFull;
}
__host__ __device__ inline double fx_value(unsigned long long l0, unsigned long long l1) {
    return (double)l1 * kFxHi + (double)l0 * kFxLo;
}

// complex128 adaptive slicer: per-order constants in double (entries of 32 bytes, so the byte
// offsets of the eight entries still fit the per-element code bytes), the same decisions and
// bit handling as adaptive_diff; both FMAs of each axis in asm (the clamp bit, and no in-place
// v_fmac rebuilding the rounding constant).
// Two 16-byte vectors, each read by one ds_read_b128: ma = {mul, add}: level coordinate / (side - 1)
// = z mul - add, clamped; times smax; sm = {smax, meta} with the meta word in the low half of the
// second element's bits (written and read through bit casts, never as arithmetic).  Field by field
// the compiler read ds_read2_b64 + ds_read_b64 + ds_read_b32 per element, and the 2-address read
// serves a lane group at half the rate and conflicts for entries 4 apart.
struct alignas(16) OrderParams64 {
    f64x2 ma, sm;
    __device__ static OrderParams64 make(double mul, double add, double smax, uint32_t meta) {
        return OrderParams64{f64x2{mul, add}, f64x2{smax, __builtin_bit_cast(double, (uint64_t)meta)}};
    }
};
static_assert(sizeof(OrderParams64) == 32, "two 16-byte halves");
// SCALED: z unscaled and s[j] its MMSE scale, folded into the order's level multiplier
template <bool SMALL, bool SCALED = false>
__device__ __forceinline__ uint32_t adaptive_diff64(const cpx<double> (&z)[4], const OrderParams64* const (&op)[4],
                                                    uint32_t txw, double magic, const double (&s)[4]) {
    uint32_t li[4], lq[4], meta[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const f64x2 ma = op[j]->ma;  // {mul, add}
        const f64x2 sm = op[j]->sm;  // {smax, meta}
        const double m = SCALED ? s[j] * ma.x : ma.x;
        double vi, vq, fi, fq;
        asm("v_fma_f64 %0, %1, %2, -%3 clamp" : "=v"(vi) : "v"(z[j].re), "v"(m), "v"(ma.y));
        asm("v_fma_f64 %0, -%1, %2, -%3 clamp" : "=v"(vq) : "v"(z[j].im), "v"(m), "v"(ma.y));
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(fi) : "v"(vi), "v"(sm.x), "s"(magic));
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(fq) : "v"(vq), "v"(sm.x), "s"(magic));
        li[j] = (uint32_t)__builtin_bit_cast(uint64_t, fi);
        lq[j] = (uint32_t)__builtin_bit_cast(uint64_t, fq);
        asm("" : "+v"(li[j]), "+v"(lq[j]));
        // (the meta word through a bit cast of the whole vector: clang 20 resolved a bit cast of the
        // element sm.y to element 0's register)
        typedef uint32_t u32x4m __attribute__((ext_vector_type(4)));
        meta[j] = __builtin_bit_cast(u32x4m, sm).z;
    }
    return adaptive_combine<SMALL>(li, lq, meta, txw);
}

// ------------------------------------------------------------------ reductions
// Sum over the TPS threads of one symbol group (t = threadIdx.x % TPS).  All threads
// of the workgroup must call it (uses a workgroup barrier for TPS > 64).
template <typename T, int TPS>
__device__ __forceinline__ T group_sum(T v, T* scratch /* block / 64 entries */) {
    if constexpr (TPS == 1) {
        return v;
    } else if constexpr (TPS <= 64) {
#pragma unroll
        for (int off = TPS / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        return v;
    } else {
        // TPS = 128 or 256: per-wave reduce then combine through LDS
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) scratch[wave] = v;
        __syncthreads();
        const int first = (threadIdx.x / TPS) * (TPS / 64);
        T s = 0;
#pragma unroll
        for (int w = 0; w < TPS / 64; ++w) s += scratch[first + w];
        __syncthreads();
        return s;
    }
}

template <typename T, int BLK = kBlock>
__device__ __forceinline__ T block_sum(T v, T* scratch /* BLK / 64 entries */) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < BLK / 64; ++w) s += scratch[w];
    __syncthreads();
    return s;  // valid in thread 0
}

template <typename T, int BLK = kBlock>
__device__ __forceinline__ T block_max(T v, T* scratch /* BLK / 64 entries */) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < BLK / 64; ++w) s = scratch[w] > s ? scratch[w] : s;
    __syncthreads();
    return s;
}

// ------------------------------------------------------------------ Philox4x32-10
struct u4 {
    uint32_t x, y, z, w;
};

// a ^ b ^ k in one v_bitop3_b32 (truth table 0x96); k wave-uniform.  The compiler emits
// two v_xor_b32 for the expression.
__device__ __forceinline__ uint32_t xor3_s(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

// OFDM_PHILOX_ROUNDS: diagnostic builds only (timing of the seeding cost); the stream
// definition is Philox4x32-10
#ifndef OFDM_PHILOX_ROUNDS
#define OFDM_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
    // keep the key schedule in the loop (SALU adds next to the VALU rounds): hoisted out of
    // a symbol loop it is 20 live SGPRs and spills
    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int i = 0; i < OFDM_PHILOX_ROUNDS; ++i) {
        // one v_mad_u64_u32 per 32x32->64 product, one v_bitop3 per three-way xor
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        u4 n;
        if (i == 0) {  // round 0: c.y, c.w are wave-uniform (symbol index, stream id)
            n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
            n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        } else {
            n.x = xor3_s((uint32_t)(p1 >> 32), c.y, k0);
            n.z = xor3_s((uint32_t)(p0 >> 32), c.w, k1);
        }
        n.y = (uint32_t)p1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// ------------------------------------------------------------------ throughput-mode streams
// Definition (philox mode, stream version 3): thread t of OFDM symbol s owns elements
// k = t + TPS*i.  One Philox4x32-10 block per lane, key = seed, counter = (t, s mod 2^32,
// s >> 32, kLane), gives words P0..P3.  The lane's 128 payload bits are the words
// (P2, P3, m0, m1) (element i takes the low b_k bits of byte i, see lane_bits), where m0, m1,
// ... are the outputs of an MWC64X generator seeded with x = P0, c = (P1 >> 1) | 1.  The
// generator then continues into the lane's noise samples j = 0, 1, ... (the E elements, then
// the zero-padding tail samples it owns): before samples j = 0, 4, 8, ... it draws a phase
// word q, and every sample draws its radius word w (Mwc64x::draw) -- outputs m2 = q0,
// m3..m6 = w0..w3, m7 = q1, ...  Sample j's complex normal is radius(w) times phase-table
// entry (q >> 8 (j & 3)) & 63 (Mwc64x::add_noise).  Everything depends only on (seed, s, N),
// so results do not depend on how symbols are batched or sharded.
// (Stream version 2 took the phase from bits 3..8 of the radius word and forced them to one
// in the radius, which truncated the radius at 5.65 sigma; version 3 gives the radius the whole
// word -- the Rayleigh quantile at the midpoints of 2^31 equiprobable cells, exact at every cell
// boundary down to P = 2^-31 at 6.555 sigma -- and costs one generator step per four samples,
// where version 2 recomputed x ^ c for each phase.)
constexpr uint32_t kLane = 0x1A7E5EEDu;

__device__ __forceinline__ u4 philox_lane(uint64_t seed, int64_t s, uint32_t t, uint32_t stream) {
    u4 c;
    c.x = t;
    c.y = (uint32_t)s;
    c.z = (uint32_t)((uint64_t)s >> 32);
    c.w = stream;
    return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Element i of a lane takes the low b bits of byte i of the lane's 128-bit block
// (byte i = bits 8*(i&3).. of word i>>2): one v_bfe_u32, and four elements of the rx
// decisions compare against one word.
__device__ __forceinline__ uint32_t lane_word(const u4& w, int q) {
    return q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
}
__device__ __forceinline__ uint32_t lane_bits(const u4& w, int i, int b) {
    return (lane_word(w, i >> 2) >> (8 * (i & 3))) & ((1u << b) - 1u);
}

// Noise phase table: kNoisePhases points e^{2 pi i (j + 1/2) / 64} scaled by
// sigma sqrt(2 ln 2) (float32), one per workgroup in static LDS.  A uniform phase taken on 64
// points leaves the noise's projection on any direction Gaussian to within the trapezoid rule's
// error on the smooth periodic tail integrand: P(Re(n e^{-i phi}) > d sigma) is off by < 2e-6
// relative for every phi and d >= 1, < 1e-10 at d >= 3 (tests/test_oracle_philox.py).
constexpr int kNoisePhases = 64;
constexpr double kSqrt2Ln2 = 1.1774100225154747;  // sqrt(2 ln 2)

// MWC64X (D. B. Thomas, multiply-with-carry, base 2^32, A = 4294883355): state (x, c),
// output x ^ c, then (c, x) <- hi/lo of A x + c -- one v_mad_u64_u32 (plus the move of the
// carry into the addend pair and the xor) per 32-bit output.  Seeded from one Philox block:
// c = (P1 >> 1) | 1 < A, so the state is never one of the two fixed points.
constexpr uint32_t kMwcA = 4294883355u;
// sqrt(32 - log2(float(w | 1))) on the float32 hardware log2 / sqrt: sigma sqrt(-2 ln u) / (sigma
// sqrt(2 ln 2)) with u = float(w | 1) 2^-32 in [2^-32, 1] (words 2k and 2k + 1 share the cell
// midpoint (2k + 1) 2^-32, so u > 0; the largest radius is sqrt(32) sqrt(2 ln 2) = 6.660 sigma, the
// next 6.493).  The |.| (a free source
// modifier) keeps the square root real when the approximate log2 of a word rounding to 2^32 comes
// out slightly above 32: the radius is then ~0 instead of NaN.
__device__ __forceinline__ float noise_radius(uint32_t w) {
    return __builtin_amdgcn_sqrtf(__builtin_fabsf(32.0f - __builtin_amdgcn_logf((float)(w | 1u))));
}

struct Mwc64x {
    uint32_t x, c;
    uint32_t q;  // the current phase word (noise samples 4 (j >> 2) .. 4 (j >> 2) + 3)
    __device__ __forceinline__ void seed(uint32_t p0, uint32_t p1) {
        x = p0;
        c = (p1 >> 1) | 1u;
    }
    __device__ __forceinline__ uint32_t next() {
        const uint32_t r = x ^ c;
        const uint64_t v = (uint64_t)kMwcA * x + c;
        x = (uint32_t)v;
        c = (uint32_t)(v >> 32);
        return r;
    }
    // noise sample j of the lane (j a compile-time constant in the unrolled kernels): the phase
    // word first when j = 0 mod 4, then the sample's radius word
    __device__ __forceinline__ uint32_t draw(int j) {
        if ((j & 3) == 0) q = next();
        return next();
    }
    // byte offset of sample j's phase entry in a table of ENTRY-byte entries
    template <int ENTRY>
    __device__ __forceinline__ uint32_t phase_off(int j) const {
        return ((q >> (8 * (j & 3))) & (uint32_t)(kNoisePhases - 1)) * (uint32_t)ENTRY;
    }
    // One complex normal with per-component standard deviation sigma, noise sample j: radius
    // sigma sqrt(-2 ln u) = sigma sqrt(2 ln 2) sqrt(32 - log2(w | 1)) on the hardware v_log_f32
    // (log2) / v_sqrt_f32, the phase entry (already holding sigma sqrt(2 ln 2)) from the phase word.
    __device__ __forceinline__ f32x2 sample(int j, const f32x2* ntab, float& r) {
        r = noise_radius(draw(j));
        return *(const f32x2*)((const unsigned char*)ntab + phase_off<sizeof(f32x2)>(j));
    }
    __device__ __forceinline__ void add_noise(f32x2& x0, const f32x2* ntab, int j) {
        float r;
        const f32x2 e = sample(j, ntab, r);
        x0 = __builtin_elementwise_fma(f32x2{r, r}, e, x0);
    }
    __device__ __forceinline__ f32x2 noise(const f32x2* ntab, int j) {
        float r;
        const f32x2 e = sample(j, ntab, r);
        return f32x2{r, r} * e;
    }
    // complex128 without the widened table (the generic kernel, zero-padding tail samples): the
    // same exact product of the float32 radius and entry, fused into the sample
    __device__ __forceinline__ void add_noise_f64(double& re, double& im, const f32x2* ntab, int j) {
        float r;
        const f32x2 e = sample(j, ntab, r);
        re = __builtin_fma((double)r, (double)e.x, re);
        im = __builtin_fma((double)r, (double)e.y, im);
    }
    // complex128 kernels: the same radius and phase entry, the product taken in double against
    // ntab64 = the float32 table entries widened (exact), fused into the sample: one conversion
    // and two v_fma_f64 instead of a float product and two conversions.  (16 copies of the table,
    // one per 16-byte bank slot so that a ds_read_b128 lane group never meets on a bank, measured
    // slower: config b RX 3.07 -> 3.25 ms, profiles/r03m_ab.txt.)
    __device__ __forceinline__ void add_noise64(double& re, double& im, const f64x2* ntab64, int j) {
        const float r = noise_radius(draw(j));
        const f64x2 e = *(const f64x2*)((const unsigned char*)ntab64 + phase_off<sizeof(f64x2)>(j));
        const double rd = (double)r;
        re = __builtin_fma(rd, e.x, re);
        im = __builtin_fma(rd, e.y, im);
    }
};

// A workgroup prologue's copy of a global table into LDS, split into load() and store() so that
// a kernel issues the reads of all its tables before the first wait: each copy loop waited for
// its own loads (global_load, s_waitcnt vmcnt(0), ds_write per trip), and the prologues of the
// fused kernels chained five or six memory latencies per workgroup (neutral on the steady state,
// DESIGN.md section 4, but no longer a chain).  The first K trips
// of each thread are held in registers; a longer table (MAXN > 8 BLK, or a count not bounded by
// MAXN: BOUNDED false) copies its remainder in store().  The caller syncs.
template <int BLK, int MAXN, typename T, bool BOUNDED = true>
struct Staged {
    static constexpr int K = MAXN <= 0 ? 0 : ((MAXN + BLK - 1) / BLK < 8 ? (MAXN + BLK - 1) / BLK : 8);
    T v[K > 0 ? K : 1];
    const T* src = nullptr;
    int n = 0;
    __device__ __forceinline__ void load(const T* s, int cnt) {
        src = s;
        n = cnt;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = (int)threadIdx.x + k * BLK;
            if (i < n) v[k] = s[i];
        }
    }
    template <class F>
    __device__ __forceinline__ void store(T* dst, F f) const {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = (int)threadIdx.x + k * BLK;
            if (i < n) dst[i] = f(v[k]);
        }
        if constexpr (!BOUNDED || MAXN > K * BLK)
            for (int i = (int)threadIdx.x + K * BLK; i < n; i += BLK) dst[i] = f(src[i]);
    }
    __device__ __forceinline__ void store(T* dst) const {
        store(dst, [](const T& x) { return x; });
    }
};

// a struct's bytes as dwords: staged as such, a struct of byte arrays (AxisInfo) is copied with
// its loads' registers as they are, not split into bytes and packed again
template <typename T>
struct Dwords {
    static_assert(sizeof(T) % 4 == 0, "dword-sized");
    uint32_t w[sizeof(T) / 4];
};

// Build the noise phase table in LDS (threads < 64; caller syncs); ntab64 (complex128 kernels,
// or null): the same float32 entries widened to double.
__device__ __forceinline__ void build_noise_table(f32x2* ntab, double sigma, f64x2* ntab64 = nullptr) {
    if (threadIdx.x < kNoisePhases) {
        const float s = (float)(sigma * kSqrt2Ln2);
        const double th = (2.0 * threadIdx.x + 1.0) / kNoisePhases;  // (j + 1/2) / 32 half-turns
        const f32x2 e = f32x2{s * (float)cospi(th), s * (float)sinpi(th)};
        ntab[threadIdx.x] = e;
        if (ntab64) ntab64[threadIdx.x] = f64x2{(double)e.x, (double)e.y};
    }
}

// ------------------------------------------------------------------ constellation tables
template <typename R>
__device__ __forceinline__ int slice_axis(R u, const AxisInfo& a) {
    R t = (u - (R)a.lev0) * (R)a.inv_step + (R)0.5;
    int k = (int)floor(t);
    k = k < 0 ? 0 : k;
    k = k > a.side - 1 ? a.side - 1 : k;
    return k;
}

template <typename R>
__device__ __forceinline__ uint32_t slice(cpx<R> z, const AxisInfo& a) {
    const int ki = slice_axis<R>(z.re, a), kq = slice_axis<R>(z.im, a);
    return ((uint32_t)a.qpat[kq] << a.hbits) | (uint32_t)a.ipat[ki];
}

// b (<= 8) bits at bit offset o of an MSB-first byte buffer with >= 1 byte of slack.
__device__ __forceinline__ uint32_t extract_bits(const uint8_t* bytes, int64_t o, int b) {
    const int64_t B = o >> 3;
    const uint32_t w = ((uint32_t)bytes[B] << 8) | (uint32_t)bytes[B + 1];
    return (w >> (16 - (int)(o & 7) - b)) & ((1u << b) - 1u);
}

}  // namespace ofdm
