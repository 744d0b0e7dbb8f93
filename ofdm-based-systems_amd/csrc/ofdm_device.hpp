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

// ------------------------------------------------------------------ small DFTs
template <typename R, bool INV>
__device__ __forceinline__ void dft2(cpx<R>& a, cpx<R>& b) {
    cpx<R> t = a - b;
    a = a + b;
    b = t;
}

template <typename R, bool INV>
__device__ __forceinline__ void dft4(cpx<R>& v0, cpx<R>& v1, cpx<R>& v2, cpx<R>& v3) {
    cpx<R> t0 = v0 + v2, t1 = v0 - v2, t2 = v1 + v3, t3 = rot90<R, INV>(v1 - v3);
    v0 = t0 + t2;
    v2 = t0 - t2;
    v1 = t1 + t3;
    v3 = t1 - t3;
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
        a[1][2] = rot90<R, INV>(a[1][2]);
        a[1][3] = cmul(a[1][3], w16<R, INV>(6));
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            cpx<R> p = a[0][k1], q = a[1][k1];
            v[k1] = p + q;
            v[k1 + 4] = p - q;
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
                if (e == 4)
                    a[n2][k1] = rot90<R, INV>(a[n2][k1]);
                else
                    a[n2][k1] = cmul(a[n2][k1], w16<R, INV>(e));
            }
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            cpx<R> b0 = a[0][k1], b1 = a[1][k1], b2 = a[2][k1], b3 = a[3][k1];
            dft4<R, INV>(b0, b1, b2, b3);
            v[k1] = b0;
            v[k1 + 4] = b1;
            v[k1 + 8] = b2;
            v[k1 + 12] = b3;
        }
    }
}

// ------------------------------------------------------------------ FFT geometry
template <int LOGN>
struct Geo {
    static constexpr int N = 1 << LOGN;
    static constexpr int LOGE = LOGN < 4 ? LOGN : 4;
    static constexpr int E = 1 << LOGE;   // elements per thread
    static constexpr int TPS = N / E;     // threads per symbol
    static constexpr int SPB = kBlock / TPS;  // symbols per workgroup
    static constexpr int PADN = N + (N >> 4) + 1;  // padded LDS row (complex elements)
};

__device__ __forceinline__ int pad(int i) { return i + (i >> 4); }

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
        __syncthreads();
    }
}

// One Stockham pass with the data distribution "thread t owns elements t + i*TPS".
// FIRST: inputs come from x[] (valid because the first pass has RAD = E, STRIDE = TPS);
// LAST: outputs stay in x[] (the last pass writes j + r*NS with j = t + q*TPS and
// NS = TPS*E/RAD, i.e. element t + (q + r*NB)*TPS); otherwise through the LDS row.
template <typename R, int LOGN, int LOGR, int LOGNS, bool INV, bool FIRST, bool LAST>
__device__ __forceinline__ void reg_pass(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                         const cpx<R>* hi, int t) {
    using G = Geo<LOGN>;
    constexpr int RAD = 1 << LOGR;
    constexpr int NS = 1 << LOGNS;
    constexpr int NB = G::E / RAD;
    constexpr int STRIDE = G::N / RAD;
    cpx<R> v[NB][RAD];
    if constexpr (FIRST) {
        static_assert(NB == 1 && STRIDE == G::TPS, "first pass consumes the register layout");
#pragma unroll
        for (int r = 0; r < RAD; ++r) v[0][r] = x[r];
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
        if constexpr (LOGNS > 0) {
            // w^r by recurrence from one table lookup: 2 live registers instead of the
            // RAD-1 hoisted table loads (<= 15 roundings: ~1e-6 in f32, ~2e-15 in f64)
            const cpx<R> w1 = twiddle<R, LOGN, INV>(k << (LOGN - LOGNS - LOGR), lo, hi);
            cpx<R> wr = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmul(v[q][r], wr);
                if (r + 1 < RAD) wr = cmul(wr, w1);
            }
        }
        dft<R, RAD, INV>(v[q]);
        if constexpr (LAST) {
#pragma unroll
            for (int r = 0; r < RAD; ++r) x[q + r * NB] = v[q][r];
        } else {
            const int idx = ((j >> LOGNS) << (LOGNS + LOGR)) + k;
#pragma unroll
            for (int r = 0; r < RAD; ++r) buf[pad(idx + r * NS)] = v[q][r];
        }
    }
    if constexpr (!LAST) sym_sync<G::TPS>();
}

template <typename R, int LOGN, int LOGNS, bool INV>
__device__ __forceinline__ void reg_passes(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                           const cpx<R>* hi, int t) {
    if constexpr (LOGNS < LOGN) {
        constexpr int REM = LOGN - LOGNS;
        constexpr int LOGR = REM >= 4 ? 4 : REM;
        reg_pass<R, LOGN, LOGR, LOGNS, INV, LOGNS == 0, LOGNS + LOGR == LOGN>(x, buf, lo, hi, t);
        reg_passes<R, LOGN, LOGNS + LOGR, INV>(x, buf, lo, hi, t);
    }
}

// FFT of one symbol: on entry and exit thread t (of TPS) holds element t + i*TPS in
// x[i].  Unnormalised.  buf is the symbol's private padded LDS row; the caller must
// sym_sync() between an earlier use of buf and this call when TPS > 64.
template <typename R, int LOGN, bool INV>
__device__ __forceinline__ void fft_reg(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* buf, const cpx<R>* lo,
                                        const cpx<R>* hi, int t) {
    if constexpr (LOGN <= 4) {
        dft<R, (1 << LOGN), INV>(x);  // one register-resident pass (TPS = 1)
    } else {
        reg_passes<R, LOGN, 0, INV>(x, buf, lo, hi, t);
    }
}

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

// ------------------------------------------------------------------ reductions
// Sum over the TPS threads of one symbol group (t = threadIdx.x % TPS).  All threads
// of the workgroup must call it (uses a workgroup barrier for TPS > 64).
template <typename T, int TPS>
__device__ __forceinline__ T group_sum(T v, T* scratch /* kBlock entries */) {
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

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kBlock / 64; ++w) s += scratch[w];
    __syncthreads();
    return s;  // valid in thread 0
}

template <typename T>
__device__ __forceinline__ T block_max(T v, T* scratch) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kBlock / 64; ++w) s = scratch[w] > s ? scratch[w] : s;
    __syncthreads();
    return s;
}

// ------------------------------------------------------------------ Philox4x32-10
struct u4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        u4 n;
        n.x = hi1 ^ c.y ^ k0;
        n.y = lo1;
        n.z = hi0 ^ c.w ^ k1;
        n.w = lo0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

constexpr uint32_t kStreamBits = 0xB175B175u;
constexpr uint32_t kStreamNoise = 0x4015E000u;

// Philox bit word w of OFDM symbol s: word (w & 3) of block (w >> 2).
__device__ __forceinline__ u4 philox_bits_block(uint64_t seed, int64_t s, uint32_t blk) {
    u4 c;
    c.x = blk;
    c.y = (uint32_t)s;
    c.z = (uint32_t)((uint64_t)s >> 32);
    c.w = kStreamBits;
    return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Two standard complex normals (re, im each N(0,1)) for kept samples 2p, 2p+1 of
// symbol s.  Box-Muller in fp32 on the hardware transcendentals: v_log_f32 (log2),
// v_sqrt_f32, v_sin_f32 / v_cos_f32 (argument in revolutions).
__device__ __forceinline__ void philox_noise_pair(uint64_t seed, int64_t s, uint32_t p, float& r0,
                                                  float& i0, float& r1, float& i1) {
    u4 c;
    c.x = p;
    c.y = (uint32_t)s;
    c.z = (uint32_t)((uint64_t)s >> 32);
    c.w = kStreamNoise;
    const u4 o = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float k = 2.3283064365386963e-10f;  // 2^-32
    const float u0 = ((float)o.x + 0.5f) * k, v0 = ((float)o.y) * k;
    const float u1 = ((float)o.z + 0.5f) * k, v1 = ((float)o.w) * k;
    const float a0 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u0));
    const float a1 = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
    r0 = a0 * __builtin_amdgcn_cosf(v0);
    i0 = a0 * __builtin_amdgcn_sinf(v0);
    r1 = a1 * __builtin_amdgcn_cosf(v1);
    i1 = a1 * __builtin_amdgcn_sinf(v1);
}

// ------------------------------------------------------------------ throughput-mode streams
// Definition (philox mode): thread t of OFDM symbol s owns elements k = t + TPS*i.
//  * bits : one Philox4x32-10 block keyed (seed; ctr = t, s, kLaneBits) = 128 bits,
//           MSB-first; element i takes the next b_k bits in element order.
//  * noise: xoshiro128** seeded by one Philox4x32-10 block (seed; t, s, kLaneNoise);
//           element i consumes two outputs (u1, u2) -> Box-Muller -> (re, im).
// Both depend only on (seed, s, N), so results do not depend on how symbols are
// batched or sharded across GPUs.
constexpr uint32_t kLaneBits = 0x1A7EB175u;
constexpr uint32_t kLaneNoise = 0x1A7E4015u;

__device__ __forceinline__ u4 philox_lane(uint64_t seed, int64_t s, uint32_t t, uint32_t stream) {
    u4 c;
    c.x = t;
    c.y = (uint32_t)s;
    c.z = (uint32_t)((uint64_t)s >> 32);
    c.w = stream;
    return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// b bits at compile-time offset O of the 128-bit block w0..w3.
template <int O, int Bb>
__device__ __forceinline__ uint32_t bits128_c(const u4& w) {
    constexpr int q = O >> 5, s = O & 31;
    const uint32_t a[4] = {w.x, w.y, w.z, w.w};
    if constexpr (s + Bb <= 32) {
        return (a[q] >> (32 - s - Bb)) & ((1u << Bb) - 1u);
    } else {
        return ((a[q] << (s + Bb - 32)) | (a[q + 1] >> (64 - s - Bb))) & ((1u << Bb) - 1u);
    }
}

// b bits at run-time offset o (o + b <= 128).
__device__ __forceinline__ uint32_t bits128(const u4& w, int o, int b) {
    const int q = o >> 5, s = o & 31;
    const uint32_t hi = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    const uint32_t lo = q == 0 ? w.y : q == 1 ? w.z : q == 2 ? w.w : 0u;
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    return (uint32_t)(x >> (64 - s - b)) & ((1u << b) - 1u);
}

// xoshiro128** (Blackman & Vigna): 4x32-bit state, ~12 simple ALU ops per output.
struct Xoshiro128ss {
    uint32_t s0, s1, s2, s3;
    __device__ __forceinline__ static uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
    __device__ __forceinline__ void seed(const u4& v) {
        s0 = v.x;
        s1 = v.y;
        s2 = v.z;
        s3 = v.w | ((v.x | v.y | v.z) == 0u ? 1u : 0u);  // never the all-zero state
    }
    __device__ __forceinline__ uint32_t next() {
        const uint32_t r = rotl(s1 * 5u, 7) * 9u;
        const uint32_t t = s1 << 9;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl(s3, 11);
        return r;
    }
    // one complex standard normal (re, im each N(0,1)) by Box-Muller on the hardware
    // transcendentals (v_log_f32 = log2, v_sin/cos_f32 take revolutions)
    __device__ __forceinline__ void normal2(float& re, float& im) {
        const float k = 2.3283064365386963e-10f;  // 2^-32
        const float u = ((float)next() + 0.5f) * k;
        const float v = (float)next() * k;
        const float a = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u));
        re = a * __builtin_amdgcn_cosf(v);
        im = a * __builtin_amdgcn_sinf(v);
    }
};

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
