// ofdm_fused.hpp -- the two fused hot-path kernels (included by ofdm_kernels.hpp).
//
// Data distribution: a symbol is owned by TPS = N/E threads; thread t holds
// elements k = t + i*TPS (i < E) in registers from the constellation map through
// the IFFT to the channel output (TX), and from the HBM load through the FFT to
// the error count (RX).  LDS carries only the Stockham transposes between FFT
// passes, the symbol's tx bit words, and (TX, multipath) the extended serial
// stream for the FIR.  With TPS <= 64 a symbol lives in one wavefront and every
// synchronisation is wave-local (sym_sync), so the 4 waves of a workgroup run
// decoupled.
#pragma once

// Minimum waves per SIMD requested per fused kernel (register budget 512/waves), tuned on
// MI355X (tools/ab.sh): TX 3 waves/SIMD, RX unconstrained.  Build-time knobs (Makefile
// TX_WAVES / RX_WAVES) for occupancy studies.
#ifndef OFDM_TX_WAVES
#define OFDM_TX_WAVES 3
#endif
#ifndef OFDM_RX_WAVES
#define OFDM_RX_WAVES 1
#endif

namespace ofdm {

// Stage OFDM symbol s's tx bit stream as 32-bit words in W (stream bit 32w+j =
// bit 31-j of word w).  Returns the offset of the symbol's first bit in word 0.
// Reference mode: the packed bytes of the run (symbol s starts at bit s*bps, zero past
// the end).  Throughput mode: Philox4x32-10 blocks keyed by (seed, s).
template <int TPS>
__device__ __forceinline__ int stage_words(const TxRxCommon& a, int64_t s, uint32_t* W, int t) {
    const int nw = a.words_per_sym;
    if (a.bits) {
        const int64_t bit0 = s * a.bps;
        const int64_t B0 = bit0 >> 3;
        for (int w = t; w < nw; w += TPS) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t B = B0 + 4 * w + i;
                v = (v << 8) | (uint32_t)((B < a.n_bytes && s >= 0) ? a.bits[B] : 0);
            }
            W[w] = v;
        }
        return (int)(bit0 & 7);
    }
    for (int blk = t; blk < (nw >> 2); blk += TPS) {
        const u4 o = philox_bits_block(a.seed, s, (uint32_t)blk);
        uint4 v;
        v.x = o.x;
        v.y = o.y;
        v.z = o.z;
        v.w = o.w;
        *reinterpret_cast<uint4*>(W + 4 * blk) = v;
    }
    return 0;
}

template <typename R>
__device__ __forceinline__ R recip(R d) {
    if constexpr (sizeof(R) == 4)
        return __builtin_amdgcn_rcpf(d);  // v_rcp_f32 (1 ulp): throughput mode
    else
        return (R)1 / d;
}

// MMSE filter coefficient conj(H)/(|H|^2 + nv) (equalization/models.py:58-61).  In f64 the
// two divisions of the reference are kept; in f32 one reciprocal.
template <typename R>
__device__ __forceinline__ cpx<R> mmse_coef(cpx<R> hc, R h2, R nv) {
    const R d = h2 + nv;
    if constexpr (sizeof(R) == 4) {
        const R inv = recip<R>(d);
        return mk<R>(hc.re * inv, hc.im * inv);
    } else {
        return mk<R>(hc.re / d, hc.im / d);
    }
}

// ============================================================ fused TX
// Each symbol group walks `chunk` consecutive OFDM symbols so the FIR tail (last L-1
// stream samples of the previous symbol) is carried in LDS; the first symbol of a chunk
// regenerates its predecessor's tail (one extra IFFT per chunk, L > 1 only).
template <typename R, int LOGN>
__global__ __launch_bounds__(kBlock, OFDM_TX_WAVES) void k_tx(TxArgs a) {
    using G = Geo<LOGN>;
    using C = cpx<R>;
    constexpr int N = G::N, E = G::E, TPS = G::TPS;
    const TxRxCommon& cm = a.c;
    const int cp = cm.cp, L = a.L;
    const int slot = a.slot;  // complex elements per symbol row (>= PADN and >= L-1+cp+N)
    const int tls = L > 1 ? L - 1 : 1;
    Carve cv(ofdm_smem);
    C* tw = cv.take<C>(128);
    C* lut = cv.take<C>(cm.lut_len);
    C* h = cv.take<C>(32);
    AxisInfo* axis = cv.take<AxisInfo>(4);
    C* rows = cv.take<C>((size_t)G::SPB * slot);
    C* tails = cv.take<C>((size_t)G::SPB * tls);
    uint32_t* words = cv.take<uint32_t>((size_t)G::SPB * cm.words_per_sym);
    double* red = cv.take<double>(kBlock / 64);

    load_twiddles<R>(tw, (const C*)cm.tw);
    for (int i = threadIdx.x; i < cm.lut_len; i += kBlock) lut[i] = ((const C*)cm.lut)[i];
    if (threadIdx.x < L) h[threadIdx.x] = ((const C*)a.h)[threadIdx.x];
    if (threadIdx.x < cm.n_axis) axis[threadIdx.x] = cm.axis[threadIdx.x];
    __syncthreads();

    const int ls = threadIdx.x / TPS, t = threadIdx.x % TPS;
    C* row = rows + ls * slot;
    C* tl = tails + ls * tls;
    uint32_t* W = words + ls * cm.words_per_sym;
    C* yout = (C*)a.y;
    const R scale = (R)cm.scale;
    const C h0 = h[0];
    const int64_t ngroups = (cm.n_sym + a.chunk - 1) / a.chunk;
    const int64_t niter = (ngroups + G::SPB - 1) / G::SPB;
    double py = 0, px = 0, mx = 0;

    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        const int64_t grp = it * G::SPB + ls;
        const int64_t sbeg = grp * a.chunk;  // local symbol index
        for (int c = (L > 1 ? -1 : 0); c < a.chunk; ++c) {
            const int64_t sl = sbeg + c;
            const int64_t sg = cm.sym0 + sl;
            const bool active = grp < ngroups && sl < cm.n_sym && sg >= 0;
            int base_bit = 0;
            if (active && !(a.flags & 1)) base_bit = stage_words<TPS>(cm, sg, W, t);
            sym_sync<TPS>();
            // map (QAMConstellationMapper.encode, constellation/models.py:240-246); the
            // 1/sqrt(N) of ifft(norm="ortho") folded in
            C x[E];
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int k = t + i * TPS;
                C v = mk<R>(0, 0);
                if (active) {
                    if (cm.adaptive) {
                        const ScInfo sc = cm.sc[k];
                        if (sc.lut >= 0) v = lut[axis[sc.lut].lut_off + extract_w(W, base_bit + sc.bitoff, sc.bits)];
                    } else {
                        v = lut[extract_w(W, base_bit + k * cm.b, cm.b)];
                    }
                }
                x[i] = cscale(v, scale);
            }
            if (!(a.flags & 2)) fft_reg<R, LOGN, true>(x, row, tw, tw + 64, t);
            // PAPR statistics over the modulated symbol incl. its prefix (simulation/models.py:519-522)
            if (active && c >= 0) {
                R pxs = 0, mxs = 0;  // per-symbol partials in the arithmetic precision
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const int k = t + i * TPS;
                    const R p2 = norm2(x[i]);
                    pxs += k >= N - cp ? 2 * p2 : p2;
                    mxs = fmax(mxs, p2);
                }
                px += pxs;
                mx = fmax(mx, (double)mxs);
            }
            if (L == 1) {
                // flat channel: y = h0 x, no inter-symbol memory
                if (active && c >= 0) {
                    R pys = 0;
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const int k = t + i * TPS;
                        const C yv = cmul(h0, x[i]);
                        const R p2 = norm2(yv);
                        pys += k >= N - cp ? 2 * p2 : p2;
                        if (yout && !(a.flags & 4)) yout[sl * N + k] = yv;
                    }
                    py += pys;
                }
                sym_sync<TPS>();  // W / row reuse by the next symbol
            } else {
                // extended serial stream in the row: [tail (L-1) | prefix (cp) | x (N)]
                sym_sync<TPS>();  // the last FFT pass has read the row
                const int o = L - 1 + cp;
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const int k = t + i * TPS;
                    row[o + k] = x[i];
                    if (k >= N - cp) row[L - 1 + k - (N - cp)] = x[i];
                }
                for (int j = t; j < L - 1; j += TPS) row[j] = tl[j];
                sym_sync<TPS>();
                if (active && c >= 0) {
                    // linear convolution with the unit-power CIR (channel/models.py:52-55)
                    R pys = 0;
                    for (int m = t; m < N + cp; m += TPS) {
                        C yv = mk<R>(0, 0);
                        const C* e = row + (L - 1 + m);
#pragma unroll 8
                        for (int l = 0; l < L; ++l) yv = yv + cmul(h[l], e[-l]);
                        pys += norm2(yv);
                        if (yout && m >= cp && !(a.flags & 4)) yout[sl * N + (m - cp)] = yv;
                    }
                    py += pys;
                }
                // tail for the next symbol: the last L-1 stream samples (zeros before symbol 0)
                for (int j = t; j < L - 1; j += TPS) tl[j] = active ? row[N + cp + j] : mk<R>(0, 0);
                sym_sync<TPS>();
            }
        }
    }
    py = block_sum<double>(py, red);
    px = block_sum<double>(px, red);
    mx = block_max<double>(mx, red);
    if (threadIdx.x == 0) {
        a.partials[blockIdx.x * 3 + 0] = py;
        a.partials[blockIdx.x * 3 + 1] = px;
        a.partials[blockIdx.x * 3 + 2] = mx;
    }
}

// ============================================================ fused RX
// EQ: OFDM_EQ_* fixed at compile time, or -1 = read from the plan at run time.
// FAST: fixed constellation, Philox bits and Philox (or no) noise -- the throughput
// configuration -- with everything else compiled out; otherwise the generic kernel
// (reference-stream bytes and normals, adaptive bit loading).
template <typename R, int LOGN, int EQ, bool FAST>
__global__ __launch_bounds__(kBlock, OFDM_RX_WAVES) void k_rx(RxArgs a) {
    using G = Geo<LOGN>;
    using C = cpx<R>;
    constexpr int N = G::N, E = G::E, TPS = G::TPS;
    const TxRxCommon& cm = a.c;
    const int eq = EQ >= 0 ? EQ : cm.eq;
    const bool adaptive = FAST ? false : (bool)cm.adaptive;
    Carve cv(ofdm_smem);
    C* tw = cv.take<C>(128);
    AxisInfo* axis = cv.take<AxisInfo>(4);
    C* rows = cv.take<C>((size_t)G::SPB * G::PADN);
    uint32_t* words = cv.take<uint32_t>((size_t)G::SPB * cm.words_per_sym);
    R* red = cv.take<R>(kBlock);
    unsigned long long* redc = cv.take<unsigned long long>(kBlock / 64);

    load_twiddles<R>(tw, (const C*)cm.tw);
    if (threadIdx.x < cm.n_axis) axis[threadIdx.x] = cm.axis[threadIdx.x];
    __syncthreads();

    // a symbol group of >= 64 threads is whole wavefronts: make its index wave-uniform
    const int ls = TPS >= 64 ? __builtin_amdgcn_readfirstlane(threadIdx.x / TPS) : threadIdx.x / TPS;
    const int t = threadIdx.x % TPS;
    C* row = rows + ls * G::PADN;
    uint32_t* W = words + ls * cm.words_per_sym;
    const C* eqa = (const C*)cm.eq_a;
    const R* eqb = (const R*)cm.eq_b;
    const int cp = cm.cp;
    const R scale = (R)cm.scale;
    Slicer<R> slicer;
    if (!adaptive) slicer.load(axis[0]);

    // sigma from the whole-stream mean power (noise/models.py:13-22)
    R sigma = 0;
    if (a.noise_on && !(a.flags & 1)) {
        const double p = a.stats[0] / (double)a.total_samples;
        sigma = (R)sqrt((p / a.snr_lin) / 2.0);
    }
    const bool noise = a.noise_on && !(a.flags & 1);
    const bool array_noise = !FAST && a.nr != nullptr && noise;
    const int64_t niter = (cm.n_sym + G::SPB - 1) / G::SPB;
    unsigned long long be = 0, se = 0;

    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        const int64_t sl = it * G::SPB + ls;
        const int64_t sg = cm.sym0 + sl;
        const bool active = sl < cm.n_sym;
        int base_bit = 0;
        if (active && !(a.flags & 4)) base_bit = stage_words<TPS>(cm, sg, W, t);
        // kept channel samples + AWGN; the 1/sqrt(N) of fft(norm="ortho") folded in
        const C* ys = (const C*)a.y + sl * N;
        C x[E];
#pragma unroll
        for (int i = 0; i < E; ++i)
            x[i] = (active && !(a.flags & 16)) ? ys[t + i * TPS] : mk<R>(0, 0);
        if (active && array_noise) {
            const double* nr = a.nr + sg * (N + cp) + cp;
            const double* ni = a.ni + sg * (N + cp) + cp;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                x[i].re += sigma * (R)nr[t + i * TPS];
                x[i].im += sigma * (R)ni[t + i * TPS];
            }
        } else if (active && noise) {
            // Philox noise: one call = two complex normals, for elements i and i+1
#pragma unroll
            for (int i = 0; i < E; i += 2) {
                float r0, i0, r1, i1;
                philox_noise_pair(cm.seed, sg, (uint32_t)(t + (i >> 1) * TPS), r0, i0, r1, i1);
                x[i].re += sigma * (R)r0;
                x[i].im += sigma * (R)i0;
                if (i + 1 < E) {
                    x[i + 1].re += sigma * (R)r1;
                    x[i + 1].im += sigma * (R)i1;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < E; ++i) x[i] = cscale(x[i], scale);
        if (!(a.flags & 2)) fft_reg<R, LOGN, false>(x, row, tw, tw + 64, t);
        sym_sync<TPS>();  // tx bit words visible to the whole symbol group
        // MMSE noise variance per OFDM symbol (equalization/models.py:39-49)
        R nv = 0;
        if (eq == OFDM_EQ_MMSE) {
            R p = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) p += norm2(x[i]);
            p = group_sum<R, TPS>(p, red);
            nv = cm.gain_mean == 0.0 ? (R)INFINITY : ((p / (R)N) / (R)a.snr_lin) / (R)cm.gain_mean;
        }
        if (active && !(a.flags & 8)) {
            const int64_t sbit = sg * cm.bps;
            const bool all_valid = FAST || sbit + cm.bps <= a.n_valid_bits;
            uint32_t bes = 0, ses = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int k = t + i * TPS;
                C v = x[i];
                if (eq == OFDM_EQ_ZF) {
                    v = cmul(v, eqa[k]);
                } else if (eq == OFDM_EQ_MMSE) {
                    v = cmul(v, mmse_coef<R>(eqa[k], eqb[k], nv));
                }
                if (!FAST && sl < a.z_keep) ((C*)a.z_out)[sl * N + k] = v;
                uint32_t ridx;
                int b, off;
                if (adaptive) {
                    const ScInfo sc = cm.sc[k];
                    if (sc.lut < 0) continue;
                    b = sc.bits;
                    off = sc.bitoff;
                    ridx = slice<R>(v, axis[sc.lut]);
                } else {
                    b = cm.b;
                    off = k * b;
                    ridx = slicer(v);
                }
                uint32_t d = ridx ^ extract_w(W, base_bit + off, b);
                ses += d != 0u;
                if (!all_valid) {
                    const int64_t nvb = a.n_valid_bits - (sbit + off);
                    const int keep = nvb <= 0 ? 0 : (nvb >= b ? b : (int)nvb);
                    d &= ((1u << keep) - 1u) << (b - keep);
                }
                bes += __popc(d);
            }
            be += bes;
            se += ses;
        }
        sym_sync<TPS>();  // W and the FFT row are rewritten by the next symbol
    }
    be = block_sum<unsigned long long>(be, redc);
    se = block_sum<unsigned long long>(se, redc);
    if (threadIdx.x == 0) {
        if (be) atomicAdd((unsigned long long*)&a.counters[0], be);
        if (se) atomicAdd((unsigned long long*)&a.counters[1], se);
    }
}

}  // namespace ofdm
