// ofdm_kernels.hpp -- gfx950 kernels for the OFDM modem path (templated on the
// real type R = float | double and on log2 N).  Instantiated per precision in
// ofdm_kernels_f32.hip / ofdm_kernels_f64.hip, launched from ofdm_abi.hip.
//
// Hot path (Simulation.run, simulation/models.py:454-606) = two fused kernels:
//   k_tx : bits -> LUT map -> IFFT(ortho) -> cyclic prefix -> L-tap FIR across symbol
//          boundaries -> kept channel samples to HBM + sum|y|^2 / PAPR partials
//   k_rx : HBM samples + AWGN -> FFT(ortho) -> ZF/MMSE -> slicer -> XOR/popcount
//          against the tx bits -> u64 error counters
// Everything between the two HBM touches of y lives in LDS/registers.
#pragma once

#include "ofdm_device.hpp"
#include "ofdm_launch.hpp"

namespace ofdm {

// LDS carve helper: 16-byte aligned bump allocator over the dynamic LDS region.
struct Carve {
    unsigned char* p;
    __device__ explicit Carve(unsigned char* base) : p(base) {}
    template <typename T>
    __device__ T* take(size_t n) {
        T* r = reinterpret_cast<T*>(p);
        p += (n * sizeof(T) + 15) & ~size_t(15);
        return r;
    }
};

extern __shared__ __attribute__((aligned(16))) unsigned char ofdm_smem[];

// ============================================================ operator rows kernel
// One workgroup iteration = SPB rows of N.  MODE: 0 = FFT (in place), 1 = modulate
// (inverse FFT + cyclic prefix), 2 = demodulate (strip prefix, forward FFT, equalise).
template <typename R, int LOGN, int MODE>
__global__ __launch_bounds__(kBlock) void k_rows(RowsArgs a) {
    using G = Geo<LOGN>;
    using C = cpx<R>;
    Carve cv(ofdm_smem);
    C* tw = cv.take<C>(128);
    C* data = cv.take<C>((size_t)G::SPB * G::PADN);
    R* rowscale = cv.take<R>(G::SPB);
    R* red = cv.take<R>(kBlock);
    load_twiddles<R>(tw, (const C*)a.tw);
    __syncthreads();

    const C* in = (const C*)a.in;
    C* out = (C*)a.out;
    const bool inv = MODE == 1 || (MODE == 0 && a.inverse);
    const int ls = threadIdx.x / G::TPS, t = threadIdx.x % G::TPS;
    const R scale = (R)a.scale;
    const int64_t ngroups = (a.n_rows + G::SPB - 1) / G::SPB;
    for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        const int64_t row0 = g * G::SPB;
        // cooperative, coalesced load of SPB rows
#pragma unroll
        for (int j = 0; j < G::E; ++j) {
            const int e = threadIdx.x + j * kBlock;
            const int rl = e >> LOGN, k = e & (G::N - 1);
            const int64_t row = row0 + rl;
            C v = mk<R>(0, 0);
            if (row < a.n_rows) {
                const C* r = in + row * a.in_stride + a.in_off;
                v = r[k];
                if (MODE == 2 && k < a.zp) v = v + r[G::N + k];  // ZP overlap-add
                v = cscale(v, scale);
            }
            data[rl * G::PADN + pad(k)] = v;
        }
        __syncthreads();
        C* buf = data + ls * G::PADN;
        if (inv)
            fft_passes<R, LOGN, 0, true>(buf, tw, tw + 64, t);
        else
            fft_passes<R, LOGN, 0, false>(buf, tw, tw + 64, t);
        if (MODE == 2 && a.eq == OFDM_EQ_MMSE) {
            R p = 0;
#pragma unroll
            for (int i = 0; i < G::E; ++i) p += norm2(buf[pad(t + i * G::TPS)]);
            p = group_sum<R, G::TPS>(p, red);
            if (t == 0) {
                const R sp = p / (R)G::N;
                rowscale[ls] = a.gain_mean == 0.0 ? (R)INFINITY : (sp / (R)a.snr_lin) / (R)a.gain_mean;
            }
            __syncthreads();
        }
        const int olen = G::N + a.out_cp;
        for (int e = threadIdx.x; e < G::SPB * olen; e += kBlock) {
            const int rl = e / olen, m = e - rl * olen;
            const int64_t row = row0 + rl;
            if (row >= a.n_rows) continue;
            C v;
            if (MODE == 1 && a.zp) {
                v = m < G::N ? data[rl * G::PADN + pad(m)] : mk<R>(0, 0);
            } else {
                const int k = m < a.out_cp ? G::N - a.out_cp + m : m - a.out_cp;
                v = data[rl * G::PADN + pad(k)];
            }
            const int k = m < a.out_cp ? 0 : m - a.out_cp;  // subcarrier (MODE 2: out_cp = 0)
            if (MODE == 2) {
                if (a.eq == OFDM_EQ_ZF) {
                    v = cmul(v, ((const C*)a.eq_a)[k]);
                } else if (a.eq == OFDM_EQ_MMSE) {
                    const C hc = ((const C*)a.eq_a)[k];
                    const R d = ((const R*)a.eq_b)[k] + rowscale[rl];
                    v = cmul(v, mk<R>(hc.re / d, hc.im / d));
                }
            }
            out[row * a.out_stride + m] = v;
        }
        __syncthreads();
    }
}

// ============================================================ equalise rows (no FFT)
template <typename R>
__global__ __launch_bounds__(kBlock) void k_equalize(EqArgs a) {
    using C = cpx<R>;
    __shared__ R red[kBlock / 64];
    const C* Y = (const C*)a.Y;
    C* Z = (C*)a.Z;
    for (int64_t row = blockIdx.x; row < a.n_rows; row += gridDim.x) {
        R nv = 0;
        if (a.eq == OFDM_EQ_MMSE) {
            R p = 0;
            for (int k = threadIdx.x; k < a.n; k += kBlock) p += norm2(Y[row * a.n + k]);
            p = block_sum<R>(p, red);
            if (threadIdx.x == 0) red[0] = p;
            __syncthreads();
            p = red[0];
            __syncthreads();
            nv = a.gain_mean == 0.0 ? (R)INFINITY : ((p / (R)a.n) / (R)a.snr_lin) / (R)a.gain_mean;
        }
        for (int k = threadIdx.x; k < a.n; k += kBlock) {
            C v = Y[row * a.n + k];
            if (a.eq == OFDM_EQ_ZF) {
                v = cmul(v, ((const C*)a.eq_a)[k]);
            } else if (a.eq == OFDM_EQ_MMSE) {
                const C hc = ((const C*)a.eq_a)[k];
                const R d = ((const R*)a.eq_b)[k] + nv;
                v = cmul(v, mk<R>(hc.re / d, hc.im / d));
            }
            Z[row * a.n + k] = v;
        }
    }
}

// ============================================================ constellation map (encode)
template <typename R>
__global__ __launch_bounds__(kBlock) void k_map(MapArgs a) {
    using C = cpx<R>;
    const C* lut = (const C*)a.lut;
    C* out = (C*)a.out;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < a.n_out; e += stride) {
        int64_t o;
        int b, lutoff;
        if (a.adaptive) {
            const int64_t s = e / a.n_fft;
            const int k = (int)(e - s * a.n_fft);
            const ScInfo sc = a.sc[k];
            if (sc.lut < 0) {
                out[e] = mk<R>(0, 0);
                continue;
            }
            o = s * a.bps + sc.bitoff;
            b = sc.bits;
            lutoff = a.axis[sc.lut].lut_off;
        } else {
            o = e * a.b;
            b = a.b;
            lutoff = 0;
        }
        // bits past the input read as zero (encode zero-pads, constellation/models.py:235-237)
        uint32_t idx = 0;
        for (int i = 0; i < b; ++i) {
            const int64_t p = o + i;
            const int64_t B = p >> 3;
            const uint32_t bit = B < a.n_bytes ? (a.bytes[B] >> (7 - (int)(p & 7))) & 1u : 0u;
            idx = (idx << 1) | bit;
        }
        out[e] = lut[lutoff + idx];
    }
}

// ============================================================ brute-force NN (decode)
// argmin_m |z - C_m| with np.abs semantics (hypot), first index on ties
// (NNClassifier.classify, constellation/models.py:19-27).
__device__ __forceinline__ int nn_index(double zr, double zi, const double* lut, int m) {
    int best = 0;
    double bd = hypot(zr - lut[0], zi - lut[1]);
    for (int i = 1; i < m; ++i) {
        const double d = hypot(zr - lut[2 * i], zi - lut[2 * i + 1]);
        if (d < bd) {
            bd = d;
            best = i;
        }
    }
    return best;
}

// decode: one thread per output byte; each element's NN index is recomputed by every
// byte it touches.  Fixed mode: element e owns bits [e*b, e*b+b).  Adaptive mode:
// element (s, k) owns bits [s*bps + off_k, +b_k) (constellation/adaptive.py:236-255).
template <typename R>
__global__ __launch_bounds__(kBlock) void k_demap(DemapArgs a) {
    using C = cpx<R>;
    const C* z = (const C*)a.z;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t B = (int64_t)blockIdx.x * kBlock + threadIdx.x; B < a.n_bytes; B += stride) {
        uint32_t byte = 0;
        const int64_t p0 = B * 8;
        int64_t cur_e = -1;
        uint32_t cur_idx = 0;
        int cur_b = 0;
        int64_t cur_o = 0;
        for (int i = 0; i < 8; ++i) {
            const int64_t p = p0 + i;
            uint32_t bit = 0;
            if (p < a.total_bits) {
                int64_t e;
                if (a.adaptive) {
                    const int64_t s = p / a.bps;
                    const int r = (int)(p - s * a.bps);
                    // subcarrier holding stream bit r (binary search over bit offsets)
                    int lo = 0, hi = a.n_active - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (a.sc[a.active[mid]].bitoff <= r) lo = mid; else hi = mid - 1;
                    }
                    e = s * a.n_fft + a.active[lo];
                } else {
                    e = p / a.b;
                }
                if (e != cur_e) {
                    cur_e = e;
                    int lutoff, m;
                    if (a.adaptive) {
                        const int k = (int)(e % a.n_fft);
                        const ScInfo sc = a.sc[k];
                        lutoff = a.axis[sc.lut].lut_off;
                        m = 1 << sc.bits;
                        cur_b = sc.bits;
                        cur_o = (e / a.n_fft) * a.bps + sc.bitoff;
                    } else {
                        lutoff = 0;
                        m = 1 << a.b;
                        cur_b = a.b;
                        cur_o = e * a.b;
                    }
                    const C v = z[e];
                    cur_idx = (uint32_t)nn_index((double)v.re, (double)v.im, a.lut64 + 2 * lutoff, m);
                }
                const int pos = (int)(p - cur_o);
                bit = (cur_idx >> (cur_b - 1 - pos)) & 1u;
            }
            byte = (byte << 1) | bit;
        }
        a.bytes[B] = (uint8_t)byte;
    }
}

// ============================================================ decode + error count
// QAMConstellationMapper.decode (constellation/models.py:251-295) / AdaptiveConstellationMapper.decode
// (constellation/adaptive.py:203-265) followed by Simulation.run's comparison against the tx bits
// (simulation/models.py:596-606), fused: one thread per (symbol, subcarrier) decides the nearest
// point (per-axis slicer for the separable square-QAM LUTs, brute-force |z - C_m| with the first
// index on ties otherwise), XORs its index with the tx bits and counts; counters[0] += bit errors
// over stream bits < n_valid_bits, counters[1] += symbol errors (index mismatches).
template <typename R>
__global__ __launch_bounds__(kBlock) void k_demap_count(DemapCountArgs a) {
    using C = cpx<R>;
    __shared__ unsigned long long red[kBlock / 64];
    const C* z = (const C*)a.z;
    const int64_t n = a.n_sym * a.n_fft;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    unsigned long long be = 0, se = 0;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
        const int64_t s = e / a.n_fft;
        const int k = (int)(e - s * a.n_fft);
        int b, off, lut;
        if (a.adaptive) {
            const ScInfo sc = a.sc[k];
            if (sc.lut < 0) continue;  // unused subcarrier: 0+0j on both sides
            b = sc.bits;
            off = sc.bitoff;
            lut = sc.lut;
        } else {
            b = a.b;
            off = k * a.b;
            lut = 0;
        }
        const C v = z[e];
        const AxisInfo& ax = a.axis[lut];
        const uint32_t ridx = a.separable ? slice<R>(v, ax)
                                          : (uint32_t)nn_index((double)v.re, (double)v.im, a.lut64 + 2 * ax.lut_off, 1 << b);
        const int64_t o = s * (int64_t)a.bps + off;
        uint32_t t = 0;
        for (int i = 0; i < b; ++i) {
            const int64_t p = o + i;
            const int64_t B = p >> 3;
            t = (t << 1) | (B < a.n_tx_bytes ? (a.tx[B] >> (7 - (int)(p & 7))) & 1u : 0u);
        }
        uint32_t d = ridx ^ t;
        se += d != 0u;
        const int64_t nvb = a.n_valid_bits - o;
        const int keep = nvb <= 0 ? 0 : (nvb >= b ? b : (int)nvb);
        d &= ((1u << keep) - 1u) << (b - keep);
        be += __popc(d);
    }
    be = block_sum<unsigned long long>(be, red);
    se = block_sum<unsigned long long>(se, red);
    if (threadIdx.x == 0) {
        if (be) atomicAdd(&a.counters[0], be);
        if (se) atomicAdd(&a.counters[1], se);
    }
}

// ============================================================ channel convolution
// y[n] = sum_l h[l] s[n-l] (s[<0] = 0), truncated to len (channel/models.py:52-55);
// per-block sum |y|^2 into partials.
template <typename R>
__global__ __launch_bounds__(kBlock) void k_conv(ConvArgs a) {
    using C = cpx<R>;
    __shared__ double red[kBlock / 64];
    const C* s = (const C*)a.s;
    const C* h = (const C*)a.h;
    C* y = (C*)a.y;
    double acc = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x; n < a.len; n += stride) {
        C v = mk<R>(0, 0);
        for (int l = 0; l < a.L; ++l) {
            if (n - l < 0) break;
            v = v + cmul(h[l], s[n - l]);
        }
        y[n] = v;
        acc += (double)norm2(v);
    }
    acc = block_sum<double>(acc, red);
    if (threadIdx.x == 0) a.partials[blockIdx.x] = acc;
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_power(PowerArgs a) {
    using C = cpx<R>;
    __shared__ double red[kBlock / 64];
    const C* y = (const C*)a.y;
    double acc = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x; n < a.len; n += stride)
        acc += (double)norm2(y[n]);
    acc = block_sum<double>(acc, red);
    if (threadIdx.x == 0) a.partials[blockIdx.x] = acc;
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_awgn(AwgnArgs a) {
    using C = cpx<R>;
    C* y = (C*)a.y;
    const double p = *a.power_sum / (double)a.len;
    const double sigma = sqrt((p / a.snr_lin) / 2.0);
    const R sg = (R)sigma;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x; n < a.len; n += stride) {
        C v = y[n];
        v.re += sg * (R)a.nr[n];
        v.im += sg * (R)a.ni[n];
        y[n] = v;
    }
}

#ifdef OFDM_SUPPORT_KERNELS
// Deterministic fixed-order reduction of per-block partials: stats[j] += / max= ...
// field f is a max when bit f of max_mask is set, else a sum.
__global__ __launch_bounds__(kBlock) void k_finalize(const double* partials, int nblocks, int nfields,
                                                     int max_mask, double* stats) {
    __shared__ double red[kBlock / 64];
    for (int f = 0; f < nfields; ++f) {
        const int op = (max_mask >> f) & 1;
        double v = 0.0;
        for (int i = threadIdx.x; i < nblocks; i += kBlock) {
            const double x = partials[(int64_t)i * nfields + f];
            v = op == 1 ? (x > v ? x : v) : v + x;
        }
        v = op == 1 ? block_max<double>(v, red) : block_sum<double>(v, red);
        if (threadIdx.x == 0) stats[f] = op == 1 ? (v > stats[f] ? v : stats[f]) : stats[f] + v;
        __syncthreads();
    }
}

// Fused-TX partials -> ofdm_stats: the fixed-point power limbs are summed as integers (exact, any
// order), normalised and added to the record's limbs; power_sum is recomputed from them
// (fx_value), so it depends only on the integer total.  sum |x|^2 (fixed order) and max |x|^2 as
// k_finalize.
__global__ __launch_bounds__(kBlock) void k_finalize_tx(const double* partials, int nblocks, double* stats) {
    __shared__ double red[kBlock / 64];
    const unsigned long long* pu = (const unsigned long long*)partials;
    unsigned long long q0 = 0, q1 = 0;
    double px = 0, mx = 0;
    for (int i = threadIdx.x; i < nblocks; i += kBlock) {
        q0 += pu[(size_t)i * kTxFields + 0];
        q1 += pu[(size_t)i * kTxFields + 1];
        px += partials[(size_t)i * kTxFields + 2];
        mx = fmax(mx, partials[(size_t)i * kTxFields + 3]);
    }
    q0 = block_sum<unsigned long long>(q0, (unsigned long long*)red);
    q1 = block_sum<unsigned long long>(q1, (unsigned long long*)red);
    px = block_sum<double>(px, red);
    mx = block_max<double>(mx, red);
    if (threadIdx.x == 0) {
        unsigned long long* limb = (unsigned long long*)(stats + 3);
        unsigned long long l0 = limb[0] + q0, l1 = limb[1] + q1;
        fx_normalize(l0, l1);
        limb[0] = l0;
        limb[1] = l1;
        stats[0] = fx_value(l0, l1);
        stats[1] += px;
        stats[2] = fmax(stats[2], mx);
    }
}

__global__ __launch_bounds__(kBlock) void k_nn_classify(const double* lut, int m, const double* z,
                                                        int64_t n, int64_t* idx) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride)
        idx[e] = nn_index(z[2 * e], z[2 * e + 1], lut, m);
}

// The throughput-mode noise radius of each word (noise_radius: the fused receivers' float32
// hardware log2 / sqrt, the one operation of the stream definition that is not IEEE-specified),
// for the checker (ofdm_noise_radius).
__global__ __launch_bounds__(kBlock) void k_noise_radius(const uint32_t* w, int64_t n, float* r) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) r[e] = noise_radius(w[e]);
}

#endif  // OFDM_SUPPORT_KERNELS

}  // namespace ofdm

#include "ofdm_fused.hpp"
