// ofdm_abi.hip -- C ABI of libofdm_hip.so (include/ofdm_hip.h): plan management,
// argument validation, error reporting, and dispatch to the gfx950 kernels.
//
// A plan owns only constant tables (twiddles, LUTs, normalised CIR, equaliser
// response) and a partial-sum workspace.  All data buffers belong to the caller.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ofdm_hip.h"
#include "ofdm_launch.hpp"

using namespace ofdm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// (kNotInBuild: a dispatch that reached a shape an OFDM_AB_ONLY experiment build does not
// instantiate -- reported as a bad argument naming the build, not as a HIP error)
#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (kAbOnly && _e == kNotInBuild)                                                  \
            return fail(OFDM_E_INVALID, std::string(#expr ": kernel not in this build (an "  \
                                                    "OFDM_AB_ONLY variant instantiates "     \
                                                    "N = 1024..4096 only)"));               \
        if (_e != hipSuccess)                                                              \
            return fail(OFDM_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e));      \
    } while (0)

// H[k] = sum_l h_raw[l] exp(-2 pi i (l k mod N) / N): np.fft.fft(h_raw, N)
// (simulation/models.py:264) as a direct L-tap DFT in double precision.
__global__ void k_taps_dft(const double* h, int L, int N, double* H) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    double re = 0, im = 0;
    for (int l = 0; l < L; ++l) {
        const long long m = ((long long)l * k) % N;
        double s, c;
        sincospi(-2.0 * (double)m / (double)N, &s, &c);
        re += h[2 * l] * c - h[2 * l + 1] * s;
        im += h[2 * l] * s + h[2 * l + 1] * c;
    }
    H[2 * k] = re;
    H[2 * k + 1] = im;
}

// Equaliser tables from H (equalization/models.py:22-63):
//   ZF   : eq_a = 1 / where(H == 0, 1e-10, H)
//   MMSE : eq_a = conj(H), eq_b = |H|^2 (np.abs(H)**2)
// gsum[0] = sum |H|^2 (single block, fixed order).
template <typename R>
__global__ void k_eq_tables(const double* H, int N, int eq, R* eq_a, R* eq_b, double* gsum) {
    __shared__ double red[4];
    double acc = 0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const double hr = H[2 * k], hi = H[2 * k + 1];
        const double a = hypot(hr, hi);
        const double g = a * a;
        acc += g;
        if (eq == OFDM_EQ_ZF) {
            double zr = hr, zi = hi;
            if (hr == 0.0 && hi == 0.0) zr = 1e-10;
            const double d = zr * zr + zi * zi;
            eq_a[2 * k] = (R)(zr / d);
            eq_a[2 * k + 1] = (R)(-zi / d);
        } else {
            eq_a[2 * k] = (R)hr;
            eq_a[2 * k + 1] = (R)(-hi);
        }
        eq_b[k] = (R)g;
    }
    acc = block_sum<double>(acc, red);
    if (threadIdx.x == 0) gsum[0] = acc;
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct ofdm_plan_s {
    int n, logn, cp, prec, eq, L;
    int adaptive, b, bps, n_axis, lut_len, n_active;
    double gain_mean;
    DevBuf tw, ptw, lut, lut64, h, eq_a, eq_b, axis, sc, active, H64;
    double gtap[3][kWinTaps];  // normalised taps in Gauss form (TxArgs::gtap)
    // partial-sum workspaces (3 x kMaxGrid doubles), one per HIP stream the plan has been
    // used on: launches on different streams may run concurrently, and a reduction's
    // partials must not be overwritten by another stream's kernel before k_finalize reads
    // them.  Same-stream launches are ordered, so one record per stream is enough.
    std::mutex ws_mu;
    std::map<void*, DevBuf> ws;
    int has_const, has_channel, separable, zp, single_carrier;
    int upat;  // all LUTs use the reference's square-QAM level -> index patterns (kUPat)
    int psk_m; // the single LUT is the reference's M-PSK (LUT[gray(i)] = exp(2 pi j i / M)), M <= 32
    size_t csize() const { return prec == OFDM_F32 ? 8 : 16; }
};

namespace {

template <typename T>
int upload(DevBuf& d, const T* src, size_t n, hipStream_t s) {
    if (n == 0) return OFDM_OK;
    if (hipMalloc(&d.p, n * sizeof(T)) != hipSuccess) return fail(OFDM_E_ALLOC, "hipMalloc failed");
    HIPCHK(hipMemcpyAsync(d.p, src, n * sizeof(T), hipMemcpyHostToDevice, s));
    return OFDM_OK;
}

// Store complex doubles in the plan precision.
int upload_cpx(DevBuf& d, const std::vector<double>& v, int prec, hipStream_t s) {
    if (prec == OFDM_F64) return upload(d, v.data(), v.size(), s);
    std::vector<float> f(v.begin(), v.end());
    return upload(d, f.data(), f.size(), s);
}

// Decision tables for one LUT.  Square-QAM LUTs as QAMConstellationMapper.generate_constellation
// builds them (constellation/models.py:180-218) are separable: LUT[i] = lev[ki] + j lev[kq] with
// i = (qpat[kq] << b/2) | ipat[ki], which the fused slicer needs.  Any other LUT (PSK, :356-380)
// gets side = 0: the operator map/demap (LUT gather, brute-force NN) still work, the fused path
// refuses the plan.
int build_axis(const double* lut, int m, int lut_off, AxisInfo& ax) {
    int b = 0;
    while ((1 << b) < m) ++b;
    if (m < 2 || m > 256 || (1 << b) != m)
        return fail(OFDM_E_INVALID, "constellation order must be a power of two in [2, 256]");
    memset(&ax, 0, sizeof(ax));
    ax.bits = b;
    ax.lut_off = lut_off;
    ax.side = 0;
    const int side = (int)std::lround(std::sqrt((double)m));
    if (side * side != m || (b & 1)) return OFDM_OK;
    std::vector<double> lev;
    for (int i = 0; i < m; ++i) lev.push_back(lut[2 * i]);
    std::sort(lev.begin(), lev.end());
    lev.erase(std::unique(lev.begin(), lev.end()), lev.end());
    if ((int)lev.size() != side) return OFDM_OK;
    const double inv_step = (side - 1) / (lev[side - 1] - lev[0]);
    std::vector<int> iset(side, -1), qset(side, -1);
    for (int i = 0; i < m; ++i) {
        const int ki = (int)(std::find(lev.begin(), lev.end(), lut[2 * i]) - lev.begin());
        const int kq = (int)(std::find(lev.begin(), lev.end(), lut[2 * i + 1]) - lev.begin());
        if (ki >= side || kq >= side) return OFDM_OK;
        const int lo = i & (side - 1), hi = i >> (b / 2);
        if ((iset[ki] >= 0 && iset[ki] != lo) || (qset[kq] >= 0 && qset[kq] != hi)) return OFDM_OK;
        iset[ki] = lo;
        qset[kq] = hi;
    }
    // uniform level spacing for the rounding slicer
    for (int k = 1; k < side; ++k)
        if (std::fabs((lev[k] - lev[k - 1]) * inv_step - 1.0) > 1e-9) return OFDM_OK;
    ax.lev0 = lev[0];
    ax.inv_step = inv_step;
    ax.side = side;
    ax.hbits = b / 2;
    for (int k = 0; k < side; ++k) {
        ax.ipat[k] = (uint8_t)iset[k];
        ax.qpat[k] = (uint8_t)qset[k];
    }
    return OFDM_OK;
}

// True when every axis maps levels to index bits like the reference's square-QAM LUTs:
// ipat[k] = U[k], qpat[k] = U[side - 1 - k] (ofdm_device.hpp, kUPat), at most 4 LUTs.
bool universal_patterns(const std::vector<AxisInfo>& axes) {
    if (axes.empty() || axes.size() > 4) return false;
    for (const AxisInfo& ax : axes) {
        if (ax.side < 2 || ax.side > 16) return false;
        for (int k = 0; k < ax.side; ++k) {
            const uint32_t u = (kUPat[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            const int kq = ax.side - 1 - k;
            const uint32_t uq = (kUPat[kq >> 2] >> (8 * (kq & 3))) & 0xFFu;
            if (ax.ipat[k] != u || ax.qpat[k] != uq) return false;
        }
    }
    return true;
}

// M if the LUT is the reference's M-PSK (constellation/models.py:356-380: LUT[gray(i)] =
// exp(2 pi j i / M)) with 2 <= M <= 32, else 0.
int psk_order(const double* lut, int m) {
    if (m < 2 || m > 32 || (m & (m - 1))) return 0;
    for (int i = 0; i < m; ++i) {
        const int g = i ^ (i >> 1);
        const double a = 2.0 * M_PI * i / m;
        if (std::fabs(lut[2 * g] - std::cos(a)) > 1e-12 || std::fabs(lut[2 * g + 1] - std::sin(a)) > 1e-12) return 0;
    }
    return m;
}

// Multipath TX: consecutive OFDM symbols per symbol group; the group's first symbol regenerates
// its predecessor's tail (one extra bits + map + IFFT per group).  32 against 16: complex128 TX
// c 5.15 -> 5.00, d 5.24 -> 5.04, e 5.19 -> 5.00 ms per step (profiles/r03ag_ab.txt).  Since each
// launch picks its chunk in [max / 2, max] to fill whole rounds of resident workgroups (tx_chunk),
// 64 (64 against 32: TX d 4.53 -> 4.44 ms, c and e within 0.5 %; 128: d 4.40, c and e 1 % slower
// and the 1e5-symbol sweep points 20 %, profiles/r05n_ab_tx_chunk.txt)
#ifndef OFDM_TX_CHUNK
#define OFDM_TX_CHUNK 64
#endif

#if OFDM_ABLATION
// Diagnostic ablation switches for timing studies (tools/ablate.py), compiled only into
// OFDM_ABLATION builds: the product library has no environment-controlled work skipping.
int env_flags(const char* name) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : 0;
}
#define OFDM_ENV_FLAGS(name) env_flags(name)
#else
#define OFDM_ENV_FLAGS(name) 0
#endif

int log2_exact(int n) {
    int l = 0;
    while ((1 << l) < n) ++l;
    return (1 << l) == n ? l : -1;
}

// 32-bit words of one OFDM symbol's bit stream staged in LDS: the stream plus a <8-bit
// misalignment of the symbol start, one slack word for the 64-bit extraction window,
// rounded up to whole Philox blocks (4 words).
int lds_words_per_sym(int bps) { return (((bps + 7 + 31) / 32 + 1) + 3) & ~3; }

}  // namespace

extern "C" {

int ofdm_abi_version(void) { return OFDM_ABI_VERSION; }

const char* ofdm_last_error(void) { return g_err.c_str(); }

int ofdm_plan_create(ofdm_plan_t* out, const ofdm_desc* d, void* stream) {
    if (!out || !d) return fail(OFDM_E_INVALID, "null argument");
    *out = nullptr;
    hipStream_t s = (hipStream_t)stream;
    const int logn = log2_exact(d->n_fft);
    if (d->n_fft < 1 || d->n_fft > 4096 || logn < 0)
        return fail(OFDM_E_INVALID, "n_fft must be a power of two in [1, 4096]");
    if (d->cp < 0) return fail(OFDM_E_INVALID, "Prefix length must be a non-negative integer.");
    if (d->cp > d->n_fft) return fail(OFDM_E_INVALID, "Input symbols length must be greater than prefix length.");
    if (d->precision != OFDM_F32 && d->precision != OFDM_F64) return fail(OFDM_E_INVALID, "bad precision");
    if (d->equalizer < 0 || d->equalizer > 2) return fail(OFDM_E_INVALID, "bad equalizer");
    if (d->n_taps < 0 || d->n_taps > kMaxTaps) return fail(OFDM_E_INVALID, "n_taps must be in [0, 32]");
    if (d->n_luts < 0 || d->n_luts > kMaxLuts) return fail(OFDM_E_INVALID, "n_luts must be in [0, 8]");

    ofdm_plan_s* p = new ofdm_plan_s();
    std::unique_ptr<ofdm_plan_s> guard(p);
    p->n = d->n_fft;
    p->logn = logn;
    p->cp = d->cp;
    p->prec = d->precision;
    p->eq = d->equalizer;
    p->L = d->n_taps;
    p->gain_mean = 0;
    if (d->prefix != OFDM_PREFIX_CYCLIC && d->prefix != OFDM_PREFIX_ZERO)
        return fail(OFDM_E_INVALID, "bad prefix kind");
    p->zp = d->prefix == OFDM_PREFIX_ZERO;
    if (d->modulator != OFDM_MOD_OFDM && d->modulator != OFDM_MOD_SC) return fail(OFDM_E_INVALID, "bad modulator kind");
    p->single_carrier = d->modulator == OFDM_MOD_SC;
    if (p->zp && p->cp > p->n) return fail(OFDM_E_INVALID, "zero padding needs prefix length <= n_fft");
    p->adaptive = d->sc_lut != nullptr;
    p->has_const = d->n_luts > 0;
    p->has_channel = d->n_taps > 0 || d->H != nullptr;
    int rc;

    // twiddles lo[j] = W_N^j (j < 64), hi[j] = W_N^(64 j)
    {
        std::vector<double> tw(2 * 128, 0.0);
        const double N = (double)p->n;
        for (int j = 0; j < 64; ++j) {
            const double a = -2.0 * M_PI * (double)(j % p->n) / N;
            tw[2 * j] = std::cos(a);
            tw[2 * j + 1] = std::sin(a);
            const long long m = (64LL * j) % p->n;
            const double a2 = -2.0 * M_PI * (double)m / N;
            tw[2 * (64 + j)] = std::cos(a2);
            tw[2 * (64 + j) + 1] = std::sin(a2);
        }
        if ((rc = upload_cpx(p->tw, tw, p->prec, s))) return rc;
    }
    // per-pass twiddle tables of the throughput kernels (ofdm_device.hpp tt_from):
    // [forward | inverse], pass (LOGR, LOGNS > 0): T[(r-1) NS + k] = exp(-+2 pi i k r / (NS RAD)),
    // r = 1 only for compact passes (tt_compact)
    if (p->logn > 4) {
        const int tts = tt_size(p->logn);
        std::vector<double> tt(4 * (size_t)tts, 0.0);
        size_t at = 0;
        for (int logns = 0; logns < p->logn;) {
            const int logr = std::min(4, p->logn - logns);
            const int ns = 1 << logns, rad = 1 << logr;
            if (logns > 0) {
                const int rmax = tt_compact(p->logn, logns) ? 2 : rad;  // compact: W^k only
                for (int r = 1; r < rmax; ++r)
                    for (int k = 0; k < ns; ++k, ++at) {
                        const double a = -2.0 * M_PI * (double)(k * r) / (double)(ns * rad);
                        tt[2 * at] = std::cos(a);
                        tt[2 * at + 1] = std::sin(a);
                        tt[2 * (tts + at)] = std::cos(a);
                        tt[2 * (tts + at) + 1] = -std::sin(a);
                    }
            }
            logns += logr;
        }
        if ((int)at != tts) return fail(OFDM_E_INVALID, "internal: twiddle table size");
        if ((rc = upload_cpx(p->ptw, tt, p->prec, s))) return rc;
    }

    // constellations
    if (p->has_const) {
        std::vector<AxisInfo> axes(d->n_luts);
        int off = 0;
        for (int i = 0; i < d->n_luts; ++i) {
            if ((rc = build_axis(d->lut_pool + 2 * off, d->lut_orders[i], off, axes[i]))) return rc;
            off += d->lut_orders[i];
        }
        if (off > kMaxLut) return fail(OFDM_E_INVALID, "LUT pool too large");
        p->lut_len = off;
        p->n_axis = d->n_luts;
        p->separable = 1;
        for (const AxisInfo& ax : axes) p->separable &= ax.side > 0;
        p->upat = p->separable && universal_patterns(axes);
        p->psk_m = (!p->separable && d->n_luts == 1) ? psk_order(d->lut_pool, d->lut_orders[0]) : 0;
        std::vector<double> pool(d->lut_pool, d->lut_pool + 2 * off);
        if ((rc = upload_cpx(p->lut, pool, p->prec, s))) return rc;
        if ((rc = upload(p->lut64, pool.data(), pool.size(), s))) return rc;
        if ((rc = upload(p->axis, axes.data(), axes.size(), s))) return rc;
        if (p->adaptive) {
            std::vector<ScInfo> sc(p->n);
            std::vector<int32_t> act;
            int bit = 0;
            for (int k = 0; k < p->n; ++k) {
                const int id = d->sc_lut[k];
                if (id < -1 || id >= d->n_luts) return fail(OFDM_E_INVALID, "sc_lut entry out of range");
                sc[k].lut = (int16_t)id;
                sc[k].bits = (int16_t)(id < 0 ? 0 : axes[id].bits);
                sc[k].bitoff = bit;
                bit += sc[k].bits;
                if (id >= 0) act.push_back(k);
            }
            if (bit == 0) return fail(OFDM_E_INVALID, "No active subcarriers (all orders are zero)");
            p->bps = bit;
            p->b = -1;
            p->n_active = (int)act.size();
            if ((rc = upload(p->sc, sc.data(), sc.size(), s))) return rc;
            if ((rc = upload(p->active, act.data(), act.size(), s))) return rc;
        } else {
            if (d->n_luts != 1) return fail(OFDM_E_INVALID, "fixed mode takes exactly one LUT");
            p->b = axes[0].bits;
            p->bps = p->b * p->n;
            p->n_active = p->n;
        }
    } else {
        p->lut_len = 0;
        p->n_axis = 0;
        p->separable = 0;
        p->b = 0;
        p->bps = 0;
        p->n_active = 0;
    }

    // channel: normalised taps for the convolution, H for the equaliser
    if (d->n_taps > 0) {
        double pw = 0;
        for (int l = 0; l < d->n_taps; ++l)
            pw += d->h_raw[2 * l] * d->h_raw[2 * l] + d->h_raw[2 * l + 1] * d->h_raw[2 * l + 1];
        if (pw == 0) return fail(OFDM_E_INVALID, "Impulse response cannot be all zeros.");
        const double sc = std::sqrt(pw);
        std::vector<double> hn(2 * d->n_taps);
        for (int l = 0; l < 2 * d->n_taps; ++l) hn[l] = d->h_raw[l] / sc;
        if ((rc = upload_cpx(p->h, hn, p->prec, s))) return rc;
        for (int l = 0; l < kWinTaps; ++l) {
            const double re = l < d->n_taps ? hn[2 * l] : 0.0, im = l < d->n_taps ? hn[2 * l + 1] : 0.0;
            p->gtap[0][l] = re;
            p->gtap[1][l] = re + im;
            p->gtap[2][l] = im - re;
        }
    }
    if (p->has_channel) {
        if (hipMalloc(&p->H64.p, 16 * (size_t)p->n) != hipSuccess) return fail(OFDM_E_ALLOC, "hipMalloc failed");
        if (d->H) {
            HIPCHK(hipMemcpyAsync(p->H64.p, d->H, 16 * (size_t)p->n, hipMemcpyHostToDevice, s));
        } else {
            DevBuf hr;
            std::vector<double> hv(d->h_raw, d->h_raw + 2 * d->n_taps);
            if ((rc = upload(hr, hv.data(), hv.size(), s))) return rc;
            (void)hipGetLastError();
            hipLaunchKernelGGL(k_taps_dft, dim3((p->n + 255) / 256), dim3(256), 0, s, (const double*)hr.p,
                               d->n_taps, p->n, (double*)p->H64.p);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(s));
        }
        if (hipMalloc(&p->eq_a.p, p->csize() * p->n) != hipSuccess ||
            hipMalloc(&p->eq_b.p, p->csize() / 2 * p->n) != hipSuccess)
            return fail(OFDM_E_ALLOC, "hipMalloc failed");
        DevBuf g;
        if (hipMalloc(&g.p, sizeof(double)) != hipSuccess) return fail(OFDM_E_ALLOC, "hipMalloc failed");
        const int eqk = p->eq == OFDM_EQ_ZF ? OFDM_EQ_ZF : OFDM_EQ_MMSE;
        if (p->prec == OFDM_F32)
            hipLaunchKernelGGL(k_eq_tables<float>, dim3(1), dim3(256), 0, s, (const double*)p->H64.p, p->n, eqk,
                               (float*)p->eq_a.p, (float*)p->eq_b.p, (double*)g.p);
        else
            hipLaunchKernelGGL(k_eq_tables<double>, dim3(1), dim3(256), 0, s, (const double*)p->H64.p, p->n, eqk,
                               (double*)p->eq_a.p, (double*)p->eq_b.p, (double*)g.p);
        HIPCHK(hipGetLastError());
        double gs = 0;
        HIPCHK(hipMemcpyAsync(&gs, g.p, sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        p->gain_mean = gs / p->n;
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = guard.release();
    return OFDM_OK;
}

int ofdm_plan_destroy(ofdm_plan_t plan) {
    delete plan;
    return OFDM_OK;
}

int ofdm_plan_get_info(ofdm_plan_t p, ofdm_plan_info* info) {
    if (!p || !info) return fail(OFDM_E_INVALID, "null argument");
    info->n_fft = p->n;
    info->cp = p->cp;
    info->precision = p->prec;
    info->equalizer = p->eq;
    info->n_taps = p->L;
    info->bits_per_ofdm_symbol = p->bps;
    info->bits_per_subcarrier = p->adaptive ? -1 : p->b;
    info->adaptive = p->adaptive;
    info->channel_gain_mean = p->gain_mean;
    return OFDM_OK;
}

int ofdm_plan_response(ofdm_plan_t p, void* stream, double* H, double* gains) {
    if (!p || !H) return fail(OFDM_E_INVALID, "null argument");
    if (!p->has_channel) return fail(OFDM_E_INVALID, "plan has no channel response");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(H, p->H64.p, 16 * (size_t)p->n, hipMemcpyDeviceToDevice, s));
    if (gains) {
        if (p->prec == OFDM_F64) {
            HIPCHK(hipMemcpyAsync(gains, p->eq_b.p, 8 * (size_t)p->n, hipMemcpyDeviceToDevice, s));
        } else {
            return fail(OFDM_E_INVALID, "gains are exported by float64 plans only");
        }
    }
    return OFDM_OK;
}

#define DISPATCH(p, CALL) ((p)->prec == OFDM_F32 ? CALL(float) : CALL(double))

int ofdm_fft(ofdm_plan_t p, void* stream, void* data, int64_t batch, int32_t inverse) {
    if (!p || (!data && batch > 0) || batch < 0) return fail(OFDM_E_INVALID, "bad argument to ofdm_fft");
    RowsArgs a{};
    a.in = data;
    a.out = data;
    a.n_rows = batch;
    a.in_stride = p->n;
    a.out_stride = p->n;
    a.inverse = inverse != 0;
    a.scale = 1.0 / std::sqrt((double)p->n);
    a.tw = p->tw.p;
#define CALL(R) launch_rows<R>(p->logn, 0, a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_modulate(ofdm_plan_t p, void* stream, const void* X, int64_t n_sym, void* x) {
    if (!p || n_sym < 0 || (n_sym > 0 && (!X || !x))) return fail(OFDM_E_INVALID, "bad argument to ofdm_modulate");
    RowsArgs a{};
    a.in = X;
    a.out = x;
    a.n_rows = n_sym;
    a.in_stride = p->n;
    a.out_stride = p->n + p->cp;
    a.out_cp = p->cp;
    a.zp = p->zp ? p->cp : 0;
    a.scale = 1.0 / std::sqrt((double)p->n);
    a.tw = p->tw.p;
#define CALL(R) launch_rows<R>(p->logn, 1, a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_demodulate(ofdm_plan_t p, void* stream, const void* yt, int64_t n_sym, double snr_db, void* Z) {
    if (!p || n_sym < 0 || (n_sym > 0 && (!yt || !Z))) return fail(OFDM_E_INVALID, "bad argument to ofdm_demodulate");
    if (p->eq != OFDM_EQ_NONE && !p->has_channel) return fail(OFDM_E_INVALID, "plan has no channel response");
    RowsArgs a{};
    a.in = yt;
    a.out = Z;
    a.n_rows = n_sym;
    a.in_stride = p->n + p->cp;
    a.in_off = p->zp ? 0 : p->cp;
    a.zp = p->zp ? p->cp : 0;
    a.out_stride = p->n;
    a.eq = p->eq;
    a.scale = 1.0 / std::sqrt((double)p->n);
    a.snr_lin = std::pow(10.0, snr_db / 10.0);
    a.gain_mean = p->gain_mean;
    a.tw = p->tw.p;
    a.eq_a = p->eq_a.p;
    a.eq_b = p->eq_b.p;
#define CALL(R) launch_rows<R>(p->logn, 2, a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_equalize(ofdm_plan_t p, void* stream, const void* Y, int64_t n_rows, double snr_db, void* Z) {
    if (!p || n_rows < 0 || (n_rows > 0 && (!Y || !Z))) return fail(OFDM_E_INVALID, "bad argument to ofdm_equalize");
    if (p->eq != OFDM_EQ_NONE && !p->has_channel) return fail(OFDM_E_INVALID, "plan has no channel response");
    EqArgs a{};
    a.Y = Y;
    a.Z = Z;
    a.n_rows = n_rows;
    a.n = p->n;
    a.eq = p->eq;
    a.snr_lin = std::pow(10.0, snr_db / 10.0);
    a.gain_mean = p->gain_mean;
    a.eq_a = p->eq_a.p;
    a.eq_b = p->eq_b.p;
#define CALL(R) launch_equalize<R>(a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_map(ofdm_plan_t p, void* stream, const uint8_t* bytes, int64_t n_bytes, int64_t n_out, void* symbols) {
    if (!p || !p->has_const) return fail(OFDM_E_INVALID, "plan has no constellation");
    if (n_bytes < 0 || n_out < 0 || (n_out > 0 && !symbols) || (n_bytes > 0 && !bytes))
        return fail(OFDM_E_INVALID, "bad argument to ofdm_map");
    if (p->adaptive && n_out % p->n) return fail(OFDM_E_INVALID, "adaptive map needs whole OFDM symbols");
    MapArgs a{};
    a.bytes = bytes;
    a.n_bytes = n_bytes;
    a.n_out = n_out;
    a.out = symbols;
    a.lut = p->lut.p;
    a.b = p->b;
    a.adaptive = p->adaptive;
    a.n_fft = p->n;
    a.bps = p->bps;
    a.sc = (const ScInfo*)p->sc.p;
    a.axis = (const AxisInfo*)p->axis.p;
#define CALL(R) launch_map<R>(a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_demap(ofdm_plan_t p, void* stream, const void* z, int64_t n, uint8_t* bytes) {
    if (!p || !p->has_const) return fail(OFDM_E_INVALID, "plan has no constellation");
    if (n < 0 || (n > 0 && (!z || !bytes))) return fail(OFDM_E_INVALID, "bad argument to ofdm_demap");
    DemapArgs a{};
    a.z = z;
    a.bytes = bytes;
    if (p->adaptive) {
        if (n % p->n) return fail(OFDM_E_INVALID, "adaptive demap needs whole OFDM symbols");
        a.total_bits = (n / p->n) * (int64_t)p->bps;
        a.n_bytes = a.total_bits / 8;
    } else {
        a.total_bits = n * (int64_t)p->b;
        a.n_bytes = (a.total_bits + 7) / 8;
    }
    a.b = p->b;
    a.adaptive = p->adaptive;
    a.n_fft = p->n;
    a.bps = p->bps;
    a.n_active = p->n_active;
    a.sc = (const ScInfo*)p->sc.p;
    a.axis = (const AxisInfo*)p->axis.p;
    a.active = (const int32_t*)p->active.p;
    a.lut64 = (const double*)p->lut64.p;
#define CALL(R) launch_demap<R>(a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_demap_count(ofdm_plan_t p, void* stream, const void* Z, const uint8_t* tx_bits, int64_t n_sym,
                     uint64_t* counters) {
    if (!p || !p->has_const) return fail(OFDM_E_INVALID, "plan has no constellation");
    if (n_sym < 0 || (n_sym > 0 && (!Z || !tx_bits || !counters)))
        return fail(OFDM_E_INVALID, "bad argument to ofdm_demap_count");
    DemapCountArgs a{};
    a.z = Z;
    a.tx = tx_bits;
    a.n_sym = n_sym;
    const int64_t total = n_sym * (int64_t)p->bps;
    // the reference compares every bit in FIXED mode, whole bytes in adaptive mode (its decode
    // drops a trailing partial byte, constellation/adaptive.py:259-263)
    a.n_valid_bits = p->adaptive ? (total / 8) * 8 : total;
    a.n_tx_bytes = (total + 7) / 8;
    a.n_fft = p->n;
    a.b = p->b;
    a.bps = p->bps;
    a.adaptive = p->adaptive;
    a.separable = p->separable;
    a.sc = (const ScInfo*)p->sc.p;
    a.axis = (const AxisInfo*)p->axis.p;
    a.lut64 = (const double*)p->lut64.p;
    a.lut_len = p->lut_len;
    a.counters = (unsigned long long*)counters;
#define CALL(R) launch_demap_count<R>(a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

int ofdm_nn_classify(void* stream, const double* lut, int32_t m, const void* z, int64_t n, int64_t* idx) {
    if (m < 1 || n < 0 || !lut || (n > 0 && (!z || !idx))) return fail(OFDM_E_INVALID, "bad argument to ofdm_nn_classify");
    HIPCHK(launch_nn_classify(lut, m, (const double*)z, n, idx, (hipStream_t)stream));
    return OFDM_OK;
}

int ofdm_noise_radius(void* stream, const uint32_t* words, int64_t n, float* radius) {
    if (n < 0 || (n > 0 && (!words || !radius))) return fail(OFDM_E_INVALID, "bad argument to ofdm_noise_radius");
    HIPCHK(launch_noise_radius(words, n, radius, (hipStream_t)stream));
    return OFDM_OK;
}

// The stream's partial-sum workspace (allocated on first use), or nullptr.
static double* workspace(ofdm_plan_t p, void* stream) {
    std::lock_guard<std::mutex> lk(p->ws_mu);
    DevBuf& d = p->ws[stream];
    if (!d.p && hipMalloc(&d.p, sizeof(double) * kTxFields * kMaxGrid) != hipSuccess) {
        d.p = nullptr;
        return nullptr;
    }
    return (double*)d.p;
}

static int reduce_into(ofdm_plan_t p, hipStream_t s, const double* ws, int grid, int nfields, int max_mask,
                       double* stats) {
    HIPCHK(launch_finalize(ws, grid, nfields, max_mask, stats, s));
    return OFDM_OK;
}

int ofdm_channel(ofdm_plan_t p, void* stream, const void* sig, int64_t len, void* y, double* power_sum) {
    if (!p || p->L < 1) return fail(OFDM_E_INVALID, "plan has no channel taps");
    if (len < 0 || (len > 0 && (!sig || !y))) return fail(OFDM_E_INVALID, "bad argument to ofdm_channel");
    if (len == 0) return OFDM_OK;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((len + 255) / 256, kMaxGrid));
    double* ws = workspace(p, stream);
    if (!ws) return fail(OFDM_E_ALLOC, "hipMalloc failed");
    ConvArgs a{sig, y, len, p->h.p, p->L, ws};
#define CALL(R) launch_conv<R>(a, grid, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    if (power_sum) return reduce_into(p, (hipStream_t)stream, ws, grid, 1, 0, power_sum);
    return OFDM_OK;
}

int ofdm_power(ofdm_plan_t p, void* stream, const void* y, int64_t len, double* power_sum) {
    if (!p || len < 0 || (len > 0 && !y) || !power_sum) return fail(OFDM_E_INVALID, "bad argument to ofdm_power");
    if (len == 0) return OFDM_OK;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((len + 255) / 256, kMaxGrid));
    double* ws = workspace(p, stream);
    if (!ws) return fail(OFDM_E_ALLOC, "hipMalloc failed");
    PowerArgs a{y, len, ws};
#define CALL(R) launch_power<R>(a, grid, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return reduce_into(p, (hipStream_t)stream, ws, grid, 1, 0, power_sum);
}

int ofdm_awgn(ofdm_plan_t p, void* stream, void* y, int64_t len, const double* nr, const double* ni,
              const double* power_sum, double snr_db) {
    if (!p || len < 0 || (len > 0 && (!y || !nr || !ni || !power_sum)))
        return fail(OFDM_E_INVALID, "bad argument to ofdm_awgn");
    AwgnArgs a{y, len, nr, ni, power_sum, std::pow(10.0, snr_db / 10.0)};
#define CALL(R) launch_awgn<R>(a, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

static void fill_common(ofdm_plan_t p, TxRxCommon& c, const uint8_t* bits, uint64_t seed, int64_t sym0,
                        int64_t n_sym, int64_t total_syms_for_bits) {
    c.bits = bits;
    c.n_bytes = (total_syms_for_bits * (int64_t)p->bps + 7) / 8;
    c.seed = seed;
    c.sym0 = sym0;
    c.n_sym = n_sym;
    c.tw = p->tw.p;
    c.ptw = p->ptw.p;
    c.lut = p->lut.p;
    c.lut_len = p->lut_len;
    c.axis = (const AxisInfo*)p->axis.p;
    c.n_axis = p->n_axis;
    c.sc = (const ScInfo*)p->sc.p;
    c.adaptive = p->adaptive;
    c.b = p->b;
    c.bps = p->bps;
    c.cp = p->cp;
    c.eq = p->eq;
    c.words_per_sym = lds_words_per_sym(p->bps);
    c.scale = 1.0 / std::sqrt((double)p->n);
    c.gain_mean = p->gain_mean;
    c.eq_a = p->eq_a.p;
    c.eq_b = p->eq_b.p;
    c.scm = p->single_carrier;
    c.zpad = p->zp && p->cp > 0;
    c.nn = !p->separable;
    c.ystride = c.zpad ? p->n + p->cp : p->n;
    c.lut64 = (const double*)p->lut64.p;
    c.upat = p->upat;
    // sector decisions for the reference's M-PSK in throughput mode (device bits) on the throughput
    // kernels; the reference-stream mode and the generic kernel keep the reference's nearest-point
    // search (complex128: the same decisions except on a sector boundary, ~1e-16 relative)
    c.psk_m = bits == nullptr ? p->psk_m : 0;
    for (int q = 0; q < 4; ++q) {
        const double tq = (c.psk_m >= 8 && q < c.psk_m / 8) ? std::tan((q + 0.5) * 2.0 * M_PI / c.psk_m) : 0.0;
        c.psk_tan[q] = (float)tq;
        c.psk_tan64[q] = tq;
    }
}

int ofdm_tx(ofdm_plan_t p, void* stream, const uint8_t* bits, uint64_t seed, int64_t sym0, int64_t n_sym,
            void* y, ofdm_stats* stats) {
    if (!p || !p->has_const || p->L < 1) return fail(OFDM_E_INVALID, "ofdm_tx needs a constellation and channel taps");
    if (p->L - 1 > p->n) return fail(OFDM_E_INVALID, "fused path needs channel order <= n_fft");
    if (n_sym < 0 || sym0 < 0 || !stats) return fail(OFDM_E_INVALID, "bad argument to ofdm_tx");
    if (n_sym == 0) return OFDM_OK;
    TxArgs a{};
    // the bits buffer covers global symbols [0, sym0 + n_sym)
    fill_common(p, a.c, bits, seed, sym0, n_sym, sym0 + n_sym);
    a.y = y;
    a.partials = workspace(p, stream);
    if (!a.partials) return fail(OFDM_E_ALLOC, "hipMalloc failed");
    a.h = p->h.p;
    a.L = p->L;
    std::memcpy(a.gtap, p->gtap, sizeof a.gtap);
    a.chunk = p->L > 1 ? OFDM_TX_CHUNK : 1;
    a.slot = tx_slot(p->logn, p->cp, p->L);
    a.flags = OFDM_ENV_FLAGS("OFDM_ABLATE_TX");
    int grid = 0;  // chosen by the launcher with the kernel (<= kMaxGrid partial records)
#define CALL(R) launch_tx<R>(p->logn, a, &grid, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    HIPCHK(launch_finalize_tx(a.partials, grid, (double*)stats, (hipStream_t)stream));
    return OFDM_OK;
}

int ofdm_rx(ofdm_plan_t p, void* stream, const void* y, const double* nr, const double* ni, uint64_t seed,
            const ofdm_stats* stats, int64_t total_samples, double snr_db, int32_t noise_on, const uint8_t* bits,
            int64_t sym0, int64_t n_sym, int64_t n_valid_bits, uint64_t* counters, void* z_out,
            int64_t z_keep) {
    if (!p || !p->has_const) return fail(OFDM_E_INVALID, "ofdm_rx needs a constellation");
    if (p->eq != OFDM_EQ_NONE && !p->has_channel) return fail(OFDM_E_INVALID, "plan has no channel response");
    if (n_sym < 0 || sym0 < 0 || !counters) return fail(OFDM_E_INVALID, "bad argument to ofdm_rx");
    if (n_sym == 0) return OFDM_OK;  // an empty run (its stream has no samples and no noise power)
    if (!y || (noise_on && (!stats || total_samples <= 0))) return fail(OFDM_E_INVALID, "bad argument to ofdm_rx");
    if ((nr == nullptr) != (ni == nullptr)) return fail(OFDM_E_INVALID, "nr and ni must both be given or both NULL");
    RxArgs a{};
    fill_common(p, a.c, bits, seed, sym0, n_sym, sym0 + n_sym);
    a.y = y;
    a.nr = nr;
    a.ni = ni;
    a.stats = (const double*)stats;
    a.total_samples = total_samples;
    a.snr_lin = std::pow(10.0, snr_db / 10.0);
    a.noise_on = noise_on;
    a.n_valid_bits = n_valid_bits;
    a.counters = counters;
    a.z_out = z_out;
    a.z_keep = z_out ? z_keep : 0;
    a.flags = OFDM_ENV_FLAGS("OFDM_ABLATE_RX");
    int grid = 0;
#define CALL(R) launch_rx<R>(p->logn, a, &grid, (hipStream_t)stream)
    HIPCHK(DISPATCH(p, CALL));
#undef CALL
    return OFDM_OK;
}

}  // extern "C"
