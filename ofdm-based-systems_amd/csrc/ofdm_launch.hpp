// ofdm_launch.hpp -- POD kernel argument blocks shared by host (ofdm_abi.hip) and
// device (ofdm_kernels.hpp), plus the per-precision launcher entry points.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ofdm_device.hpp"
#include "ofdm_hip.h"

// Diagnostic ablation switches (timing studies: tools/ablate.py, tools/power_probe.py) exist only in
// builds made with `make VARIANT=ablate EXTRA=-DOFDM_ABLATION=1`; the product library compiles
// every switch out of the kernels and never reads OFDM_ABLATE_TX / OFDM_ABLATE_RX.
#ifndef OFDM_ABLATION
#define OFDM_ABLATION 0
#endif

namespace ofdm {

__host__ __device__ constexpr int ablation_flags(int f) { return OFDM_ABLATION ? f : 0; }

constexpr int kMaxGrid = 4096;  // partial-sum workspace rows
// fused TX partials per workgroup: sum |y|^2 as fixed-point limbs (2 x u64), sum |x|^2, max |x|^2
constexpr int kTxFields = 4;
constexpr int kMaxTaps = 32;
constexpr int kWinTaps = 8;  // taps of the register-window FIR (LT = 4 / 8)
constexpr int kMaxLut = 512;
// LUTs per plan: adaptive loading uses one per distinct order (PSK: 2 .. 256, eight orders)
constexpr int kMaxLuts = 8;

struct RowsArgs {
    const void* in;
    void* out;
    int64_t n_rows, in_stride, out_stride;
    int in_off, out_cp, inverse, eq;
    int zp;  // zero-padding length: modulate appends zeros, demodulate folds the tail (overlap-add)
    double scale, snr_lin, gain_mean;
    const void* tw;
    const void* eq_a;
    const void* eq_b;
};

struct EqArgs {
    const void* Y;
    void* Z;
    int64_t n_rows;
    int n, eq;
    double snr_lin, gain_mean;
    const void* eq_a;
    const void* eq_b;
};

struct MapArgs {
    const uint8_t* bytes;
    int64_t n_bytes, n_out;
    void* out;
    const void* lut;
    int b, adaptive, n_fft, bps;
    const ScInfo* sc;
    const AxisInfo* axis;
};

struct DemapArgs {
    const void* z;
    uint8_t* bytes;
    int64_t n_bytes, total_bits;
    int b, adaptive, n_fft, bps, n_active;
    const ScInfo* sc;
    const AxisInfo* axis;
    const int32_t* active;
    const double* lut64;
};

struct DemapCountArgs {
    const void* z;            // (n_sym, N) equalised symbols
    const uint8_t* tx;        // packed tx bits, OFDM symbol s at bit s * bps
    int64_t n_sym, n_valid_bits, n_tx_bytes;
    int n_fft, b, bps, adaptive, separable;
    const ScInfo* sc;
    const AxisInfo* axis;
    const double* lut64;
    int lut_len;
    unsigned long long* counters;
};

struct ConvArgs {
    const void* s;
    void* y;
    int64_t len;
    const void* h;
    int L;
    double* partials;
};

struct PowerArgs {
    const void* y;
    int64_t len;
    double* partials;
};

struct AwgnArgs {
    void* y;
    int64_t len;
    const double* nr;
    const double* ni;
    const double* power_sum;
    double snr_lin;
};

struct TxRxCommon {
    const uint8_t* bits;
    int64_t n_bytes;
    uint64_t seed;
    int64_t sym0, n_sym;
    const void* tw;
    const void* ptw;  // per-pass twiddle tables [forward | inverse], tt_size(logn) each
    const void* lut;
    int lut_len;
    const AxisInfo* axis;
    int n_axis;
    const ScInfo* sc;
    int adaptive, b, bps, cp, eq;
    int words_per_sym;  // LDS words staged per OFDM symbol (stream + misalignment + slack)
    double scale, gain_mean;
    const void* eq_a;
    const void* eq_b;
    // generic-kernel variants: single-carrier OFDM, zero-padding guard,
    // nearest-point decisions over the double LUT for non-separable constellations (PSK)
    int scm, zpad, nn;
    int ystride;  // stored channel samples per OFDM symbol: N, or N + cp with zero padding
    const double* lut64;
    int upat;  // every LUT has the reference's square-QAM level patterns (kUPat): adaptive fast path
    int psk_m;          // > 0: the single LUT is the reference's M-PSK (M <= 32): sector decisions
    float psk_tan[4];   // tan((q + 1/2) 2 pi / M), q < M / 8 (complex64)
    double psk_tan64[4];  // the same in double (complex128)
};

struct TxArgs {
    TxRxCommon c;
    void* y;
    double* partials;
    const void* h;
    int L;
    int chunk;
    int slot;   // complex elements per symbol row in LDS
    int flags;  // diagnostic ablation (OFDM_ABLATION builds, OFDM_ABLATE_TX): 1 no bit staging, 2 no FFT,
                // 4 no y store
    // complex128 window FIR: the first kWinTaps taps in Gauss form (re, re + im, im - re), read
    // from the kernel arguments into scalar registers (the taps are wave-uniform)
    double gtap[3][kWinTaps];
};

struct RxArgs {
    TxRxCommon c;
    const void* y;
    const double* nr;
    const double* ni;
    const double* stats;
    int64_t total_samples;
    double snr_lin;
    int noise_on;
    int64_t n_valid_bits;
    uint64_t* counters;
    void* z_out;
    int64_t z_keep;
    int flags;  // diagnostic ablation (OFDM_ABLATION builds, OFDM_ABLATE_RX): 1 no noise, 2 no FFT, 4 no bit staging,
                // 8 no equalise/demap/compare, 16 no y load
};

// ---- LDS footprints (must mirror the Carve sequences in ofdm_kernels.hpp)
inline size_t rnd16(size_t n) { return (n + 15) & ~size_t(15); }
inline int geo_spb(int logn, int blk = 256) {
    const int loge = logn < 4 ? logn : 4;
    return blk / ((1 << logn) >> loge);
}
inline int geo_padn(int logn) { return (1 << logn) + ((1 << logn) >> 4); }

template <typename R>
inline size_t smem_rows(int logn) {
    const size_t c = 2 * sizeof(R);
    const int spb = geo_spb(logn);
    return rnd16(128 * c) + rnd16((size_t)spb * geo_padn(logn) * c) + rnd16(spb * sizeof(R)) +
           rnd16(256 * sizeof(R));
}
inline int tx_slot(int logn, int cp, int L) {
    const int ext = (1 << logn) + cp + (L > 1 ? L - 1 : 0);
    return geo_padn(logn) > ext ? geo_padn(logn) : ext;
}
// fused kernels, blk threads; tts = per-pass twiddle entries (0: the two-level table instead);
// fast = throughput kernel (no staged bit words); row_real = rows of reals (complex128
// throughput kernels, fft_reg_split) instead of complex rows
template <typename R>
inline size_t smem_tx(int logn, int blk, int lut_len, int wps, int L, int slot, int tts, bool wfir,
                      size_t extra /* adaptive throughput kernel: per-subcarrier table */, bool fast, bool row_real) {
    const size_t c = 2 * sizeof(R);
    const int spb = geo_spb(logn, blk);
    const int tls = L > 1 ? L - 1 : 1;
    if (fast) wps = 0;
    return rnd16((tts > 0 ? 0 : 128) * c) + rnd16((size_t)lut_len * c) + rnd16(32 * c) + rnd16(wfir ? 32 * c : 0) +
           rnd16(kMaxLuts * sizeof(AxisInfo)) +
           rnd16((size_t)spb * slot * (row_real ? sizeof(R) : c)) + rnd16((size_t)spb * tls * c) +
           rnd16((size_t)spb * wps * 4) + rnd16((size_t)(blk / 64) * sizeof(double)) + rnd16((size_t)tts * c) +
           rnd16(extra);
}
template <typename R>
inline size_t smem_rx(int logn, int blk, int wps, int tts, size_t extra /* adaptive: order table */, bool fast,
                      bool row_real) {
    const size_t c = 2 * sizeof(R);
    const int spb = geo_spb(logn, blk);
    if (fast) wps = 0;
    return rnd16((tts > 0 ? 0 : 128) * c) + rnd16(kMaxLuts * sizeof(AxisInfo)) +
           rnd16((size_t)spb * geo_padn(logn) * (row_real ? sizeof(R) : c)) + rnd16((size_t)spb * wps * 4) +
           rnd16((size_t)(blk / 64) * sizeof(R)) + rnd16((size_t)(blk / 64) * sizeof(unsigned long long)) +
           rnd16((size_t)tts * c) + rnd16(extra);
}

// A launcher's answer for a shape its build does not instantiate (OFDM_AB_ONLY experiment builds:
// N = 1024..4096 only); the ABI reports it as OFDM_E_INVALID "kernel not in this build".  Product
// builds instantiate every shape a plan accepts and never return it.
#ifdef OFDM_AB_ONLY
constexpr bool kAbOnly = true;
#else
constexpr bool kAbOnly = false;
#endif
constexpr hipError_t kNotInBuild = hipErrorNotSupported;  // (only ever meant so when kAbOnly)

// ---- launchers (instantiated for float and double in ofdm_kernels_f{32,64}.hip)
template <typename R>
hipError_t launch_rows(int logn, int mode, const RowsArgs& a, hipStream_t s);
template <typename R>
hipError_t launch_equalize(const EqArgs& a, hipStream_t s);
template <typename R>
hipError_t launch_map(const MapArgs& a, hipStream_t s);
template <typename R>
hipError_t launch_demap(const DemapArgs& a, hipStream_t s);
template <typename R>
hipError_t launch_demap_count(const DemapCountArgs& a, hipStream_t s);
template <typename R>
hipError_t launch_conv(const ConvArgs& a, int grid, hipStream_t s);
template <typename R>
hipError_t launch_power(const PowerArgs& a, int grid, hipStream_t s);
template <typename R>
hipError_t launch_awgn(const AwgnArgs& a, hipStream_t s);
// the fused launchers pick the kernel (and its workgroup size) and return the grid used
template <typename R>
hipError_t launch_tx(int logn, const TxArgs& a, int* grid, hipStream_t s);
template <typename R>
hipError_t launch_rx(int logn, const RxArgs& a, int* grid, hipStream_t s);

hipError_t launch_finalize(const double* partials, int nblocks, int nfields, int max_mask,
                           double* stats, hipStream_t s);
// the fused TX's partials into an ofdm_stats record (exact fixed-point power, ofdm_hip.h)
hipError_t launch_finalize_tx(const double* partials, int nblocks, double* stats, hipStream_t s);
hipError_t launch_nn_classify(const double* lut, int m, const double* z, int64_t n, int64_t* idx,
                              hipStream_t s);
hipError_t launch_noise_radius(const uint32_t* w, int64_t n, float* r, hipStream_t s);

}  // namespace ofdm
