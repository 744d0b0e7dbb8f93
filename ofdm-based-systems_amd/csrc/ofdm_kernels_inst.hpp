// ofdm_kernels_inst.hpp -- launcher definitions; included once per precision by
// ofdm_kernels_f32.hip / ofdm_kernels_f64.hip (explicit instantiation at the end of
// each), so the two precisions compile in parallel.
#pragma once

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

#include "ofdm_kernels.hpp"

namespace ofdm {

// OFDM_AB_ONLY: experiment builds (Makefile VARIANT=..., tools/ab.sh) instantiate only the
// N = 1024..4096, 64/256-QAM and adaptive kernels of the bench configs -- a fraction of the
// full compile
#ifdef OFDM_AB_ONLY
#define OFDM_LOGN_CASES(X) X(10) X(11) X(12)
#define OFDM_FB_CASES(X) X(6) X(8)
#define OFDM_FB64_CASES(X) X(6) X(8)
#else
#define OFDM_LOGN_CASES(X) \
    X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
#define OFDM_FB_CASES(X) X(2) X(3) X(4) X(5) X(6) X(8)
// complex128 throughput kernels: square QAM (4..256) and the reference's 4..32-PSK
#define OFDM_FB64_CASES(X) X(2) X(3) X(4) X(5) X(6) X(8)
#endif

template <typename F>
static hipError_t set_smem(F fn, size_t bytes) {
    // Dynamic LDS above 64 KiB must be opted in per kernel; idempotent and cheap.
    (void)hipGetLastError();  // drop a stale error of an earlier, already-reported call
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
}

// a log2 N outside the build's cases: a plan never asks for one in a product build (N is checked at
// plan creation); an OFDM_AB_ONLY build lacks N < 1024 (kNotInBuild)
#ifdef OFDM_AB_ONLY
constexpr hipError_t kOutOfRange = kNotInBuild;
#else
constexpr hipError_t kOutOfRange = hipErrorInvalidValue;
#endif

constexpr int kFastMinLogN = 6;  // throughput specialisations for N >= 64
// LDS per CU on gfx950: a throughput-kernel instantiation whose LDS would exceed it (a shape the plan
// allows but the specialised layout cannot hold) runs the generic kernel instead of failing at
// launch (tests/test_gpu_edges.py::test_lds_limit_shapes_run)
constexpr size_t kLdsPerCu = 160 * 1024;

static inline int clamp_grid(int64_t want) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, kMaxGrid));
}

template <typename R, int LOGN, int MODE>
static hipError_t rows_one(const RowsArgs& a, hipStream_t s) {
    const size_t sm = smem_rows<R>(LOGN);
    auto fn = k_rows<R, LOGN, MODE>;
    static const hipError_t attr = set_smem(fn, sm);
    if (attr != hipSuccess) return attr;
    const int64_t groups = (a.n_rows + Geo<LOGN>::SPB - 1) / Geo<LOGN>::SPB;
    hipLaunchKernelGGL(fn, dim3(clamp_grid(groups)), dim3(kBlock), sm, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_rows(int logn, int mode, const RowsArgs& a, hipStream_t s) {
    if (a.n_rows <= 0) return hipSuccess;
#define OFDM_ROWS_CASE(L)                                   \
    case L:                                                 \
        if (mode == 0) return rows_one<R, L, 0>(a, s);      \
        if (mode == 1) return rows_one<R, L, 1>(a, s);      \
        return rows_one<R, L, 2>(a, s);
    switch (logn) {
        OFDM_LOGN_CASES(OFDM_ROWS_CASE)
        default:
            return kOutOfRange;
    }
#undef OFDM_ROWS_CASE
}

template <typename R>
hipError_t launch_equalize(const EqArgs& a, hipStream_t s) {
    if (a.n_rows <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_equalize<R>, dim3(clamp_grid(a.n_rows)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_map(const MapArgs& a, hipStream_t s) {
    if (a.n_out <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_map<R>, dim3(clamp_grid((a.n_out + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_demap(const DemapArgs& a, hipStream_t s) {
    if (a.n_bytes <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_demap<R>, dim3(clamp_grid((a.n_bytes + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_demap_count(const DemapCountArgs& a, hipStream_t s) {
    const int64_t n = a.n_sym * a.n_fft;
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_demap_count<R>, dim3(clamp_grid((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_conv(const ConvArgs& a, int grid, hipStream_t s) {
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_conv<R>, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_power(const PowerArgs& a, int grid, hipStream_t s) {
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_power<R>, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename R>
hipError_t launch_awgn(const AwgnArgs& a, hipStream_t s) {
    if (a.len <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_awgn<R>, dim3(clamp_grid((a.len + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// Workgroups of a kernel resident on the device at once (occupancy x CUs), cached per kernel,
// device, workgroup size and dynamic LDS; 0 when the runtime cannot say.
template <typename F>
static int resident_blocks(F fn, int blk, size_t smem) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, int, size_t>, int> cached;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const auto key = std::make_tuple(reinterpret_cast<const void*>(fn), dev, blk, smem);
    std::lock_guard<std::mutex> lock(mu);
    const auto it = cached.find(key);
    if (it != cached.end()) return it->second;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), blk, smem) !=
            hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        return cached[key] = 0;
    }
    return cached[key] = per_cu * cus;
}

// Symbols per multipath symbol group (each group regenerates its predecessor's tail once): the
// chunk in [max / 2, max] whose rounds of resident workgroups times (chunk + 1) symbols per group
// is least.  A launch of 1e5 symbols (one point of an SNR sweep) at chunk 32 needed 1.5 rounds of
// workgroups -- two, the second half empty; chunk 25 fits it in two full rounds of 26-symbol
// groups instead of 33.
static inline int tx_chunk(int64_t n_sym, int max_chunk, int spb, int resident) {
    if (resident <= 0 || n_sym <= 0) return max_chunk;
    int best = max_chunk;
    int64_t best_cost = -1;
    for (int ch = max_chunk; ch >= (max_chunk + 1) / 2; --ch) {
        const int64_t blocks = ((n_sym + ch - 1) / ch + spb - 1) / spb;
        const int64_t cost = ((blocks + resident - 1) / resident) * (ch + 1);
        if (best_cost < 0 || cost < best_cost) best_cost = cost, best = ch;
    }
    return best;
}

// OFDM_GRID_RESIDENT k > 0 (A/B): the fused receiver's grid capped at k x the workgroups resident at
// once, so each workgroup stages its tables once and loops over its share of the symbols (the
// transmitter lost 4-8 % that way: profiles/r05h_ab_grid_resident.txt)
#ifndef OFDM_GRID_RESIDENT
#define OFDM_GRID_RESIDENT 0
#endif
static inline int fused_grid(int64_t want, int resident) {
    if (OFDM_GRID_RESIDENT > 0 && resident > 0) want = std::min<int64_t>(want, (int64_t)OFDM_GRID_RESIDENT * resident);
    return clamp_grid(want);
}

template <typename R, int LOGN, int FB, int LT, bool ZPW = false, bool REF = false>
static hipError_t tx_launch(const TxArgs& a0, int* grid, hipStream_t s) {
    constexpr int BLK = tx_block<R, FB, LOGN, LT, ZPW>();
    TxArgs a = a0;
    if (FB > 0 && LT > 0) {
        if constexpr (sizeof(R) == 8) {
            // complex128: the row of reals carries half a symbol's stream as complex samples, half 0's
            // m in [-(LT-1), cp + N/2) at wfir_in(A8 - cp + LT - 1 + m), and N / 2 transposed outputs
            const int A8 = (a.c.cp + 7) & ~7;
            a.slot = std::max(a.slot, 2 * (wfir_in(A8 + (1 << LOGN) / 2 + LT - 2, LT) + 1));
            a.slot = std::max(a.slot, 2 * (wfir_out((1 << LOGN) / 2 - 1) + 1));
        } else {
            // window FIR row: stream samples [-(LT-1), N+cp) at fir_pad(R0 + m)
            const int A = (a.c.cp + 15) & ~15, R0 = A - a.c.cp + LT - 1;
            a.slot = std::max(a.slot, fir_pad(R0 + (1 << LOGN) + a.c.cp) + 1);
        }
    }
    const size_t sm = smem_tx<R>(LOGN, BLK, FB > 0 ? 0 : a.c.lut_len, a.c.words_per_sym, a.L, a.slot,
                                 uses_tt<R, LOGN, FB>() ? tt_size(LOGN) : 0, FB > 0 && LT > 0,
                                 FB == 1 ? (size_t)4 << LOGN : 0, FB > 0, split_rows<R, FB>() && LT >= 0);
    if constexpr (FB > 0) {
        if (sm + tx_static_lds<R, FB, LT>() > kLdsPerCu) return tx_launch<R, LOGN, 0, -1>(a0, grid, s);
    }
    auto fn = k_tx<R, LOGN, FB, LT, ZPW, REF>;
    hipError_t e = set_smem(fn, sm);
    if (e != hipSuccess) return e;
    const int resident = resident_blocks(fn, BLK, sm);
    if (a.chunk > 1) a.chunk = tx_chunk(a.c.n_sym, a.chunk, Geo<LOGN, BLK>::SPB, resident);
    const int64_t groups = (a.c.n_sym + a.chunk - 1) / a.chunk;
    *grid = clamp_grid((groups + Geo<LOGN, BLK>::SPB - 1) / Geo<LOGN, BLK>::SPB);
    hipLaunchKernelGGL(fn, dim3(*grid), dim3(BLK), sm, s, a);
    return hipGetLastError();
}

// throughput TX by channel length: flat / window FIR (<= 4 or <= 8 taps) / run-time taps
template <typename R, int LOGN, int FB>
static hipError_t tx_fast(const TxArgs& a, int* grid, hipStream_t s) {
    constexpr int TPS = Geo<LOGN>::TPS;
    if (a.L == 1 && !a.c.zpad) return tx_launch<R, LOGN, FB, 0>(a, grid, s);
    if constexpr (LOGN >= 8) {
        // the complex64 register window assumes a cyclic prefix; the complex128 one takes zero padding
        if (a.c.cp <= TPS && (!a.c.zpad || sizeof(R) == 8)) {
            // complex128 zero padding: the window FIR with the guard compiled in (ZPW)
            if constexpr (sizeof(R) == 8) {
                if (a.c.zpad) {
                    if (a.L <= 4) return tx_launch<R, LOGN, FB, 4, true>(a, grid, s);
                    if (a.L <= 8) return tx_launch<R, LOGN, FB, 8, true>(a, grid, s);
                }
            }
            if (a.L <= 4) return tx_launch<R, LOGN, FB, 4>(a, grid, s);
            if (a.L <= 8) return tx_launch<R, LOGN, FB, 8>(a, grid, s);
        }
    }
    return tx_launch<R, LOGN, FB, -1>(a, grid, s);
}

// Reference streams (the caller's bits; RX: and normals) on the bench configs' shapes go through the
// throughput kernels' REF instantiations -- the timed kernels' bodies with the bit and noise source
// swapped (ref_lane, array normals) -- so the reference's own streams pin the benched FFT / FIR /
// slicer / count code (tests/test_gpu_ref_streams.py): complex128, OFDM with a cyclic prefix, fixed
// 64-QAM at N = 1024 (configs b, c) and 256-QAM at N = 4096 (config e), adaptive square-QAM loading
// at N = 2048 (config d, FB = 1), flat or <= 8-tap channels within the window FIR's reach.
// Everything else with caller bits takes the generic kernel.
template <typename R, int LOGN>
constexpr int ref_fb() { return sizeof(R) == 8 ? (LOGN == 10 ? 6 : LOGN == 11 ? 1 : LOGN == 12 ? 8 : 0) : 0; }

template <typename R, int LOGN>
static bool ref_shape(const TxRxCommon& c) {
    constexpr int FB = ref_fb<R, LOGN>();
    if (FB == 0 || c.bits == nullptr || c.nn || c.scm || c.zpad) return false;
    if (FB == 1) return c.adaptive && c.upat;  // (upat: square QAM of orders <= 256, the adaptive kernels')
    return !c.adaptive && c.psk_m == 0 && c.b == FB;
}

template <typename R, int LOGN>
static hipError_t tx_ref(const TxArgs& a, int* grid, hipStream_t s) {
    constexpr int FB = ref_fb<R, LOGN>();
    if constexpr (FB > 0) {
        constexpr int TPS = Geo<LOGN>::TPS;
        if (a.L == 1) return tx_launch<R, LOGN, FB, 0, false, true>(a, grid, s);
        if (a.c.cp <= TPS) {
            if (a.L <= 4) return tx_launch<R, LOGN, FB, 4, false, true>(a, grid, s);
            if (a.L <= 8) return tx_launch<R, LOGN, FB, 8, false, true>(a, grid, s);
        }
    }
    return tx_launch<R, LOGN, 0, -1>(a, grid, s);
}

// Throughput configuration (complex64, fixed square QAM or the reference's 4/8/16/32-PSK (psk_m > 0),
// Philox bits; N >= 64; OFDM or SC-OFDM, cyclic prefix or zero padding) -> the kernel specialised on the bits per
// subcarrier; adaptive bit loading over the reference's square-QAM LUTs (OFDM, cyclic
// prefix) -> the adaptive throughput kernel (FB = 1); anything else -> the generic kernel.
template <typename R, int LOGN>
static hipError_t tx_one(const TxArgs& a, int* grid, hipStream_t s) {
    if (ref_shape<R, LOGN>(a.c)) return tx_ref<R, LOGN>(a, grid, s);
    if constexpr (sizeof(R) == 8 && LOGN >= kFastMinLogN) {
        // complex128 throughput kernels: device bits; square QAM with adaptive loading (OFDM, cyclic
        // prefix); fixed square QAM or the reference's 4..32-PSK, OFDM or SC-OFDM, cyclic prefix or
        // zero padding
        if (a.c.adaptive && a.c.upat && a.c.bits == nullptr && !a.c.scm && !a.c.zpad && !a.c.nn)
            return tx_fast<R, LOGN, 1>(a, grid, s);
        if (!a.c.adaptive && a.c.bits == nullptr && (!a.c.nn || a.c.psk_m > 0) && (a.c.b % 2 == 0 || a.c.psk_m > 0)) {
#define OFDM_TX_FB64(F) \
    case F:                \
        return tx_fast<R, LOGN, F>(a, grid, s);
            switch (a.c.b) {
                OFDM_FB64_CASES(OFDM_TX_FB64)
                default: break;
            }
#undef OFDM_TX_FB64
        }
    }
    if constexpr (sizeof(R) == 4 && LOGN >= kFastMinLogN) {
        if (a.c.adaptive && a.c.upat && a.c.bits == nullptr && !a.c.scm && !a.c.zpad && !a.c.nn)
            return tx_fast<R, LOGN, 1>(a, grid, s);
        // OFDM / SC, CP / ZP, QAM / PSK (odd bits: the reference's 8/32-PSK only)
        if (!a.c.adaptive && a.c.bits == nullptr && (!a.c.nn || a.c.psk_m > 0) && (a.c.b % 2 == 0 || a.c.psk_m > 0)) {
#define OFDM_TX_FB(F) \
    case F:              \
        return tx_fast<R, LOGN, F>(a, grid, s);
            switch (a.c.b) {
                OFDM_FB_CASES(OFDM_TX_FB)
                default: break;
            }
#undef OFDM_TX_FB
        }
    }
    return tx_launch<R, LOGN, 0, -1>(a, grid, s);
}

template <typename R>
hipError_t launch_tx(int logn, const TxArgs& a, int* grid, hipStream_t s) {
#define OFDM_TX_CASE(L) \
    case L:             \
        return tx_one<R, L>(a, grid, s);
    switch (logn) {
        OFDM_LOGN_CASES(OFDM_TX_CASE)
        default:
            return kOutOfRange;
    }
#undef OFDM_TX_CASE
}

template <typename R, int LOGN, int EQ, int FB, bool MV, bool REF = false>
static hipError_t rx_launch(const RxArgs& a, int* grid, hipStream_t s) {
    constexpr int BLK = rx_block<R, FB, LOGN, EQ, MV>();
    const size_t sm = smem_rx<R>(LOGN, BLK, a.c.words_per_sym,
                                 uses_tt<R, LOGN, FB>() ? tt_size(LOGN) * (FB > 1 && a.c.scm ? 2 : 1) : 0,
                                 (FB == 1 ? 8 * (sizeof(R) == 8 ? sizeof(OrderParams64) : sizeof(OrderParams)) : 0) +
                                     (eq_in_lds<R, FB, LOGN, EQ>() ? ((size_t)2 * sizeof(R)) << LOGN : 0),
                                 FB > 0, split_rows<R, FB>());
    if constexpr (FB > 0) {
        if (sm + rx_static_lds<R, FB>() > kLdsPerCu) return rx_launch<R, LOGN, -1, 0, true>(a, grid, s);
    }
    auto fn = k_rx<R, LOGN, EQ, FB, MV, REF>;
    hipError_t e = set_smem(fn, sm);
    if (e != hipSuccess) return e;
    const int64_t want = (a.c.n_sym + Geo<LOGN, BLK>::SPB - 1) / Geo<LOGN, BLK>::SPB;
    constexpr int ROUNDS = rx_grid_rounds<R, FB, LOGN>();
    const int res = ROUNDS > 0 ? resident_blocks(fn, BLK, sm) : 0;
    *grid = res > 0 ? clamp_grid(std::min<int64_t>(want, (int64_t)ROUNDS * res))
                    : fused_grid(want, OFDM_GRID_RESIDENT > 0 ? resident_blocks(fn, BLK, sm) : 0);
    hipLaunchKernelGGL(fn, dim3(*grid), dim3(BLK), sm, s, a);
    return hipGetLastError();
}

// MV: the run-time modem variants (SC-OFDM, zero padding) compiled in.  complex128 builds them as
// separate kernels: compiled into the cyclic-prefix OFDM kernels of the bench, their second
// transform and guard overlap-add spilled the config (b) receiver (~70 dwords at 128 VGPRs)
template <typename R, int LOGN, int FB, bool MV = true, bool REF = false>
static hipError_t rx_eq(const RxArgs& a, int* grid, hipStream_t s) {
    if (a.c.eq == OFDM_EQ_NONE) return rx_launch<R, LOGN, OFDM_EQ_NONE, FB, MV, REF>(a, grid, s);
    if (a.c.eq == OFDM_EQ_ZF) return rx_launch<R, LOGN, OFDM_EQ_ZF, FB, MV, REF>(a, grid, s);
    return rx_launch<R, LOGN, OFDM_EQ_MMSE, FB, MV, REF>(a, grid, s);
}

// Throughput configuration (complex64, fixed square QAM or the reference's 4/8/16/32-PSK (psk_m > 0),
// Philox bits and noise, no received-symbol tap; N >= 64) -> kernel specialised on bits and
// equaliser; anything else -> the generic kernel.
template <typename R, int LOGN>
static hipError_t rx_one(const RxArgs& a, int* grid, hipStream_t s) {
    if constexpr (ref_fb<R, LOGN>() > 0) {
        // reference streams on a bench shape (see ref_shape): the REF receiver needs the caller's
        // normals and no received-symbol tap
        // (MV: as the timed kernels -- compiled out of the fixed-QAM ones, and in the adaptive
        // kernel's instantiation, where FB = 1 forces SC-OFDM and zero padding off)
        if (ref_shape<R, LOGN>(a.c) && a.nr != nullptr && a.z_out == nullptr)
            return rx_eq<R, LOGN, ref_fb<R, LOGN>(), ref_fb<R, LOGN>() == 1, true>(a, grid, s);
    }
    if constexpr (sizeof(R) == 8 && LOGN >= kFastMinLogN) {
        if (a.c.adaptive && a.c.upat && a.c.bits == nullptr && a.nr == nullptr && a.z_out == nullptr &&
            !a.c.scm && !a.c.zpad && !a.c.nn)
            return rx_eq<R, LOGN, 1>(a, grid, s);
        if (!a.c.adaptive && a.c.bits == nullptr && a.nr == nullptr && a.z_out == nullptr &&
            (!a.c.nn || a.c.psk_m > 0) && (a.c.b % 2 == 0 || a.c.psk_m > 0)) {
#define OFDM_RX_FB64(F)                                                              \
    case F:                                                                              \
        return (a.c.scm || a.c.zpad) ? rx_eq<R, LOGN, F, true>(a, grid, s)               \
                                     : rx_eq<R, LOGN, F, false>(a, grid, s);
            switch (a.c.b) {
                OFDM_FB64_CASES(OFDM_RX_FB64)
                default: break;
            }
#undef OFDM_RX_FB64
        }
    }
    if constexpr (sizeof(R) == 4 && LOGN >= kFastMinLogN) {
        if (a.c.adaptive && a.c.upat && a.c.bits == nullptr && a.nr == nullptr && a.z_out == nullptr &&
            !a.c.scm && !a.c.zpad && !a.c.nn)
            return rx_eq<R, LOGN, 1>(a, grid, s);
        if (!a.c.adaptive && a.c.bits == nullptr && a.nr == nullptr && a.z_out == nullptr &&
            (!a.c.nn || a.c.psk_m > 0) && (a.c.b % 2 == 0 || a.c.psk_m > 0)) {  // OFDM / SC, CP / ZP, QAM / PSK
#define OFDM_RX_FB(F) \
    case F:              \
        return rx_eq<R, LOGN, F>(a, grid, s);
            switch (a.c.b) {
                OFDM_FB_CASES(OFDM_RX_FB)
                default: break;
            }
#undef OFDM_RX_FB
        }
    }
    return rx_launch<R, LOGN, -1, 0, true>(a, grid, s);
}

template <typename R>
hipError_t launch_rx(int logn, const RxArgs& a, int* grid, hipStream_t s) {
#define OFDM_RX_CASE(L) \
    case L:             \
        return rx_one<R, L>(a, grid, s);
    switch (logn) {
        OFDM_LOGN_CASES(OFDM_RX_CASE)
        default:
            return kOutOfRange;
    }
#undef OFDM_RX_CASE
}

// The launchers are instantiated in three groups so the complex64 kernels -- the bulk of
// the compile -- build as separate translation units in parallel (ofdm_kernels_f32*.hip).
#define OFDM_INSTANTIATE_OPS(R)                                                     \
    template hipError_t launch_rows<R>(int, int, const RowsArgs&, hipStream_t);     \
    template hipError_t launch_equalize<R>(const EqArgs&, hipStream_t);             \
    template hipError_t launch_map<R>(const MapArgs&, hipStream_t);                 \
    template hipError_t launch_demap<R>(const DemapArgs&, hipStream_t);             \
    template hipError_t launch_demap_count<R>(const DemapCountArgs&, hipStream_t);  \
    template hipError_t launch_conv<R>(const ConvArgs&, int, hipStream_t);          \
    template hipError_t launch_power<R>(const PowerArgs&, int, hipStream_t);        \
    template hipError_t launch_awgn<R>(const AwgnArgs&, hipStream_t);
#define OFDM_INSTANTIATE_TX(R) template hipError_t launch_tx<R>(int, const TxArgs&, int*, hipStream_t);
#define OFDM_INSTANTIATE_RX(R) template hipError_t launch_rx<R>(int, const RxArgs&, int*, hipStream_t);
#define OFDM_INSTANTIATE(R) OFDM_INSTANTIATE_OPS(R) OFDM_INSTANTIATE_TX(R) OFDM_INSTANTIATE_RX(R)

}  // namespace ofdm
