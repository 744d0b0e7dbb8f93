// ofdm_fused.hpp -- the two fused hot-path kernels (included by ofdm_kernels.hpp).
//
// Data distribution: a symbol is owned by TPS = N/E threads; thread t holds
// elements k = t + i*TPS (i < E) in registers from the constellation map through
// the IFFT to the channel output (TX), and from the HBM load through the FFT to
// the error count (RX).  LDS carries only the Stockham transposes between FFT
// passes, (reference mode) the symbol's tx bit words, and (TX, multipath) the
// extended serial stream for the FIR.  With TPS <= 64 a symbol lives in one
// wavefront and every synchronisation is wave-local (sym_sync), so the 4 waves of a
// workgroup run decoupled.
//
// Specialisations: FB = 2/4/6/8 selects the throughput kernel (fixed square QAM -- or the
// reference's 4/16-PSK -- with b = FB bits, Philox-keyed bits and noise, complex64; OFDM or
// SC-OFDM, cyclic prefix or zero padding as wave-uniform run-time flags); FB = 3/5 the same
// kernel for the reference's 8/32-PSK (sector decisions only); FB = 1 is the throughput kernel for adaptive
// bit loading (per-subcarrier square-QAM orders, CAPACITY_BASED, OFDM with a cyclic prefix);
// FB = 0 is the generic kernel (reference-mode bytes and normals, PSK, complex128, adaptive
// SC-OFDM / zero padding).
#pragma once

#include <type_traits>

// Minimum waves per SIMD requested per fused kernel (register budget 512/waves), tuned on
// MI355X (tools/ab.sh): TX 3 waves/SIMD, RX unconstrained.  Build-time knobs (Makefile
// TX_WAVES / RX_WAVES) for occupancy studies.
#ifndef OFDM_TX_WAVES
#define OFDM_TX_WAVES 3
#endif
// throughput TX with the register-window FIR (LT = 4 / 8): 2 waves/SIMD (256 registers) --
// at 3 the window, the taps and the FFT state spill (54 VGPRs at LT = 8); measured on MI355X:
// config (c) TX 3.71 -> 2.94 ms, (e) 14.1 -> 12.5 ms per 1e6 symbols, while the generic kernel
// is faster at 3 (SC-OFDM TX 3.57 vs 4.33 ms)
#ifndef OFDM_TX_WFIR_WAVES
#define OFDM_TX_WFIR_WAVES 2
#endif
#ifndef OFDM_RX_WAVES
#define OFDM_RX_WAVES 1
#endif
// Workgroup of the throughput (FB > 0) kernels at N <= 1024 (TX; RX without equaliser):
// 8 waves share one copy of the twiddle tables and two workgroups fit the 160 KB LDS, i.e.
// 4 waves per SIMD (register budget 128).  Other variants: 256 threads, OFDM_*_WAVES.
#ifndef OFDM_TX_FAST_BLOCK
#define OFDM_TX_FAST_BLOCK 512
#endif
#ifndef OFDM_RX_FAST_BLOCK
#define OFDM_RX_FAST_BLOCK 512
#endif

// Streaming (nontemporal) loads of the channel samples in RX: y is read exactly once, and
// the nontemporal hint lifts the achievable read rate of this access pattern on MI355X from
// 6.2 to 7.1 TB/s (tools/hbm_probe.hip).  TX stores: the same hint, off for complex64 (no gain
// measured on the write side), on for the complex128 flat TX (config b TX 3.10 -> 3.00 ms,
// profiles/r03r_ab.txt; not on the window-FIR TX's lane-contiguous stores).
#ifndef OFDM_RX_NT
#define OFDM_RX_NT 1
#endif
#ifndef OFDM_TX_NT
#define OFDM_TX_NT 0
#endif
#ifndef OFDM_TX_NT_F64
#define OFDM_TX_NT_F64 1
#endif

namespace ofdm {

template <bool NT, typename C>
__device__ __forceinline__ C ld_stream(const C* p) {
    if constexpr (NT && sizeof(C) == 8) {
        C v;
        v.v = __builtin_nontemporal_load((const f32x2*)p);
        return v;
    } else if constexpr (NT && sizeof(C) == 16) {
        const f64x2 u = __builtin_nontemporal_load((const f64x2*)p);
        C v;
        v.re = u.x;
        v.im = u.y;
        return v;
    } else {
        return *p;
    }
}
template <bool NT, typename C>
__device__ __forceinline__ void st_stream(C* p, C v) {
    if constexpr (NT && sizeof(C) == 8)
        __builtin_nontemporal_store(v.v, (f32x2*)p);
    else
        *p = v;
}
template <bool NT>
__device__ __forceinline__ void st_stream(__attribute__((address_space(1))) cpx<float>* p, cpx<float> v) {
    typedef __attribute__((address_space(1))) f32x2 gf2;
    if constexpr (NT)
        __builtin_nontemporal_store(v.v, (gf2*)p);
    else
        *(gf2*)p = v.v;
}
template <bool NT>
__device__ __forceinline__ void st_stream(__attribute__((address_space(1))) cpx<double>* p, cpx<double> v) {
    typedef __attribute__((address_space(1))) f64x2 gd2;
    const f64x2 u = f64x2{v.re, v.im};
    if constexpr (NT)
        __builtin_nontemporal_store(u, (gd2*)p);
    else
        *(gd2*)p = u;
}

// Global-memory (address space 1) pointers: a pointer rebuilt from an integer would
// otherwise be generic and compile to flat_* instructions.
template <typename T>
using gptr = __attribute__((address_space(1))) T*;

// A wave-uniform pointer held in SGPRs (readfirstlane of both halves).
template <typename T>
__device__ __forceinline__ gptr<T> uniform_ptr(T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (gptr<T>)(((uint64_t)hi << 32) | lo);
}
// base + element offset as (64-bit base) + zext(32-bit byte offset): the addressing the
// global_load/store SGPR-base form matches
template <typename T>
__device__ __forceinline__ gptr<T> lane_ptr(gptr<T> base, uint32_t elem) {
    return (gptr<T>)((__attribute__((address_space(1))) char*)base + (uint64_t)(elem * (uint32_t)sizeof(T)));
}

// Raw buffer resource over `bytes` bytes at p (gfx9 word 3) and a 16-byte load at a lane byte
// offset (VGPR) plus a wave-uniform one (SGPR): one address register for any number of loads.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// (NT: the nontemporal hint, cache-policy bit 1 on gfx950)
template <typename T, bool NT = false>
__device__ __forceinline__ T buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    static_assert(sizeof(T) == 16, "16-byte element");
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, NT ? 2 : 0));
}
// (No buffer-store counterpart, deliberately: buffer_store_dwordx4 with a register SGPR offset
// corrupted the low data dword on gfx950 -- the compiler inserts no wait state between such a store
// and the next VALU write of its data VGPRs, DESIGN.md section 4.  Stores use the global_store forms;
// tests/test_isa_guard.py rejects any buffer store in the fused kernels' code.)

// complex128 multipath TX of square QAM (the plan sends only separable LUTs to the throughput
// kernels): map through the two axis tables instead of the complex LUT (TX c 5.13 -> 5.12, e 5.26
// -> 5.17 ms per step, profiles/r03aa_ab.txt)
template <typename R, int FB, int LT>
constexpr bool tx_sep_lut() { return sizeof(R) == 8 && FB >= 2 && !(FB & 1) && LT != 0; }

// complex128 RX with a symbol per wave: the channel samples through buffer loads (one address
// VGPR, the element offsets in SGPRs) instead of four 64-bit VGPR addresses (RX b 3.09 -> 3.06,
// c 3.75 -> 3.70 ms per step at the same occupancy, profiles/r03ab_ab.txt)

// MP: multipath channel (L > 1; the generic kernel always takes L from the plan)
#ifndef OFDM_TX_MP_BLOCK
#define OFDM_TX_MP_BLOCK 256
#endif
// complex128 throughput kernels (R = double, FB > 0).  The FFT exchanges through split real /
// imaginary rows (fft_reg_split: 8.5 KB per N = 1024 symbol), so the occupancy is set by the
// registers: 16 complex128 elements per lane plus a radix-16 butterfly -- RX ~160 VGPRs (3 waves
// per SIMD: one 768-thread workgroup of 12 symbols per CU), flat TX 128 (4 waves: 1024 threads).
// A 4-wave RX (1024 threads, 128 VGPRs, 7 spilled) measured config b 1.646 -> 1.648e8 symbols/s,
// within the run-to-run spread (profiles/r03k_ab_rx1024.txt); with the channel samples
// buffer-loaded (6 dwords spilled at 128) it gains: RX 3.09 -> 2.98 ms, 1.669 ->
// 1.693e8 symbols/s (profiles/r03ab_ab.txt) -- the no-equaliser RX takes 1024 threads at 4 waves.
// The window-FIR TX passes the extended stream through its row of reals twice (real, then
// imaginary parts), in 256-thread workgroups at 2 waves per SIMD: two or more workgroups per
// CU, so a symbol group's barriers (N >= 2048: TPS > 64) hold back fewer waves.  Against
// complex rows at 512 threads (256 where they did not fit, 1 wave per SIMD): TX per step
// c 5.45 -> 5.37, d 7.01 -> 5.41, e 6.37 -> 5.39 ms; rows of reals at 512 threads measured
// 5.59 / 6.67 / 6.65 (profiles/r03o_ab.txt).
#ifndef OFDM_F64_TX_BLOCK
#define OFDM_F64_TX_BLOCK 1024
#endif
#ifndef OFDM_F64_TX_WAVES
#define OFDM_F64_TX_WAVES 4
#endif
#ifndef OFDM_F64_RX_BLOCK
#define OFDM_F64_RX_BLOCK 1024
#endif
#ifndef OFDM_F64_RX_WAVES
#define OFDM_F64_RX_WAVES 4
#endif
#ifndef OFDM_F64_FIR_BLOCK
#define OFDM_F64_FIR_BLOCK 256
#endif
#ifndef OFDM_F64_FIR_WAVES
#define OFDM_F64_FIR_WAVES 2
#endif
// N = 4096 (config e, 4 waves per symbol): 3 waves per SIMD (168 VGPRs, 18 dwords spilled) --
// TX e 4.65 -> 4.46 ms, 2.833 -> 2.877e7 symbols/s (profiles/r04q_ab_e_fir_3waves.txt); at N = 1024 /
// 2048 the same step spills 39 / 51 dwords (config c measured 15 % slower, profiles/r04b_ab_fir.txt)
#ifndef OFDM_F64_FIR_WAVES_4K
#define OFDM_F64_FIR_WAVES_4K 3
#endif
// complex64 throughput kernels at N >= 2048 (configs d, e): workgroup and waves per SIMD of RX
// and of the window-FIR TX (two or four waves per symbol).  With the compact twiddle tables the
// LDS no longer caps a CU at two workgroups, so 3 waves per SIMD fit: config e RX 3.37 -> 2.84 ms
// per 2.5e5 symbols; N = 2048 (config d) prefers 768-thread workgroups (RX 3.08 -> 2.99 ms per
// 5e5 symbols), N = 4096 256 (profiles/r03h_ab.txt)
#ifndef OFDM_RX_BIG_BLOCK
#define OFDM_RX_BIG_BLOCK(LOGN) ((LOGN) == 11 ? 768 : 256)
#endif
#ifndef OFDM_RX_BIG_WAVES
#define OFDM_RX_BIG_WAVES 3
#endif
#ifndef OFDM_TX_BIG_WFIR_WAVES
#define OFDM_TX_BIG_WFIR_WAVES 3
#endif
// LDS of the complex128 FIR TX at blk threads (upper estimate of its Carve sequence, smem_tx):
// FIR rows -- window FIR: half a symbol's stream as complex samples, wfir_in(N/2 + 48) + 1 of
// them (cp <= 32), or the FFT's N + N/16 reals if more; the run-time-tap FIR: fir_pad(N + 32) + 1
// complex -- and the 7 complex tail samples per symbol, per-pass twiddles, the static LUT
// (adaptive: the 512-entry pool and the per-subcarrier table), taps
constexpr int f64_fir_lds(int fb, int logn, int blk, bool real_rows) {
    const int n = 1 << logn, tps = logn < 4 ? 1 : n >> 4, spb = blk / tps;
    const int fir = (n + 32) + ((n + 32) >> 4) + 1, half = 2 * (n / 2 + 48 + ((n / 2 + 48 + 7) >> 3) + 1);
    const int padn = n + (n >> 4);
    const int rows = spb * ((real_rows ? (half > padn ? half : padn) * 8 : fir * 16) + 7 * 16);
    const int tt = tt_size(logn) * 16;
    const int lut = fb == 1 ? (kMaxLut + 1) * 16 + 4 * n : (16 << fb);
    return rows + tt + lut + 1024;
}
// static (__shared__) LDS of the fused kernels beside their dynamic rows (kLdsPerCu checks)
template <typename R, int FB>
constexpr size_t rx_static_lds() {
    return 8 * kNoisePhases + (sizeof(R) == 8 && FB > 0 ? 16 * kNoisePhases : 16);
}
template <typename R, int FB, int LT>
constexpr size_t tx_static_lds() {
    const size_t lut = FB == 1 ? kMaxLut + 1 : (FB > 1 ? ((size_t)1 << FB) : 1);
    const size_t sep = (sizeof(R) == 8 && FB >= 2 && !(FB & 1) && LT != 0) ? 2 * ((size_t)1 << (FB / 2)) : 1;
    return lut * 2 * sizeof(R) + sep * sizeof(R);
}
// LT (throughput TX): 0 flat channel; 4 / 8 multipath with <= LT taps through the register
// window FIR (N >= 256, cp <= TPS); -1 any multipath (run-time loop over taps).  ZPW: the complex128
// window FIR with the zero-padding guard (and its run-time flat path for a one-tap channel) compiled
// in; without it (cyclic prefix, L > 1: the bench configs) the kernel needs ~139 VGPRs instead of
// 205-227 (3 waves per SIMD would fit with nothing spilled; measured no faster)
template <typename R, int FB, int LOGN, int LT, bool ZPW = false>
constexpr int tx_block() {
    if (sizeof(R) == 8 && FB > 0) {
        if (LT == 0) return OFDM_F64_TX_BLOCK;
        return f64_fir_lds(FB, LOGN, OFDM_F64_FIR_BLOCK, LT > 0) <= 160 * 1024 ? OFDM_F64_FIR_BLOCK : 256;
    }
    return FB > 0 && LOGN <= 10 ? (LT != 0 ? OFDM_TX_MP_BLOCK : OFDM_TX_FAST_BLOCK) : kBlock;
}
constexpr int block_waves(int blk, int dflt) { return blk >= 512 ? 4 : dflt; }
template <typename R, int FB, int LOGN, int LT, bool ZPW = false>
constexpr int tx_waves() {
    if (sizeof(R) == 8 && FB > 0) {
        if (LT == 0) return OFDM_F64_TX_WAVES;
        return LOGN >= 12 ? OFDM_F64_FIR_WAVES_4K : OFDM_F64_FIR_WAVES;
    }
    if (FB > 0 && LT > 0 && LOGN > 10) return OFDM_TX_BIG_WFIR_WAVES;
    return block_waves(tx_block<R, FB, LOGN, LT>(), FB > 0 && LT > 0 ? OFDM_TX_WFIR_WAVES : OFDM_TX_WAVES);
}
// padded FIR row index of the throughput multipath TX: one slot per 16 elements
__host__ __device__ constexpr int fir_pad(int i) { return i + (i >> 4); }
// complex128 window-FIR TX, LDS slots (16 bytes) of the half-symbol row.  Stream phase: stream
// index kk at wfir_in(kk) -- one pad slot per 8, placed so that the FFT elements (kk = LT - 1 +
// t + TPS i mod 8: every 8 lanes one aligned run) are written without a pad inside an 8-lane
// group, and the lanes' windows (kk = 8 t + W) read at lane stride 9.  Output phase: output kk at
// wfir_out(kk), an XOR swizzle of the 8-slot runs -- the lanes' runs of 8 outputs are written to
// distinct banks and the stores' reads (kk = t + TPS i) hit 16 distinct 4-bank sets per
// ds_read_b128 lane group.  Against wfir_slot (kk + kk / 8) for both phases: no bank conflicts
// (SQ_LDS_BANK_CONFLICT 197 cycles per config-c symbol, tools/lds_banks.py --fir models 192).
__host__ __device__ constexpr int wfir_ioff(int lt) { return (9 - lt) & 7; }
__host__ __device__ constexpr int wfir_in(int kk, int lt) { return kk + ((kk + wfir_ioff(lt)) >> 3); }
__host__ __device__ constexpr int wfir_out(int kk) { return (kk & ~7) | ((kk ^ (kk >> 3)) & 7); }
// complex128 RX of fixed QAM at N = 4096 (config e): one symbol per 256-thread workgroup at 3 waves
// per SIMD, the equaliser coefficients read from the plan's table after the FFT (rx_eq_late)
// instead of a 64 KB LDS copy per workgroup -- with the copy, two symbols per 512-thread workgroup
// at 2 waves per SIMD, one barrier coupling both symbols' FFT exchanges.  Config e RX 5.02 ->
// 4.21 ms per 2.5e5 symbols (2 waves per SIMD: 4.63); the step gains less (9.99 -> 9.64 ms): the
// TX that follows runs 0.4 ms slower at the power cap (profiles/r03y_ab.txt)
#ifndef OFDM_F64_RX_SOLO_WAVES
#define OFDM_F64_RX_SOLO_WAVES 3
#endif
// the complex128 adaptive receiver at N = 2048 (config d): one 128-thread symbol per workgroup
#ifndef OFDM_F64_RX_ADAPT_WAVES
#define OFDM_F64_RX_ADAPT_WAVES 2
#endif
// the OFDM_F64_RX_BLOCK / _WAVES shape: no-equaliser RX of 64/256-QAM at N = 1024 (at 128 VGPRs the
// QPSK / 16-QAM and smaller-N kernels spill 22-33 dwords, so they stay at 768 threads, 3 waves;
// with an equaliser the 16 KB coefficient table beside 16 symbols' rows exceeds the LDS)
template <int FB, int LOGN, int EQ, bool MV = false>
constexpr bool f64_rx_wide() { return EQ == OFDM_EQ_NONE && FB >= 6 && LOGN == 10 && !MV; }
// (the same for the adaptive RX at N = 2048 (config d) -- 128-thread workgroups
// of one symbol at 2 waves per SIMD, instead of four symbols per 512-thread workgroup: RX 5.12 ->
// 4.67 ms, step 10.11 -> 9.93 ms per 5e5 symbols, profiles/r03ad_ab.txt)
template <typename R, int FB, int LOGN>
constexpr bool f64_rx_solo() {
    return sizeof(R) == 8 && ((FB > 1 && LOGN == 12) || (FB == 1 && LOGN == 11));
}
// MV: the complex128 SC-OFDM / zero-padding kernels (k_rx MV), ~10-50 VGPRs above their cyclic-prefix
// OFDM twins: never the 4-wave shape, and the one-symbol N = 4096 shape at 2 waves per SIMD
template <typename R, int FB, int LOGN, int EQ, bool MV = false>
constexpr int rx_block() {
    // (the adaptive kernel's per-order tables take ~200 VGPRs in complex128: 2 waves per SIMD)
    if (f64_rx_solo<R, FB, LOGN>()) return (1 << LOGN) / 16;  // one symbol
    if (sizeof(R) == 8 && FB > 0)
        return (LOGN > 10 || FB == 1) ? 512 : (f64_rx_wide<FB, LOGN, EQ, MV>() ? OFDM_F64_RX_BLOCK : 768);
    if (FB > 0 && LOGN > 10) return OFDM_RX_BIG_BLOCK(LOGN);
    return FB > 1 && LOGN <= 10 && EQ == OFDM_EQ_NONE ? OFDM_RX_FAST_BLOCK : kBlock;
}
template <typename R, int FB, int LOGN, int EQ, bool MV = false>
constexpr int rx_waves() {
    if (f64_rx_solo<R, FB, LOGN>()) return FB == 1 ? OFDM_F64_RX_ADAPT_WAVES : MV ? 2 : OFDM_F64_RX_SOLO_WAVES;
    if (sizeof(R) == 8 && FB > 0)
        return (LOGN > 10 || FB == 1) ? 2 : (f64_rx_wide<FB, LOGN, EQ, MV>() ? OFDM_F64_RX_WAVES : 3);
    if (FB > 0 && LOGN > 10) return OFDM_RX_BIG_WAVES;
    return rx_block<R, FB, LOGN, EQ>() >= 512 ? 4 : OFDM_RX_WAVES;
}
// throughput RX: equaliser coefficients staged in LDS up to N = 2^OFDM_EQ_LDS_MAX_LOGN (beyond,
// the table would cost a resident workgroup per CU)
#ifndef OFDM_EQ_LDS_MAX_LOGN
#define OFDM_EQ_LDS_MAX_LOGN 11
#endif
// complex128 at N = 4096: the table (64 KB) fits beside two symbols' split rows and the compact
// twiddles, and preloading 16 complex128 coefficients would spill
template <typename R, int FB, int LOGN, int EQ>
constexpr bool eq_in_lds() {
    return FB > 0 && EQ > OFDM_EQ_NONE && LOGN <= (sizeof(R) == 8 ? 12 : OFDM_EQ_LDS_MAX_LOGN) &&
           !f64_rx_solo<R, FB, LOGN>();
}
// complex128 throughput receivers at N = 1024 (configs b, c): one workgroup holds a CU, and each
// start and drain of one idles it -- the grid is OFDM_RX_GRID_ROUNDS rounds of the resident
// workgroups instead of up to kMaxGrid.  Config c RX 3.556 -> 3.50 ms per 1e6 symbols and
// 0.43 -> 0.37 ms per 1e5 (a sweep point); one round (static striding) lost 2 % at 1e6, and the
// other receivers (several workgroups per CU) lost 1-5 % with two (profiles/r05h_ab_grid_resident.txt).
// (A queue the waves took their symbols from was 3.4x slower: one atomic counter serialised
// ~12 ns per symbol, profiles/r05j_ab_rx_symbol_queue.txt.)
#ifndef OFDM_RX_GRID_ROUNDS
#define OFDM_RX_GRID_ROUNDS 2
#endif
template <typename R, int FB, int LOGN>
constexpr int rx_grid_rounds() {
    return sizeof(R) == 8 && FB > 0 && LOGN == 10 ? OFDM_RX_GRID_ROUNDS : 0;
}
// the lane's coefficients loaded after the FFT (in flight across the MMSE power reduction)
template <typename R, int FB, int LOGN, int EQ>
constexpr bool rx_eq_late() { return f64_rx_solo<R, FB, LOGN>() && EQ > OFDM_EQ_NONE; }
// MMSE in complex128: the reciprocals of |H|^2 + nv of four elements from one v_rcp_f64 (+ two
// Newton steps) and nine products (Montgomery's batch inversion; ~3 roundings more than one
// reciprocal each, well inside the decision bracket's 8 u of equaliser arithmetic).  RX c 3.80 ->
// 3.75, e 4.21 -> 4.16 ms per step (profiles/r03y_ab.txt)
// complex128 throughput kernels exchange FFT data through rows of reals (fft_reg_split)
template <typename R, int FB>
constexpr bool split_rows() { return sizeof(R) == 8 && FB > 0; }


// Reference mode: stage OFDM symbol s's tx bits from the packed bytes of the run
// (symbol s starts at bit s*bps, zeros past the end) as 32-bit words in W
// (stream bit 32w+j = bit 31-j of word w).  Returns the symbol's bit offset in word 0.
template <int TPS>
__device__ __forceinline__ int stage_words(const TxRxCommon& a, int64_t s, uint32_t* W, int t) {
    const int64_t bit0 = s * a.bps;
    const int64_t B0 = bit0 >> 3;
    for (int w = t; w < a.words_per_sym; w += TPS) {
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

template <typename R>
__device__ __forceinline__ R recip(R d) {
    if constexpr (sizeof(R) == 4) {
        return __builtin_amdgcn_rcpf(d);  // v_rcp_f32 (1 ulp): throughput mode
    } else {
        // v_rcp_f64 and two Newton steps (~1 ulp) instead of the IEEE division sequence
        R r = __builtin_amdgcn_rcp(d);
        r = __builtin_fma(__builtin_fma(-d, r, (R)1), r, r);
        return __builtin_fma(__builtin_fma(-d, r, (R)1), r, r);
    }
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

// The lane block of a reference-stream symbol for the throughput kernels' REF instantiations: byte
// i = the FB bits of element i (subcarrier k = t + i TPS), read MSB first from the caller's byte
// stream at bit s bps + k FB (the reference's bit order, bits_generation/models.py:26-44 and
// serial_parallel/models.py:12-33) -- the layout lane_bits reads, so the kernel body is the
// throughput kernel's.  Global byte reads (uncoalesced: REF runs are parity runs, not timed).
template <int FB, int TPS>
__device__ __forceinline__ u4 ref_lane(const TxRxCommon& a, int64_t s, int t) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    const int64_t bit0 = s * a.bps;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t o = bit0 + (int64_t)(t + i * TPS) * FB;
        const int64_t B = o >> 3;
        const uint32_t hi = B < a.n_bytes ? (uint32_t)a.bits[B] : 0u;
        const uint32_t lo = B + 1 < a.n_bytes ? (uint32_t)a.bits[B + 1] : 0u;
        const uint32_t v = (((hi << 8) | lo) >> (16 - (int)(o & 7) - FB)) & ((1u << FB) - 1u);
        w[i >> 2] |= v << (8 * (i & 3));
    }
    return u4{w[0], w[1], w[2], w[3]};
}

// The same for adaptive loading (FB = 1): byte i = the b_k bits of subcarrier k = t + i TPS, read MSB
// first at bit s bps + bitoff_k (constellation/adaptive.py:178-199: each OFDM symbol's bits laid out
// subcarrier-major with variable b_k), zero for an unused subcarrier -- the lane byte the adaptive
// kernels mask with (1 << b_k) - 1.  b_k <= 8 (the plan's upat: orders <= 256), so three bytes cover
// any alignment.
template <int TPS>
__device__ __forceinline__ u4 ref_lane_adaptive(const TxRxCommon& a, int64_t s, int t) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    const int64_t bit0 = s * a.bps;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const ScInfo sc = a.sc[t + i * TPS];
        if (sc.lut < 0 || sc.bits <= 0) continue;
        const int64_t o = bit0 + sc.bitoff;
        const int64_t B = o >> 3;
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) v = (v << 8) | (B + j < a.n_bytes ? (uint32_t)a.bits[B + j] : 0u);
        v = (v >> (24 - (int)(o & 7) - sc.bits)) & ((1u << sc.bits) - 1u);
        w[i >> 2] |= v << (8 * (i & 3));
    }
    return u4{w[0], w[1], w[2], w[3]};
}

// Per-element tx constellation indices of one symbol for this lane, from whichever
// source the launch uses: the lane generator's first 128 bits (philox mode) or the
// staged words (reference mode).  FB > 0: fixed b = FB, compile-time offsets.  In philox
// mode the generator g continues into the lane's noise (RX).  REF: the throughput kernel's lane
// block filled from the caller's bits instead (ref_lane; adaptive: ref_lane_adaptive).
template <int FB, int TPS, bool REF = false>
struct TxBits {
    u4 lane;
    Mwc64x g;
    const uint32_t* W;
    int base_bit;
    bool from_words;

    // payload words (P2, P3, m0, m1); the generator continues into the lane's noise
    __device__ __forceinline__ void seed_lane(uint64_t seed, int64_t s, int t) {
        const u4 p = philox_lane(seed, s, (uint32_t)t, kLane);
        g.seed(p.x, p.y);
        lane.x = p.z;
        lane.y = p.w;
        lane.z = g.next();
        lane.w = g.next();
    }
    __device__ __forceinline__ void load(const TxRxCommon& a, int64_t s, int t, uint32_t* Wslot, bool active) {
        from_words = FB == 0 && a.bits != nullptr;
        W = Wslot;
        base_bit = 0;
        lane.x = lane.y = lane.z = lane.w = 0u;
        if constexpr (REF && FB == 1) {
            if (active) lane = ref_lane_adaptive<TPS>(a, s, t);
        } else if constexpr (REF && FB > 1) {
            if (active) lane = ref_lane<FB, TPS>(a, s, t);
        } else if (from_words) {
            if (active) base_bit = stage_words<TPS>(a, s, Wslot, t);
        } else if (active) {
            seed_lane(a.seed, s, t);
        }
    }
    template <int I>
    __device__ __forceinline__ uint32_t fixed() const {
        return lane_bits(lane, I, FB);
    }
    // i: the element's index in the lane (philox mode); stream_off: its offset inside the
    // symbol's bit stream (reference mode)
    __device__ __forceinline__ uint32_t generic(int i, int b, int stream_off) const {
        if (from_words) return extract_w(W, base_bit + stream_off, b);
        return lane_bits(lane, i, b);
    }
};

// M-PSK as the reference builds it (constellation/models.py:356-380: LUT[gray(i)] =
// exp(2 pi j i / M)), complex64: the nearest point is the nearest angle, found without a
// search.  The point is folded into the first octant (|x|, |y|, swap when |y| > |x|), the
// sector inside the octant is counted against tan((q + 1/2) 2 pi / M) for q < M/8, and the
// three reflections are undone on the sector index k; the LUT index is gray(k).  M = 2 and
// 4 have no in-octant boundaries.  Decisions differ from the brute-force search only on a
// decision boundary (|y| = |x| or an exact tangent), a probability-zero event under noise.
template <typename R>
__device__ __forceinline__ uint32_t psk_decide(cpx<R> v, const TxRxCommon& cm) {
    const int M = cm.psk_m;
    const R ax = fabs(v.re), ay = fabs(v.im);
    const bool sw = ay > ax, sx = v.re < (R)0, sy = v.im < (R)0;
    const R u = fmax(ax, ay), w = fmin(ax, ay);  // angle of (u, w) in [0, pi/4]
    int k;
    if (M == 2) {
        k = sx ? 1 : 0;
    } else {
        int q = 0;
        for (int j = 0; j < (M >> 3); ++j) q += w > (sizeof(R) == 8 ? (R)cm.psk_tan64[j] : (R)cm.psk_tan[j]) * u;
        const int quarter = M >> 2;
        int k1 = sw ? quarter - q : q;        // reflect about 45 degrees
        if (M == 4) k1 = sw ? 1 : 0;
        int k2 = sx ? 2 * quarter - k1 : k1;  // reflect about 90 degrees
        k = sy ? (M - k2) & (M - 1) : k2;     // reflect about 0 degrees
    }
    return (uint32_t)(k ^ (k >> 1));
}

// Nearest constellation point of a non-separable LUT (PSK): the m points at offset off of the
// LUT pool (adaptive loading: the subcarrier's order; fixed: the whole single LUT).  complex128:
// the reference's |z - C_m| with hypot and the first index on ties (nn_index); complex64: the
// sector decision above for the reference's fixed M-PSK in throughput mode (cm.psk_m > 0 only
// there, ofdm_abi.hip fill_common), else squared distances in float against the plan-precision LUT.
template <typename R>
__device__ __forceinline__ uint32_t nn_decide(cpx<R> v, const TxRxCommon& cm, int off, int count) {
    if constexpr (sizeof(R) == 8) {
        return (uint32_t)nn_index(v.re, v.im, cm.lut64 + 2 * off, count);
    } else {
        if (cm.psk_m > 0) return psk_decide(v, cm);
        const cpx<float>* L = (const cpx<float>*)cm.lut + off;
        float bd = INFINITY;
        uint32_t best = 0;
        for (int m = 0; m < count; ++m) {
            const float dr = v.re - L[m].re, di = v.im - L[m].im;
            const float d = dr * dr + di * di;
            if (d < bd) {
                bd = d;
                best = (uint32_t)m;
            }
        }
        return best;
    }
}


// FFT of one symbol in a fused kernel: complex128 throughput kernels exchange through a row of
// reals (fft_reg_split), complex64 ones through the complex row with per-pass LDS twiddles, the
// generic kernel with the two-level table and recurrence.
template <typename R, int LOGN, bool INV, int FB>
__device__ __forceinline__ void fft_sym(cpx<R> (&x)[Geo<LOGN>::E], cpx<R>* row, const cpx<R>* tw,
                                        const cpx<R>* tt, int t) {
    if constexpr (split_rows<R, FB>())
        fft_reg_split<R, LOGN, INV, fast_tt<R, LOGN>()>(x, (R*)row, tw, tw + 64, t, tt);
    else
        fft_reg<R, LOGN, INV, (FB > 0)>(x, row, tw, tw + 64, t, tt);
}
// per-pass twiddle tables in LDS (throughput kernels while they fit) vs the two-level table
template <typename R, int LOGN, int FB>
constexpr bool uses_tt() { return FB > 0 && fast_tt<R, LOGN>(); }

// ============================================================ fused TX
// Each symbol group walks `chunk` consecutive OFDM symbols so the FIR tail (last L-1
// stream samples of the previous symbol) is carried in LDS; the first symbol of a chunk
// regenerates its predecessor's tail (one extra IFFT per chunk, L > 1 only).
// REF: the throughput kernel fed the caller's bits (reference streams, ref_lane) -- the same body
template <typename R, int LOGN, int FB, int LT, bool ZPW = false, bool REF = false>
__global__ __launch_bounds__((tx_block<R, FB, LOGN, LT, ZPW>()), (tx_waves<R, FB, LOGN, LT, ZPW>())) void k_tx(
    TxArgs a) {
    constexpr int BLK = tx_block<R, FB, LOGN, LT, ZPW>();
    constexpr bool WFIR = FB > 0 && LT > 0;  // register window FIR
    constexpr bool TX_NT = OFDM_TX_NT || (sizeof(R) == 8 && OFDM_TX_NT_F64);  // nontemporal y stores
    using G = Geo<LOGN, BLK>;
    using C = cpx<R>;
    constexpr int N = G::N, E = G::E, TPS = G::TPS;
    const TxRxCommon& cm = a.c;
    const int flags = ablation_flags(a.flags);
    const bool adaptive = FB ? false : (bool)cm.adaptive;
    // generic kernel variants: single-carrier OFDM (no IFFT, modulation/models.py:
    // 58-70) and the zero-padding guard (prefix/models.py:55-67: [x | 0 ... 0])
    const bool scm = FB == 1 ? false : (bool)cm.scm;  // SC-OFDM (run-time, uniform)
    // zero-padding guard (run-time, uniform); compiled out of the flat throughput TX (a zero
    // guard needs cp > 0, the launcher sends it to the LT = -1 kernel), where the run-time
    // row stride alone cost 15 % (config b TX 1.64 -> 1.92 ms)
    // (window FIR: only the ZPW instantiation -- the launcher sends zero padding there, and a one-tap
    // channel without it to the flat kernel, so the CP window FIR never takes the flat path below)
    constexpr bool ZP_OK = !(FB == 1 || (FB > 1 && LT == 0)) && (!WFIR || ZPW);
    constexpr bool FLAT_OK = !WFIR || ZPW;
    const bool zp = ZP_OK ? (bool)cm.zpad : false;
    const int ystride = ZP_OK ? cm.ystride : N;  // stored samples per OFDM symbol: N, or N + cp (ZP)
    const int cp = cm.cp, L = LT != 0 ? a.L : 1;
    const int slot = a.slot;  // complex elements per symbol row (>= PADN and >= L-1+cp+N)
    const int tls = L > 1 ? L - 1 : 1;
    constexpr bool TT = uses_tt<R, LOGN, FB>();
    // complex128 flat and window-FIR TX: a row of reals (fft_reg_split)
    // (the window FIR passes its stream through the row of reals twice: real, then imaginary parts)
    constexpr bool ROW_REAL = split_rows<R, FB>() && LT >= 0;
    Carve cv(ofdm_smem);
    C* tw = cv.take<C>(TT ? 0 : 128);  // two-level twiddles (generic kernel, complex128 N > 1024)
    // throughput kernels: the LUT in static LDS at a link-time address, so an element's LUT read
    // is addressed by its index bits alone (2^FB entries; adaptive: the pool + a zero entry);
    // generic kernel: dynamic
    constexpr int LUT_STATIC = FB == 1 ? kMaxLut + 1 : (FB > 1 ? (1 << FB) : 1);
    __shared__ C lut_s[LUT_STATIC];
    // complex128 multipath TX of square QAM: the LUT as its two axis tables (tx_sep_lut)
    constexpr bool SEP = tx_sep_lut<R, FB, LT>();
    constexpr int HB = FB / 2, SIDE = 1 << HB;
    __shared__ R sep_s[SEP ? 2 * SIDE : 1];
    C* lut = FB > 0 ? lut_s : cv.take<C>(cm.lut_len);
    C* h = cv.take<C>(32);
    C* hsw = cv.take<C>(WFIR ? 32 : 0);  // window FIR: the taps swizzled, (-im, re)
    AxisInfo* axis = cv.take<AxisInfo>(kMaxLuts);
    unsigned char* rowmem = cv.take<unsigned char>((size_t)G::SPB * slot * (ROW_REAL ? sizeof(R) : sizeof(C)));
    C* tails = cv.take<C>((size_t)G::SPB * tls);
    uint32_t* words = cv.take<uint32_t>(FB ? 0 : (size_t)G::SPB * cm.words_per_sym);  // reference bits
    double* red = cv.take<double>(BLK / 64);
    constexpr int TTS = TT ? tt_size(LOGN) : 0;
    C* tt = cv.take<C>(TTS);  // throughput kernel: inverse per-pass twiddles
    // adaptive throughput kernel: per subcarrier (LUT offset << 8 | tx bit mask); unused
    // subcarriers point at a zero entry appended to the LUT pool
    uint32_t* sce = cv.take<uint32_t>(FB == 1 ? N : 0);

    // the tables' global reads issued first (Staged), then the LDS writes
    constexpr bool FOLD_H0 = FB > 0 && LT == 0;
    const C* glut = (const C*)cm.lut;
    Staged<BLK, TTS, C> st_tt;
    Staged<BLK, (FB > 0 ? LUT_STATIC : BLK), C, (FB > 0)> st_lut;  // (generic kernel: any LUT length)
    Staged<BLK, (FB == 1 ? N : 0), ScInfo> st_sc;
    Staged<BLK, kMaxLuts, Dwords<AxisInfo>> st_ax;
    static_assert(kMaxLuts <= BLK && 32 <= BLK, "one axis entry / tap per thread");
    C hq = mk<R>(0, 0), sep_a = mk<R>(0, 0), sep_b = mk<R>(0, 0), hf = mk<R>(1, 0);
    int ax_off = 0;
    if constexpr (FOLD_H0) hf = ((const C*)a.h)[0];
    st_tt.load((const C*)cm.ptw + TTS, TTS);
    st_lut.load(glut, cm.lut_len);
    if constexpr (FB == 1) st_sc.load(cm.sc, N);
    st_ax.load((const Dwords<AxisInfo>*)cm.axis, cm.n_axis);
    if (threadIdx.x < L && threadIdx.x < 32) hq = ((const C*)a.h)[threadIdx.x];
    // adaptive: lane l of every wave holds order l's LUT offset, for the codes' lane shuffle
    if constexpr (FB == 1) {
        if ((int)(threadIdx.x & 63) < cm.n_axis) ax_off = cm.axis[threadIdx.x & 63].lut_off;
    }
    if constexpr (SEP) {
        if (threadIdx.x < SIDE) sep_a = glut[threadIdx.x], sep_b = glut[threadIdx.x << HB];
    }
    if constexpr (!TT) load_twiddles<R>(tw, (const C*)cm.tw);
    // the 1/sqrt(N) of ifft(norm="ortho") folded into the LUT (same product per element);
    // flat throughput kernel: the channel tap too (y = h0 ifft(X) = ifft(h0 X)), so the
    // symbol leaves the IFFT as the channel output
    const R lut_scale = scm ? (R)1 : (R)cm.scale;
    st_tt.store(tt);
    st_lut.store(lut, [&](const C& v) { return cscale(FOLD_H0 ? cmul(hf, v) : v, lut_scale); });
    if constexpr (SEP) {
        // LUT[i] = I[i & (SIDE - 1)] + j Q[i >> HB] exactly (the plan's build_axis verified it):
        // I from the entries with Q index 0, Q from those with I index 0, the same scaled values
        if (threadIdx.x < SIDE) {
            sep_s[threadIdx.x] = sep_a.re * lut_scale;
            sep_s[SIDE + threadIdx.x] = sep_b.im * lut_scale;
        }
    }
    st_ax.store((Dwords<AxisInfo>*)axis);
    if constexpr (FB == 1) {
        if (threadIdx.x == 0) lut[cm.lut_len] = mk<R>(0, 0);
        auto code = [&](const ScInfo& sc, int off) {
            return sc.lut < 0 ? (uint32_t)cm.lut_len << 8 : ((uint32_t)off << 8) | ((1u << sc.bits) - 1u);
        };
        // the order's LUT offset from the lane holding it (a dependent global read per element
        // had been waited for one by one); entries past the staged ones (N > 8 BLK) read directly
        int k0 = threadIdx.x;
#pragma unroll
        for (int q = 0; q < st_sc.K; ++q, k0 += BLK) {
            const ScInfo sc = st_sc.v[q];
            // (a slot past N was never loaded: its lane index is taken as 0, not read)
            const int lid = k0 < N ? (int)sc.lut : -1;
            const int off = __shfl(ax_off, lid < 0 ? 0 : lid);
            if (k0 < N) sce[k0] = code(sc, off);
        }
        for (int k = k0; k < N; k += BLK) {
            const ScInfo sc = cm.sc[k];
            sce[k] = code(sc, sc.lut < 0 ? 0 : cm.axis[sc.lut].lut_off);
        }
    }
    if (threadIdx.x < 32) {
        h[threadIdx.x] = hq;
        if (WFIR) hsw[threadIdx.x] = mk<R>(-hq.im, hq.re);  // window FIR (complex64): taps swizzled
    }
    __syncthreads();

    const int ls = TPS >= 64 ? __builtin_amdgcn_readfirstlane(threadIdx.x / TPS) : threadIdx.x / TPS;
    const int t = threadIdx.x % TPS;
    C* row = (C*)(rowmem + (size_t)ls * slot * (ROW_REAL ? sizeof(R) : sizeof(C)));
    C* tl = tails + ls * tls;
    uint32_t* W = words + ls * cm.words_per_sym;
    C* yout = (C*)a.y;
    const C h0 = h[0];
    // window FIR: the stream sample m in [-(LT-1), N+cp) lives at row[fir_pad(R0 + m)], R0 chosen
    // so that lane t's window (samples cp + 16 t - (LT-1) ..) starts at row index A + 16 t,
    // A = 16 ceil(cp/16)
    constexpr int LTN = WFIR ? LT : 1;
    const int A = (cp + 15) & ~15, R0 = A - cp + LTN - 1;
    const int64_t ngroups = (cm.n_sym + a.chunk - 1) / a.chunk;
    const int64_t niter = (ngroups + G::SPB - 1) / G::SPB;
    // sum |y|^2 in exact fixed point (fx_accum, per lane and symbol); |x|^2 statistics in double
    unsigned long long pq0 = 0, pq1 = 0;
    double px = 0, mx = 0;

    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        const int64_t grp = it * G::SPB + ls;
        const int64_t sbeg = grp * a.chunk;  // local symbol index
        for (int c = (L > 1 ? -1 : 0); c < a.chunk; ++c) {
            const int64_t sl = sbeg + c;
            const int64_t sg = cm.sym0 + sl;
            const bool active = grp < ngroups && sl < cm.n_sym && sg >= 0;
            TxBits<FB, TPS, REF> tb;
            tb.load(cm, sg, t, W, active && !(flags & 1));
            if (FB == 0) sym_sync<TPS>();  // staged words visible
            // map (QAMConstellationMapper.encode, constellation/models.py:240-246); the
            // 1/sqrt(N) of ifft(norm="ortho") folded in
            // (throughput kernels: an inactive symbol maps its zero lane words -- nothing of it
            // is stored or counted, and its tail is zeroed below)
            C x[E];
            if constexpr (FB == 1) {
                // element i: the low b_k bits of lane byte i through its subcarrier's LUT.  The
                // table index is made opaque per symbol so the 16 loop-invariant reads are not
                // hoisted out of the symbol loop as 16 live registers.
                int st = t;
                asm volatile("" : "+v"(st));
                static_for<0, E>([&](auto I) {
                    const uint32_t e = sce[st + I * TPS];
                    const uint32_t v = (lane_word(tb.lane, I >> 2) >> (8 * (I & 3))) & e & 0xFFu;
                    x[I] = lut[(e >> 8) + v];
                });
            } else if (SEP && cm.psk_m == 0) {
                // two 8-byte reads from SIDE-entry tables: distinct entries sit on distinct banks
                // (the 2^FB-entry complex table's random 16-byte reads conflicted); the reference's
                // 4/16-PSK (not separable) take the complex table below
                static_for<0, E>([&](auto I) {
                    const uint32_t v = tb.template fixed<I>();
                    x[I] = mk<R>(sep_s[v & (SIDE - 1)], sep_s[SIDE + (v >> HB)]);
                });
            } else if constexpr (FB > 0) {
                static_for<0, E>([&](auto I) { x[I] = lut[tb.template fixed<I>()]; });
            } else {
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const int k = t + i * TPS;
                    C v = mk<R>(0, 0);
                    if (active) {
                        if (adaptive) {
                            const ScInfo sc = cm.sc[k];
                            if (sc.lut >= 0) v = lut[axis[sc.lut].lut_off + tb.generic(i, sc.bits, sc.bitoff)];
                        } else {
                            v = lut[tb.generic(i, cm.b, k * cm.b)];
                        }
                    }
                    x[i] = v;
                }
            }
            if (!(flags & 2) && !scm) fft_sym<R, LOGN, true, FB>(x, row, tw, tt, t);
            // The prefix repeats samples k >= N - cp.  With cp <= TPS only the lane's last
            // element can be one of them (one loop-invariant compare); otherwise the compares
            // are made per symbol against an opaque copy of N - cp, so they are not hoisted
            // as E live 64-bit masks (SGPR spills).
            int ncp = N - cp;
            asm volatile("" : "+s"(ncp));
            auto prefix_sum = [&](auto&& pw) -> R {
                if (zp) return (R)0;  // the zero guard adds no power
                if (WFIR || cp <= TPS) return t >= TPS - cp ? pw(E - 1) : (R)0;  // (window FIR: cp <= TPS)
                R acc = 0;
#pragma unroll
                for (int i = 0; i < E; ++i)
                    if (t + i * TPS >= ncp) acc += pw(i);
                return acc;
            };
            // PAPR statistics over the modulated symbol incl. its prefix (simulation/models.py:519-522)
            R pxs = 0;
            if (active && c >= 0) {
                R mxs = 0;  // per-symbol partials in the arithmetic precision
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const R p2 = norm2(x[i]);
                    pxs += p2;
                    // (complex128 flat channel: v_max_f64 directly, 15 VALU per symbol and lane fewer;
                    // the window-FIR kernels schedule fmax without the quieting step already, and the
                    // complex64 ones grow with it)
                    mxs = (sizeof(R) == 8 && LT == 0) ? peak_max(mxs, p2) : fmax(mxs, p2);
                }
                pxs += prefix_sum([&](int i) { return norm2(x[i]); });
                px += pxs;
                mx = fmax(mx, (double)mxs);
            }
            if (FLAT_OK && L == 1) {
                // flat channel: y = h0 x, no inter-symbol memory
                if (active && c >= 0) {
                    C* yo = yout + sl * ystride;
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const C yv = FOLD_H0 ? x[i] : cmul(h0, x[i]);
                        if (!yout || (flags & 4)) continue;
                        if constexpr (FB > 0 && TPS >= 64) {
                            // the row base is wave-uniform: made explicit, the stores take the
                            // SGPR-base + 32-bit lane-offset form instead of a loop-carried 64-bit
                            // VGPR pointer (which spilled to scratch, and whose per-symbol reload's
                            // vmcnt(0) waited for all of the previous symbol's stores)
                            st_stream<TX_NT>(lane_ptr(uniform_ptr(yo), (uint32_t)(t + i * TPS)), yv);
                        } else {
                            st_stream<(FB > 0 && TX_NT)>(yo + t + i * TPS, yv);
                        }
                    }
                    if (zp && yout)
                        for (int j = t; j < cp; j += TPS) yo[N + j] = mk<R>(0, 0);
                    if constexpr (FOLD_H0) {
                        fx_accum((R)pxs, pq0, pq1);  // the statistics above were taken on y (x |h0|^2 fixed below)
                    } else if constexpr (FB > 0) {
                        fx_accum((R)(norm2(h0) * pxs), pq0, pq1);  // |y|^2 = |h0|^2 |x|^2 (complex64 mode)
                    } else {
                        R pys = 0;
#pragma unroll
                        for (int i = 0; i < E; ++i) pys += norm2(cmul(h0, x[i]));
                        pys += prefix_sum([&](int i) { return norm2(cmul(h0, x[i])); });
                        fx_accum((R)pys, pq0, pq1);
                    }
                }
                sym_sync<TPS>();  // W / row reuse by the next symbol
            } else if constexpr (WFIR) {
                // throughput multipath (L <= LT, cp <= TPS, E = 16, TPS >= 16): lane t computes the
                // 16 consecutive kept samples k = 16 t + j from a register window of 16 + LT - 1
                // stream samples read once from LDS (fir_pad: lane stride 17 elements, conflict
                // free; offsets compile-time) -- 23 LDS reads instead of 2 L per output
                static_assert(E == 16 && TPS >= 16, "window FIR geometry");
                constexpr int WN = E + LT - 1;
                if constexpr (sizeof(R) == 8) {
                    // complex128: the FIR runs over the symbol in two halves of N / 2 kept samples,
                    // through the symbol's row of reals used as complex samples, one pad slot per 8
                    // (wfir_in).  Half h holds the stream samples m in [cp + h N/2 - (LT-1),
                    // cp + (h+1) N/2) at wfir_in(B_h + m) -- half 0 from m = -(LT-1): the previous
                    // symbol's tail and the prefix region too -- and lane t computes the 8
                    // consecutive kept samples k = h N/2 + 8 t + j from a window of 8 + LT - 1
                    // complex samples (ds_read_b128 at lane stride 9: conflict free), streamed one
                    // sample at a time through the outputs' accumulators in Gauss's three-
                    // multiplication form:
                    //   T = sum hr (wr + wi),  U = sum (hr + hi) wi,  V = sum (hi - hr) wr,
                    //   y = (T - U, T + V)
                    // (3 v_fma_f64 per tap and output; the taps' three forms in scalar registers,
                    // TxArgs::gtap, zero past L).  Live at once: half a symbol's elements, 24
                    // accumulators and the streamed sample -- against two whole windows of reals and
                    // 16 outputs' sums when the row carried the real and then the imaginary parts.
                    // The outputs leave through the row (kk = 8 t + j at wfir_out(kk), read back as
                    // kk = t + TPS i) and buffer stores: lanes 8 m .. 8 m + 7 store one whole
                    // 128-byte line.
                    // Zero padding (prefix/models.py:55-67, the stream [x | 0 ... 0]): x starts at
                    // stream sample 0 instead of cp, every one of the N + cp outputs is stored
                    // (ystride N + cp: the receiver overlap-adds the guard), the guard outputs
                    // N + t (t < cp) from the last LT - 1 samples of x in half 1's row, and the
                    // tail for the next symbol from that row too (the stream ends in the guard).
                    static_assert(LT <= kWinTaps, "window FIR taps");
                    constexpr int WH = 8 + LT - 1;
                    C* crow = (C*)row;
                    // (a complex sample as one ds_write_b128: as two ds_write_b64 -- 12 LDS cycles per KB
                    // against 13 -- TX e ran 4.78 -> 5.02 ms, profiles/r04m_ab_fir_write_b64.txt)
                    auto st16 = [&](int slot_, C v) { *(f64x2*)(crow + slot_) = f64x2{v.re, v.im}; };
                    auto ld16 = [&](const C* p) { const f64x2 u = *(const f64x2*)p; return mk<R>(u.x, u.y); };
                    const bool live = active && c >= 0;
                    const bool store = live && yout && !(flags & 4);
                    R hr[LT], c1[LT], c2[LT];
#pragma unroll
                    for (int q = 0; q < LT; ++q) {
                        hr[q] = a.gtap[0][q];
                        c1[q] = a.gtap[1][q];
                        c2[q] = a.gtap[2][q];
                    }
                    // LDS offsets and lane conditions from opaque per-symbol copies of t, cp and L,
                    // each offset a per-symbol base plus compile-time constants: hoisted out of the
                    // symbol loop they were ~20 loop-invariant registers, spilled to scratch
                    int to = t, cpo = cp, lo = L;
                    asm volatile("" : "+v"(to), "+s"(cpo), "+s"(lo));
                    if (c < 0 && !zp) {
                        // a group's regenerated predecessor: only its tail is needed, the last
                        // L - 1 samples of x (registers); no FIR, no stores
                        sym_sync<TPS>();  // the previous symbol's FIR has read the old tail
                        if (to >= TPS - (lo - 1)) tl[to - (TPS - (lo - 1))] = active ? x[E - 1] : mk<R>(0, 0);
                        sym_sync<TPS>();
                        continue;
                    }
                    const int so = zp ? 0 : cpo;  // stream sample of x[0]
                    const int A8 = (so + 7) & ~7;
                    R pys = 0;
                    static_for<0, 2>([&](auto HH) {
                        constexpr int h = HH;
                        constexpr int NH = N / 2;
                        // stream sample m at wfir_in(B + m); the lanes' windows start at Ah + 8 t
                        const int Ah = h == 0 ? A8 : 0;
                        const int B = Ah - so - h * NH + (LT - 1);
                        sym_sync<TPS>();  // the FFT's last pass / the previous half's stores have read the row
                        // this half's elements: kept k = t + TPS i (stream cp + k) for k in
                        // [h N/2 - (LT-1), (h+1) N/2); TPS i = N/2 at i = 8
                        // (TPS i = 0 mod 8: wfir_in(b + TPS i) = wfir_in(b) + 9 TPS i / 8)
                        const int bx = wfir_in(B + so + to, LT);
                        static_for<0, E>([&](auto I) {
                            constexpr int i = I;
                            constexpr int off = 9 * TPS * i / 8;
                            if constexpr (i >= 8 * h && i < 8 * h + 8) {
                                st16(bx + off, x[i]);
                            } else if constexpr (h == 1 && i == 7) {
                                if (to >= TPS - (LT - 1)) st16(bx + off, x[i]);
                            }
                        });
                        if constexpr (h == 0) {
                            if (!zp && to >= TPS - cpo) st16(wfir_in(B + to - (TPS - cpo), LT), x[E - 1]);  // cyclic prefix
                            if (to < LT - 1) {  // stream samples -(LT-1) .. -1: zeros, then the previous tail
                                const int z = to - (LT - lo);
                                st16(wfir_in(B - (LT - 1) + to, LT), z < 0 ? mk<R>(0, 0) : tl[z]);
                            }
                        }
                        sym_sync<TPS>();
                        if constexpr (h == 0) {
                            // this symbol's tail for the next one, from the registers (the old tail
                            // has been copied): its last L - 1 stream samples, lanes TPS - (L-1) ..
                            if (!zp && to >= TPS - (lo - 1)) tl[to - (TPS - (lo - 1))] = active ? x[E - 1] : mk<R>(0, 0);
                        } else {
                            // zero padding: the last L - 1 stream samples N + cp - (L-1) + z are x
                            // below N, guard zeros from N on
                            if (zp && to < lo - 1) {
                                const int m = N + cpo - (lo - 1) + to;
                                tl[to] = (active && m < N) ? ld16(crow + wfir_in(B + m, LT)) : mk<R>(0, 0);
                            }
                        }
                        // every lane streams its window, live or not (under the live condition the
                        // accumulators would be conditionally defined and spill)
                        // (wfir_in(Ah + 8 t + W) = wfir_in(Ah) + 9 t + W + (W + ioff) / 8)
                        constexpr int IOFF = wfir_ioff(LT);
                        R T[8], U[8], V[8];
                        // the window read two samples ahead of its use, in program order (the compiler
                        // issues all 8 + LT - 1 reads at once either way; tying each read to the previous
                        // sample's sums through an empty asm ran 1 % slower)
                        typedef const __attribute__((address_space(3))) f64x2* lwin;
                        lwin wl = (lwin)(crow + (wfir_in(Ah, LT) + 9 * to));
                        auto ldw = [&](int k) { const f64x2 u = wl[k]; return mk<R>(u.x, u.y); };
                        C ring[3];
                        ring[0] = ldw(IOFF >> 3);
                        ring[1] = ldw(1 + ((1 + IOFF) >> 3));
                        static_for<0, WH>([&](auto W) {
                            const C e = ring[W % 3];
                            const R sw = e.re + e.im;
                            if constexpr (W + 2 < WH) {
                                ring[(W + 2) % 3] = ldw((W + 2) + ((W + 2 + IOFF) >> 3));
                            }
                            static_for<0, LT>([&](auto Q) {  // tap Q of output j
                                constexpr int j = W - (LT - 1) + Q;
                                if constexpr (j >= 0 && j < 8) {
                                    if constexpr (Q == LT - 1) {  // the output's first term
                                        T[j] = hr[Q] * sw;
                                        U[j] = c1[Q] * e.im;
                                        V[j] = c2[Q] * e.re;
                                    } else {
                                        T[j] = __builtin_fma(hr[Q], sw, T[j]);
                                        U[j] = __builtin_fma(c1[Q], e.im, U[j]);
                                        V[j] = __builtin_fma(c2[Q], e.re, V[j]);
                                    }
                                }
                            });
                            __builtin_amdgcn_sched_barrier(0);
                        });
                        if constexpr (h == 1) {
                            // zero padding: guard output N + t = sum over l > t of h_l x[N + t - l]
                            // (the guard's own samples are zero), stored and counted
                            if (zp && live && to < cpo) {
                                R pT = 0, pU = 0, pV = 0;
#pragma unroll
                                for (int l = 1; l < LT; ++l) {
                                    if (l <= to) continue;
                                    const C e = ld16(crow + wfir_in(B + N + to - l, LT));
                                    pT = __builtin_fma(hr[l], e.re + e.im, pT);
                                    pU = __builtin_fma(c1[l], e.im, pU);
                                    pV = __builtin_fma(c2[l], e.re, pV);
                                }
                                const C yv = mk<R>(pT - pU, pT + pV);
                                pys = __builtin_fma(yv.re, yv.re, pys);
                                pys = __builtin_fma(yv.im, yv.im, pys);
                                if (store) yout[sl * ystride + N + to] = yv;
                            }
                        }
                        if constexpr (h == 0) {
                            if (!zp && live && to < cpo) {  // prefix-region output m = t: power only (noise/models.py:14)
                                R pT = 0, pU = 0, pV = 0;
#pragma unroll
                                for (int l = 0; l < LT; ++l) {
                                    const C e = ld16(crow + wfir_in(B + to - l, LT));
                                    pT = __builtin_fma(hr[l], e.re + e.im, pT);
                                    pU = __builtin_fma(c1[l], e.im, pU);
                                    pV = __builtin_fma(c2[l], e.re, pV);
                                }
                                const R pr = pT - pU, pi = pT + pV;
                                pys = __builtin_fma(pr, pr, pys);
                                pys = __builtin_fma(pi, pi, pys);
                            }
                        }
                        sym_sync<TPS>();  // every window is read: the outputs take the row
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const C yv = mk<R>(T[j] - U[j], T[j] + V[j]);
                            pys = __builtin_fma(yv.re, yv.re, pys);
                            pys = __builtin_fma(yv.im, yv.im, pys);
                            st16(8 * to + (j ^ (to & 7)), yv);  // wfir_out(8 t + j)
                        }
                        sym_sync<TPS>();
                        if (store) {
                            // global stores off two wave-uniform bases (elements i < 4 and i >= 4),
                            // the lane's 32-bit byte offset in one VGPR and element i's in the
                            // instruction's offset field (per-element 64-bit VGPR addresses were
                            // loop-invariant registers).  (Buffer stores with SGPR offsets here
                            // corrupted the last store's low data dword on gfx950: the compiler
                            // inserts no wait state between such a store and a VALU write of its
                            // data VGPRs.)
                            C* yh = yout + sl * ystride + h * NH;
                            const C* rb = crow + wfir_out(to);
#pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                // (TPS = 0 mod 64: wfir_out(t + TPS i) = wfir_out(t) + TPS i)
                                const C* ri = TPS % 64 == 0 ? rb + TPS * i : crow + wfir_out(to + TPS * i);
                                if constexpr (TPS >= 64) {
                                    gptr<C> yg = uniform_ptr(yh + (i >> 2) * 4 * TPS);
                                    st_stream<TX_NT>(lane_ptr(yg, (uint32_t)to) + (i & 3) * TPS, ld16(ri));
                                } else {
                                    st_stream<TX_NT>((gptr<C>)yh + to + TPS * i, ld16(ri));
                                }
                            }
                        }
                    });
                    if (live) fx_accum((R)pys, pq0, pq1);
                    sym_sync<TPS>();
                } else {
                    sym_sync<TPS>();  // the last FFT pass has read the row
                    {
                        const int u = R0 + cp + t;  // stream sample cp + t + TPS i at fir_pad(u + TPS i)
                        const int bx = fir_pad(u);
#pragma unroll
                        for (int i = 0; i < E; ++i) row[bx + TPS * i + (TPS * i >> 4)] = x[i];  // TPS i = 0 mod 16
                    }
                    if (t >= TPS - cp) row[fir_pad(R0 + t - (TPS - cp))] = x[E - 1];  // cyclic prefix
                    if (t < LT - 1) {  // stream samples -(LT-1) .. -1: zeros, then the previous tail
                        const int z = t - (LT - L);
                        row[fir_pad(R0 - (LT - 1) + t)] = z < 0 ? mk<R>(0, 0) : tl[z];
                    }
                    sym_sync<TPS>();
                    // complex64: taps (zero past L), LDS broadcast reads; the opaque offset keeps
                    // the reads in the symbol loop (hoisted, the 4 LT registers stay live through
                    // the FFT and spill)
                    const bool live = active && c >= 0;
                    int ho = 0;
                    asm volatile("" : "+v"(ho));
                    f32x2 hv[LT], hs[LT];
#pragma unroll
                    for (int q = 0; q < LT; ++q) {
                        hv[q] = f32x2{(float)h[ho + q].re, (float)h[ho + q].im};
                        hs[q] = f32x2{(float)hsw[ho + q].re, (float)hsw[ho + q].im};
                    }
                    // the window (every lane, live or not), the prefix-region output and the tail
                    // leave the row first: the outputs take its place
                    const C* wb = row + (A + (A >> 4) + 17 * t);
                    f32x2 win[WN];
#pragma unroll
                    for (int w = 0; w < WN; ++w) {
                        const C ev = wb[w + (w >> 4)];
                        win[w] = f32x2{(float)ev.re, (float)ev.im};
                    }
                    R pys = 0;
                    if (live && t < cp) {  // prefix-region outputs: power only (noise/models.py:14)
                        f32x2 yp = f32x2{0.f, 0.f};
#pragma unroll
                        for (int l = 0; l < LT; ++l) {
                            const C ev = row[fir_pad(R0 + t - l)];
                            const f32x2 e = f32x2{(float)ev.re, (float)ev.im};
                            yp = __builtin_elementwise_fma(e.xx, hv[l], yp);
                            yp = __builtin_elementwise_fma(e.yy, hs[l], yp);
                        }
                        pys = yp.x * yp.x + yp.y * yp.y;
                    }
                    // tail for the next symbol: the last L-1 stream samples (zeros before symbol 0)
                    if (t < L - 1) tl[t] = active ? row[fir_pad(R0 + N + cp - (L - 1) + t)] : mk<R>(0, 0);
                    sym_sync<TPS>();
                    // the lane's 16 consecutive outputs k = 16 t + j go to row[fir_pad(k)] and
                    // leave as k = t + TPS i: whole-line stores instead of 16 lines per lane
                    f32x2 pacc = f32x2{0.f, 0.f};  // (sum Re^2, sum Im^2): one packed FMA per output
#pragma unroll
                    for (int j = 0; j < E; j += 2) {
                        f32x2 y0 = f32x2{0.f, 0.f}, y1 = f32x2{0.f, 0.f};
#pragma unroll
                        for (int l = 0; l < LT; ++l) {
                            const f32x2 e0 = win[j + LT - 1 - l], e1 = win[j + LT - l];
                            y0 = __builtin_elementwise_fma(e0.xx, hv[l], y0);
                            y0 = __builtin_elementwise_fma(e0.yy, hs[l], y0);
                            y1 = __builtin_elementwise_fma(e1.xx, hv[l], y1);
                            y1 = __builtin_elementwise_fma(e1.yy, hs[l], y1);
                        }
                        pacc = __builtin_elementwise_fma(y0, y0, pacc);
                        pacc = __builtin_elementwise_fma(y1, y1, pacc);
                        row[fir_pad(E * t + j)] = mk<R>(y0.x, y0.y);
                        row[fir_pad(E * t + j + 1)] = mk<R>(y1.x, y1.y);
                    }
                    sym_sync<TPS>();
                    if (live && yout && !(flags & 4)) {
                        C* ys = yout + sl * N;
                        int to = t;  // opaque: offsets hoisted out of the loop would hold registers
                        asm volatile("" : "+v"(to));
                        gptr<C> yg = TPS >= 64 ? uniform_ptr(ys) : (gptr<C>)ys;
#pragma unroll
                        for (int i = 0; i < E; ++i)
                            st_stream<TX_NT>(lane_ptr(yg, (uint32_t)(to + TPS * i)), row[fir_pad(to + TPS * i)]);
                    }
                    if (live) fx_accum((R)(pys + pacc.x + pacc.y), pq0, pq1);
                    sym_sync<TPS>();
                }
            } else {
                // extended serial stream in the row: [tail (L-1) | prefix (cp) | x (N)], or with
                // zero padding [tail (L-1) | x (N) | zeros (cp)]
                sym_sync<TPS>();  // the last FFT pass has read the row
                const int o = zp ? L - 1 : L - 1 + cp;
#pragma unroll
                for (int i = 0; i < E; ++i) row[o + t + i * TPS] = x[i];
                if (zp) {
                    for (int j = t; j < cp; j += TPS) row[L - 1 + N + j] = mk<R>(0, 0);
                } else if (cp <= TPS) {
                    if (t >= TPS - cp) row[L - 1 + t - (TPS - cp)] = x[E - 1];
                } else {
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const int k = t + i * TPS;
                        if (k >= ncp) row[L - 1 + k - ncp] = x[i];
                    }
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
                        if (yout && !(flags & 4)) {
                            if (zp)
                                yout[sl * ystride + m] = yv;  // every stream sample (RX overlap-adds)
                            else if (m >= cp)
                                yout[sl * N + (m - cp)] = yv;
                        }
                    }
                    fx_accum((R)pys, pq0, pq1);
                }
                // tail for the next symbol: the last L-1 stream samples (zeros before symbol 0)
                for (int j = t; j < L - 1; j += TPS) tl[j] = active ? row[N + cp + j] : mk<R>(0, 0);
                sym_sync<TPS>();
            }
        }
    }
    if constexpr (FOLD_H0) {  // |x|^2 = |y|^2 / |h0|^2
        const double ih2 = 1.0 / ((double)h0.re * (double)h0.re + (double)h0.im * (double)h0.im);
        px *= ih2;
        mx *= ih2;
    }
    fx_normalize(pq0, pq1);
    pq0 = block_sum<unsigned long long, BLK>(pq0, (unsigned long long*)red);
    pq1 = block_sum<unsigned long long, BLK>(pq1, (unsigned long long*)red);
    px = block_sum<double, BLK>(px, red);
    mx = block_max<double, BLK>(mx, red);
    if (threadIdx.x == 0) {
        unsigned long long* pr = (unsigned long long*)a.partials + (size_t)blockIdx.x * kTxFields;
        pr[0] = pq0;
        pr[1] = pq1;
        a.partials[(size_t)blockIdx.x * kTxFields + 2] = px;
        a.partials[(size_t)blockIdx.x * kTxFields + 3] = mx;
    }
}

// ============================================================ fused RX
// EQ: OFDM_EQ_* fixed at compile time (throughput kernel) or -1 = from the plan.
// MV: SC-OFDM and zero padding compiled in (run-time flags); complex128 compiles them out of the
// cyclic-prefix OFDM kernels (rx_eq)
// REF: the throughput kernel fed the caller's bits and normals (reference streams) -- the same body
template <typename R, int LOGN, int EQ, int FB, bool MV, bool REF = false>
__global__ __launch_bounds__((rx_block<R, FB, LOGN, EQ, MV>()), (rx_waves<R, FB, LOGN, EQ, MV>())) void k_rx(
    RxArgs a) {
    constexpr int BLK = rx_block<R, FB, LOGN, EQ, MV>();
    using G = Geo<LOGN, BLK>;
    using C = cpx<R>;
    constexpr int N = G::N, E = G::E, TPS = G::TPS;
    const TxRxCommon& cm = a.c;
    const int flags = ablation_flags(a.flags);
    const int eq = EQ >= 0 ? EQ : cm.eq;
    const bool adaptive = FB ? false : (bool)cm.adaptive;
    // generic kernel variants: single-carrier OFDM (FFT -> equalise -> IFFT,
    // modulation/models.py:72-91), zero-padding guard (overlap-add, prefix/models.py:69-101)
    // and non-separable constellations (PSK: brute-force nearest point, constellation/models.py:19-27)
    constexpr bool F64_FAST = sizeof(R) == 8 && FB > 0;  // complex128 throughput kernels
    const bool scm = (FB == 1 || !MV) ? false : (bool)cm.scm;  // SC-OFDM (run-time, uniform)
    const bool zp = (FB == 1 || !MV) ? false : (bool)cm.zpad;  // zero-padding guard (run-time, uniform)
    const bool nn = FB ? false : (bool)cm.nn;
    const int ystride = (FB == 1 || !MV) ? N : cm.ystride;
    // odd bits per subcarrier (FB = 3, 5): the reference's 8- / 32-PSK only
    constexpr bool FB_PSK_ONLY = FB > 1 && (FB & 1);
    // noise phase table: static LDS at a link-time constant address, so a sample's entry offset
    // (from its phase word) addresses it with no add
    __shared__ f32x2 ntab[kNoisePhases];
    // complex128 throughput kernels: the table widened to double (Mwc64x::add_noise64)
    __shared__ f64x2 ntab64_s[F64_FAST ? kNoisePhases : 1];
    f64x2* ntab64 = F64_FAST ? ntab64_s : nullptr;
    Carve cv(ofdm_smem);
    constexpr bool TT = uses_tt<R, LOGN, FB>();
    constexpr bool SPLIT = split_rows<R, FB>();  // complex128 throughput: rows of reals
    C* tw = cv.take<C>(TT ? 0 : 128);  // two-level twiddles (generic kernel, complex128 N > 1024)
    AxisInfo* axis = cv.take<AxisInfo>(kMaxLuts);
    unsigned char* rowmem = cv.take<unsigned char>((size_t)G::SPB * G::PADN * (SPLIT ? sizeof(R) : sizeof(C)));
    uint32_t* words = cv.take<uint32_t>(FB ? 0 : (size_t)G::SPB * cm.words_per_sym);  // reference bits
    R* red = cv.take<R>(BLK / 64);
    unsigned long long* redc = cv.take<unsigned long long>(BLK / 64);
    constexpr int TTS = TT ? tt_size(LOGN) : 0;
    // throughput kernel: forward per-pass twiddles, plus the inverse ones for SC-OFDM's IFFT
    const int tts_all = FB > 1 && scm ? 2 * TTS : TTS;
    C* tt = cv.take<C>(tts_all);
    // adaptive: per-order slicer constants (complex128: double entries)
    using OP = std::conditional_t<sizeof(R) == 8, OrderParams64, OrderParams>;
    OP* ordt = cv.take<OP>(FB == 1 ? 8 : 0);
    // throughput kernels with an equaliser: the per-subcarrier coefficient staged in LDS once
    // per workgroup (ZF: 1/H; MMSE: conj(H), |H|^2 recomputed from it) -- read from the plan's
    // global table, every element paid an L2 round trip with a vmcnt(0) per symbol
    constexpr bool EQ_LDS = eq_in_lds<R, FB, LOGN, EQ>();
    C* eqt = cv.take<C>(EQ_LDS ? N : 0);
    // otherwise (throughput kernels at N = 4096, and the complex64 generic kernel) the lane's
    // coefficients are loaded before the FFT each symbol (L2-resident), so their latency hides
    // behind it instead of stalling each element of the equaliser
    constexpr bool EQ_LATE = rx_eq_late<R, FB, LOGN, EQ>();
    constexpr bool EQ_PRE =
        !EQ_LDS && !EQ_LATE && ((FB > 0 && EQ > OFDM_EQ_NONE) || (FB == 0 && sizeof(R) == 4));
    constexpr bool EQ_REG = EQ_PRE || EQ_LATE;  // coefficients in registers (ecoef)
    constexpr bool MMSE_BATCH = sizeof(R) == 8 && FB > 0 && EQ == OFDM_EQ_MMSE;

    // the tables' global reads issued first (Staged), the noise table built while they fly
    Staged<BLK, (FB > 1 && MV ? 2 : 1) * TTS, C> st_tt;
    Staged<BLK, EQ_LDS ? N : 0, C> st_eq;
    Staged<BLK, kMaxLuts, Dwords<AxisInfo>> st_ax;
    static_assert(kMaxLuts <= BLK, "one axis entry per thread");
    st_tt.load((const C*)cm.ptw, tts_all);
    if constexpr (EQ_LDS) st_eq.load((const C*)cm.eq_a, N);
    st_ax.load((const Dwords<AxisInfo>*)cm.axis, cm.n_axis);
    // sigma from the whole-stream mean power (noise/models.py:13-22)
    const bool noise = a.noise_on && !(flags & 1);
    double sigma_d = 0;
    if (noise) {
        const double p = a.stats[0] / (double)a.total_samples;
        sigma_d = sqrt((p / a.snr_lin) / 2.0);
    }
    const R sigma = (R)sigma_d;
    build_noise_table(ntab, sigma_d, ntab64);
    if constexpr (!TT) load_twiddles<R>(tw, (const C*)cm.tw);
    st_tt.store(tt);
    if constexpr (EQ_LDS) st_eq.store(eqt);
    st_ax.store((Dwords<AxisInfo>*)axis);
    if constexpr (FB == 1 && sizeof(R) == 8) {
        if (threadIdx.x < 8) {
            OrderParams64 o = OrderParams64::make(0.0, 0.0, 0.0, 0u);  // unused subcarrier: level 0, no bits
            if (threadIdx.x < cm.n_axis && threadIdx.x != kUnusedOrder) {
                const AxisInfo ax = __builtin_bit_cast(AxisInfo, st_ax.v[0]);  // (thread < n_axis <= kMaxLuts)
                const double span = (double)(ax.side - 1);
                o = OrderParams64::make(ax.inv_step * cm.scale / span,  // mul: the FFT output stays unscaled
                                        ax.lev0 * ax.inv_step / span,   // add: negated in the FMA
                                        span, ((1u << ax.bits) - 1u) | ((1u << ax.hbits) << 8));
            }
            ordt[threadIdx.x] = o;
        }
    } else if constexpr (FB == 1) {
        if (threadIdx.x < 8) {
            // unused subcarrier: level 0, no bits
            OrderParams o{0.f, 0.f, 0u, 0u};
            if (threadIdx.x < cm.n_axis && threadIdx.x != kUnusedOrder) {
                const AxisInfo ax = __builtin_bit_cast(AxisInfo, st_ax.v[0]);  // (thread < n_axis <= kMaxLuts)
                const double span = (double)(ax.side - 1);  // see OrderParams
                o.mul = (float)(ax.inv_step * cm.scale / span);  // the FFT output stays unscaled
                o.add = (float)(-ax.lev0 * ax.inv_step / span);
                o.smax = __float_as_uint((float)(ax.side - 1));
                o.meta = ((1u << ax.bits) - 1u) | ((1u << ax.hbits) << 8);
            }
            ordt[threadIdx.x] = o;
        }
    }
    __syncthreads();

    // a symbol group of >= 64 threads is whole wavefronts: make its index wave-uniform
    const int ls = TPS >= 64 ? __builtin_amdgcn_readfirstlane(threadIdx.x / TPS) : threadIdx.x / TPS;
    const int t = threadIdx.x % TPS;
    C* row = (C*)(rowmem + (size_t)ls * G::PADN * (SPLIT ? sizeof(R) : sizeof(C)));
    uint32_t* W = words + ls * cm.words_per_sym;
    const C* eqa = (const C*)cm.eq_a;
    const __amdgpu_buffer_rsrc_t eq_rsrc = buf_rsrc(eqa, (uint32_t)(N * sizeof(C)));
    const R* eqb = (const R*)cm.eq_b;
    // ZF / MMSE of subcarrier k (equalization/models.py:22-63); nv: the symbol's MMSE noise variance
    // (pa: the coefficient the throughput kernel preloaded for this element, or null)
    auto eq_apply = [&](C v, int k, R nv, const C* pa) -> C {
        if constexpr (EQ_LDS || EQ_REG) {
            // ZF 1/H; MMSE conj(H) with |H|^2 recomputed from it (complex64 only)
            const C c = EQ_LDS ? eqt[k] : *pa;
            if (eq == OFDM_EQ_ZF) return cmul(v, c);
            const R d = c.re * c.re + c.im * c.im + nv;  // |H|^2 + nv
            return cscale(cmul(v, c), recip<R>(d));
        } else {
            if (eq == OFDM_EQ_ZF) return cmul(v, eqa[k]);
            if (eq == OFDM_EQ_MMSE) return cmul(v, mmse_coef<R>(eqa[k], eqb[k], nv));
            return v;
        }
    };
    const int cp = cm.cp;
    const R scale = (R)cm.scale;
    Slicer<R> slicer;
    std::conditional_t<sizeof(R) == 8, PermSlicer64<(FB > 1 ? FB : 2)>, PermSlicer<(FB > 1 ? FB : 2)>> pslicer;
    // adaptive throughput kernel: the LDS byte offset of each element's order entry, four
    // elements per word (the lane's subcarriers do not change from symbol to symbol)
    uint32_t ocode[FB == 1 ? E / 4 : 1];
    bool small_orders = false;  // adaptive: every order <= 64 (3-bit levels)
    const double magic64 = PermSlicer64<2>::uniform(6755399441055744.0);  // 1.5 * 2^52 (complex128)
    if constexpr (FB == 1) {
        int side = 0;
        for (int l = 0; l < cm.n_axis; ++l) side = max(side, (int)axis[l].side);
        small_orders = side <= 8;
#pragma unroll
        for (int q = 0; q < E / 4; ++q) {
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int lid = cm.sc[t + (4 * q + j) * TPS].lut;
                w |= (uint32_t)(sizeof(OP) * (lid < 0 ? kUnusedOrder : lid)) << (8 * j);
            }
            ocode[q] = w;
        }
    } else if constexpr (FB > 1 && !FB_PSK_ONLY) {
        // the FFT output stays unscaled (x sqrt N); SC-OFDM adds the unscaled IFFT (x sqrt N).
        // The reference's 4/16-PSK (psk_m > 0) decide by sector and have no axis tables.
        if (cm.psk_m == 0) pslicer.load(axis[0], scm ? cm.scale * cm.scale : cm.scale);
    } else if (!adaptive) {
        slicer.load(axis[0]);
    }

    const bool array_noise = (FB == 0 || REF) && a.nr != nullptr && noise;
    const int64_t niter = (cm.n_sym + G::SPB - 1) / G::SPB;
    unsigned long long be = 0, se = 0;

    // kept channel samples of local symbol sl.  Past the end the wave reads the last symbol
    // again (its results are neither counted nor stored): an unconditional load, where zeroing
    // the 16 elements cost 32 v_mov_b64 per symbol in complex128.  Zeros when ablated.
    // (symbols of 2 / 4 waves too, N = 2048 / 4096: the row base is wave-uniform when TPS >= 64;
    // RX d 4.67 -> 4.63, e 4.15 -> 4.12 ms per step, profiles/r04h_ab_rxbuf_ch64.txt)
    constexpr bool RX_BUF = F64_FAST && TPS >= 64;
    auto load_sym = [&](int64_t sl, C (&dst)[E]) {
        const C* ys = (const C*)a.y + (sl < cm.n_sym ? sl : cm.n_sym - 1) * ystride;
        if (RX_BUF && !(flags & 16)) {
            // complex128, a symbol per wave: buffer loads off the symbol's row, the lane's byte
            // offset in one VGPR and element i's in the instruction's SGPR offset
            if constexpr (RX_BUF) {
                const __amdgpu_buffer_rsrc_t r = buf_rsrc(ys, (uint32_t)(N * sizeof(C)));
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    dst[i] = buf_load16<C, (bool)OFDM_RX_NT>(r, (uint32_t)t * (uint32_t)sizeof(C),
                                                             (uint32_t)(i * TPS * (int)sizeof(C)));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else if (!(flags & 16)) {
            // issued in element order, the order the noise consumes them: each add then waits
            // for its own load only (left to the scheduler, the N = 4096 complex128 RX issued
            // element 0 thirteenth and waited for 13 of 16 loads before its first add)
#pragma unroll
            for (int i = 0; i < E; ++i) {
                dst[i] = ld_stream<(FB > 0 && OFDM_RX_NT)>(ys + t + i * TPS);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < E; ++i) dst[i] = mk<R>(0, 0);
        }
    };
    for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
        const int64_t sl = it * G::SPB + ls;
        const int64_t sg = cm.sym0 + sl;
        const bool active = sl < cm.n_sym;
        TxBits<FB, TPS, REF> tb;
        // kept channel samples + AWGN; the 1/sqrt(N) of fft(norm="ortho") folded in
        const C* ys = (const C*)a.y + sl * ystride;
        C x[E];
        tb.load(cm, sg, t, W, active && (!(flags & 4) || (noise && !array_noise)));
        load_sym(sl, x);
        if (active && array_noise) {
            const double* nr = a.nr + sg * (N + cp) + (zp ? 0 : cp);
            const double* ni = a.ni + sg * (N + cp) + (zp ? 0 : cp);
#pragma unroll
            for (int i = 0; i < E; ++i) {
                x[i].re += sigma * (R)nr[t + i * TPS];
                x[i].im += sigma * (R)ni[t + i * TPS];
            }
        } else if (active && noise) {
            // noise sample j = i of the lane: a radius word per element, a phase word per four
            // (stream version 3, ofdm_device.hpp "throughput-mode streams")
#pragma unroll
            for (int i = 0; i < E; ++i) {
                if constexpr (sizeof(R) == 4) {
                    tb.g.add_noise(x[i].v, ntab, i);
                } else if constexpr (F64_FAST) {
                    tb.g.add_noise64(x[i].re, x[i].im, ntab64, i);
                } else {
                    tb.g.add_noise_f64(x[i].re, x[i].im, ntab, i);
                }
            }
        }
        if (zp && active) {
            // zero guard: received sample N + k (k < cp) is added onto sample k, noise included
            // (philox mode: the lane's noise samples continue, tail sample i is sample E + i -- the
            // tail samples a lane owns are its first ones, k < cp)
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int k = t + i * TPS;
                if (k < cp) {
                    C v = (flags & 16) ? mk<R>(0, 0) : ys[N + k];
                    if (array_noise) {
                        v.re += sigma * (R)a.nr[sg * (N + cp) + N + k];
                        v.im += sigma * (R)a.ni[sg * (N + cp) + N + k];
                    } else if (noise) {
                        if constexpr (sizeof(R) == 8) {
                            tb.g.add_noise_f64(v.re, v.im, ntab, E + i);
                        } else {
                            const f32x2 n = tb.g.noise(ntab, E + i);
                            v = v + mk<R>(n.x, n.y);
                        }
                    }
                    x[i] = x[i] + v;
                }
            }
        }
        if constexpr (FB == 0) {
#pragma unroll
            for (int i = 0; i < E; ++i) x[i] = cscale(x[i], scale);
        }
        C ecoef[EQ_REG ? E : 1];
        if constexpr (EQ_PRE) {
            if (eq != OFDM_EQ_NONE) {
#pragma unroll
                for (int i = 0; i < E; ++i) ecoef[i] = eqa[t + i * TPS];
            }
        }
        if (!(flags & 2)) fft_sym<R, LOGN, false, FB>(x, row, tw, tt, t);
        // (late loads: the first four here, each later four one slicer group ahead)
        // (buffer loads, the lane's byte offset + element i's in an SGPR: one address VGPR, where
        // 16 hoisted 64-bit addresses spilled at 3 waves per SIMD)
        auto load_coef4 = [&](int q) {
            if constexpr (EQ_LATE) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    ecoef[4 * q + j] = buf_load16<C>(eq_rsrc, (uint32_t)t * (uint32_t)sizeof(C),
                                                     (uint32_t)((4 * q + j) * TPS * (int)sizeof(C)));
            }
        };
        if constexpr (EQ_LATE) load_coef4(0);
        if (FB == 0) sym_sync<TPS>();  // staged words visible to the whole group
        // MMSE noise variance per OFDM symbol (equalization/models.py:39-49)
        R nv = 0;
        if (eq == OFDM_EQ_MMSE) {
            R p = 0;
            if constexpr (sizeof(R) == 4) {
                f32x2 pacc = f32x2{0.f, 0.f};  // (sum Re^2, sum Im^2): one packed FMA per element
#pragma unroll
                for (int i = 0; i < E; ++i) pacc = __builtin_elementwise_fma(x[i].v, x[i].v, pacc);
                p = pacc.x + pacc.y;
            } else {
#pragma unroll
                for (int i = 0; i < E; ++i) p += norm2(x[i]);
            }
            p = group_sum<R, TPS>(p, red);
            if constexpr (FB > 0) p *= scale * scale;  // power of the ortho-scaled spectrum
            nv = cm.gain_mean == 0.0 ? (R)INFINITY : ((p / (R)N) / (R)a.snr_lin) / (R)cm.gain_mean;
        }
        if (scm) {
            // single carrier: equalise every subcarrier, back to time with ifft(ortho)
            if constexpr (EQ_LATE) {
                load_coef4(1);
                load_coef4(2);
                load_coef4(3);
            }
#pragma unroll
            for (int i = 0; i < E; ++i)
                if (eq != OFDM_EQ_NONE)
                    x[i] = eq_apply(x[i], t + i * TPS, nv, &ecoef[EQ_REG ? i : 0]);
            sym_sync<TPS>();  // the forward FFT has read the row
            if constexpr (FB > 1) {
                fft_sym<R, LOGN, true, FB>(x, row, tw, tt + TTS, t);  // 1/N in the slicer
            } else {
                fft_reg<R, LOGN, true, false>(x, row, tw, tw + 64, t, tt);
#pragma unroll
                for (int i = 0; i < E; ++i) x[i] = cscale(x[i], scale);
            }
        }
        if (active && !(flags & 8)) {
            const int64_t sbit = sg * cm.bps;
            const bool all_valid = FB > 1 || sbit + cm.bps <= a.n_valid_bits;
            uint32_t bes = 0, ses = 0;
            auto equalized = [&](int i) {
                if (scm || eq == OFDM_EQ_NONE) return x[i];  // single carrier: equalised before the IFFT
                return eq_apply(x[i], t + i * TPS, nv, &ecoef[EQ_REG ? i : 0]);
            };
            // MMSE in complex128: conj(H) v / (|H|^2 + nv) of a lane word's four elements, the four
            // reciprocals from one (MMSE_BATCH)
            // (sc non-null: z = conj(H) v unscaled and sc[j] = 1 / (|H|^2 + nv), the slicer folding the
            // scale into its level multiplier: one product per element instead of two)
            auto mmse4 = [&](int q, C(&z)[4], R* sc) {
                C c[4];
                R dn[4], inv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    c[j] = EQ_LDS ? eqt[t + (4 * q + j) * TPS] : ecoef[EQ_REG ? 4 * q + j : 0];
                    dn[j] = c[j].re * c[j].re + c[j].im * c[j].im + nv;
                }
                const R p01 = dn[0] * dn[1], p012 = p01 * dn[2], p = p012 * dn[3];
                if (__builtin_expect(p >= (R)1e-280 && p <= (R)1e280, 1)) {
                    R r = recip<R>(p);  // 1 / (d0 d1 d2 d3)
                    inv[3] = r * p012;
                    r *= dn[3];  // 1 / (d0 d1 d2)
                    inv[2] = r * p01;
                    r *= dn[2];  // 1 / (d0 d1)
                    inv[1] = r * dn[0];
                    inv[0] = r * dn[1];
                } else {  // a zero, infinite or extreme factor: one reciprocal each
#pragma unroll
                    for (int j = 0; j < 4; ++j) inv[j] = recip<R>(dn[j]);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (sc) {
                        z[j] = cmul(x[4 * q + j], c[j]);
                        sc[j] = inv[j];
                    } else {
                        z[j] = cscale(cmul(x[4 * q + j], c[j]), inv[j]);
                    }
                }
            };
            if constexpr (FB == 1) {
                // four elements per lane word, each through its subcarrier's order (the codes
                // are made opaque per symbol: the order-table reads stay inside the loop)
                static_for<0, E / 4>([&](auto Q) {
                    constexpr int q = Q;
                    if constexpr (EQ_LATE && q + 1 < E / 4) load_coef4(q + 1);
                    C z[4];
                    const OP* op[4];
                    uint32_t oc = ocode[q];
                    asm volatile("" : "+v"(oc));
                    R sc[4] = {1, 1, 1, 1};  // the MMSE scale per element, folded into the slicer
                    if (MMSE_BATCH) {
                        mmse4(q, z, sc);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) z[j] = equalized(4 * q + j);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        op[j] = (const OP*)((const unsigned char*)ordt + ((oc >> (8 * j)) & 0xFFu));
                    uint32_t d;
                    if constexpr (sizeof(R) == 8)
                        d = small_orders ? adaptive_diff64<true, MMSE_BATCH>(z, op, lane_word(tb.lane, q), magic64, sc)
                                         : adaptive_diff64<false, MMSE_BATCH>(z, op, lane_word(tb.lane, q), magic64, sc);
                    else
                        d = small_orders ? adaptive_diff<true>(z, op, lane_word(tb.lane, q))
                                         : adaptive_diff<false>(z, op, lane_word(tb.lane, q));
                    ses += PermSlicer<8>::nonzero_bytes(d);
                    if (!all_valid) {
                        // a trailing partial byte of the run is not compared (constellation/
                        // adaptive.py:259-263): keep the first bits (MSB first) of the valid range.
                        static_assert(sizeof(ScInfo) == 8, "ScInfo is one 8-byte word");
                        gptr<const uint64_t> scp = (gptr<const uint64_t>)cm.sc;
                        uint32_t vm = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const ScInfo sc = __builtin_bit_cast(ScInfo, (uint64_t)scp[t + (4 * q + j) * TPS]);
                            if (sc.lut < 0) continue;
                            const int64_t nvb = a.n_valid_bits - (sbit + sc.bitoff);
                            const int keep = nvb <= 0 ? 0 : (nvb >= sc.bits ? sc.bits : (int)nvb);
                            vm |= (((1u << keep) - 1u) << (sc.bits - keep)) << (8 * j);
                        }
                        d &= vm;
                    }
                    bes += __popc(d);
                });
            } else if constexpr (FB > 0) {
                // four elements per lane word: slice, look up, compare, count
                static_for<0, E / 4>([&](auto Q) {
                    constexpr int q = Q;
                    if constexpr (EQ_LATE && q + 1 < E / 4) {
                        if (!scm) load_coef4(q + 1);  // (single carrier: loaded before its equaliser)
                    }
                    C z[4];
                    R sc[4];  // MMSE_BATCH: the scale per element, folded into the QAM slicer
                    const bool fold = MMSE_BATCH && !scm;
                    if (fold) {
                        mmse4(q, z, sc);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) z[j] = equalized(4 * q + j);
                    }
                    uint32_t d = 0;
                    // the reference's M-PSK (M <= 32: 4- and 16-PSK share the QAM kernels'
                    // FB = 2 / 4, 8- and 32-PSK have FB = 3 / 5 to themselves): sector
                    // decisions (psk_decide); compiled out of the 64/256-QAM kernels
                    if (FB_PSK_ONLY || (FB <= 4 && cm.psk_m > 0)) {
                        uint32_t r = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) r |= psk_decide(fold ? cscale(z[j], sc[j]) : z[j], cm) << (8 * j);
                        d = r ^ (lane_word(tb.lane, q) & PermSlicer<FB>::BYTE_MASK);
                    } else if constexpr (!FB_PSK_ONLY) {
                        if constexpr (MMSE_BATCH) {
                            d = fold ? pslicer.diff_scaled(z, sc, lane_word(tb.lane, q)) : pslicer.diff(z, lane_word(tb.lane, q));
                        } else {
                            d = pslicer.diff(z, lane_word(tb.lane, q));
                        }
                    }
                    bes += __popc(d);
                    ses += PermSlicer<FB>::nonzero_bytes(d);
                });
            } else {
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    const int k = t + i * TPS;
                    const C v = equalized(i);
                    if (sl < a.z_keep) ((C*)a.z_out)[sl * N + k] = v;
                    uint32_t ridx;
                    int b, off;
                    if (adaptive) {
                        const ScInfo sc = cm.sc[k];
                        if (sc.lut < 0) continue;
                        b = sc.bits;
                        off = sc.bitoff;
                        // PSK orders (constellation/adaptive.py:130-265 with the PSK base mapper):
                        // the nearest point of the subcarrier's own LUT
                        ridx = nn ? nn_decide<R>(v, cm, axis[sc.lut].lut_off, 1 << sc.bits) : slice<R>(v, axis[sc.lut]);
                    } else {
                        b = cm.b;
                        off = k * b;
                        ridx = nn ? nn_decide<R>(v, cm, 0, cm.lut_len) : slicer(v);
                    }
                    uint32_t d = ridx ^ tb.generic(i, b, off);
                    ses += d != 0u;
                    if (!all_valid) {
                        const int64_t nvb = a.n_valid_bits - (sbit + off);
                        const int keep = nvb <= 0 ? 0 : (nvb >= b ? b : (int)nvb);
                        d &= ((1u << keep) - 1u) << (b - keep);
                    }
                    bes += __popc(d);
                }
            }
            be += bes;
            se += ses;
        }
        sym_sync<TPS>();  // W and the FFT row are rewritten by the next symbol
    }
    be = block_sum<unsigned long long, BLK>(be, redc);
    se = block_sum<unsigned long long, BLK>(se, redc);
    if (threadIdx.x == 0) {
        if (be) atomicAdd((unsigned long long*)&a.counters[0], be);
        if (se) atomicAdd((unsigned long long*)&a.counters[1], se);
    }
}

}  // namespace ofdm
