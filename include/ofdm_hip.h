/*
 * ofdm_hip.h -- C ABI of libofdm_hip.so, the MI355X (gfx950) implementation of the
 * per-symbol OFDM modem path of JomarJunior/ofdm-based-systems.
 *
 * Boundary: the reference is pure Python/NumPy; its "operator" interfaces
 * (src/ofdm_based_systems/<pkg>/models.py ABCs) are called from
 * Simulation.run (simulation/models.py:214-818).  This library exports the
 * arithmetic those operators perform; the Python package
 * ofdm-based-systems_amd/ofdm_based_systems mirrors the reference API and calls
 * these entry points through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every buffer argument is a DEVICE pointer owned by the caller (PyTorch
 *    allocates it).  The library owns only plan-scoped constant tables and a
 *    small partial-sum workspace per stream the plan is used on.
 *  - Complex arrays are interleaved (re, im) in the plan's precision:
 *    OFDM_F32 -> float2 (complex64), OFDM_F64 -> double2 (complex128).
 *  - Every call is asynchronous on the given hipStream_t (NULL = default stream);
 *    no call synchronises the device.  One plan may be used on several streams
 *    whose work overlaps (the reductions keep one workspace per stream); it must
 *    not be used on the SAME stream from two host threads at once.
 *  - Return 0 on success, a negative OFDM_E* code on failure; the message is in
 *    ofdm_last_error() (thread-local).  Nothing throws across the ABI.
 *  - Bits are packed MSB-first in bytes (simulation/models.py:59-69,
 *    constellation/models.py:227-233).
 */
#ifndef OFDM_HIP_H
#define OFDM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFDM_ABI_VERSION 5

#define OFDM_OK 0
#define OFDM_E_INVALID (-1)  /* bad argument / unsupported shape          */
#define OFDM_E_HIP (-2)      /* HIP runtime error                          */
#define OFDM_E_ALLOC (-3)    /* device allocation failed (plan creation)   */

enum ofdm_precision { OFDM_F32 = 0, OFDM_F64 = 1 };
/* equalization/models.py:22-68 */
enum ofdm_equalizer { OFDM_EQ_NONE = 0, OFDM_EQ_ZF = 1, OFDM_EQ_MMSE = 2 };

/* prefix/models.py:29-113 (NoPrefixScheme = OFDM_PREFIX_CYCLIC with cp = 0) */
enum ofdm_prefix { OFDM_PREFIX_CYCLIC = 0, OFDM_PREFIX_ZERO = 1 };
/* modulation/models.py:19-91: OFDMModulator / SingleCarrierOFDMModulator */
enum ofdm_modulator { OFDM_MOD_OFDM = 0, OFDM_MOD_SC = 1 };

typedef struct ofdm_plan_s* ofdm_plan_t;

/*
 * Plan descriptor.  One plan = one (N, prefix, channel, constellation, equaliser)
 * configuration, i.e. what Simulation.run builds once per SNR point
 * (simulation/models.py:248-275, :399-404) or what one operator object holds.
 */
typedef struct ofdm_desc {
    int32_t n_fft;       /* N = num_subcarriers, power of two in [1, 4096]        */
    int32_t cp;          /* guard length (IPrefixScheme.prefix_length)            */
    int32_t prefix;      /* enum ofdm_prefix: cyclic prefix or zero padding       */
    int32_t precision;   /* enum ofdm_precision                                   */
    int32_t equalizer;   /* enum ofdm_equalizer                                   */
    /* Constellations: a pool of LUTs (interleaved re/im doubles, exactly the
       reference's QAMConstellationMapper.constellation arrays) and, per
       subcarrier, which LUT it uses.  Fixed mode: one LUT, sc_lut == NULL.
       Adaptive mode (constellation/adaptive.py:16-91): n_luts LUTs and
       sc_lut[k] in [-1, n_luts) with -1 = inactive subcarrier (order 0). */
    int32_t n_luts;              /* 0 = no constellation in this plan, at most 8   */
    const int32_t* lut_orders;   /* [n_luts] orders (powers of two 2..256)         */
    const double* lut_pool;      /* concatenated LUTs, sum(lut_orders) complex      */
    const int32_t* sc_lut;       /* [n_fft] or NULL                                 */
    /* Channel: raw CIR (h_raw).  The plan normalises it to unit power for the
       convolution (channel/models.py:37-44) and computes the equaliser response
       fft(h_raw, N) on the device (simulation/models.py:264). */
    int32_t n_taps;              /* 0 = no channel in this plan                     */
    const double* h_raw;         /* [n_taps] complex                                */
    /* Optional explicit equaliser response (IEqualizator(channel_frequency_response=H)),
       [n_fft] complex; overrides the response derived from h_raw. */
    const double* H;
    /* enum ofdm_modulator (ABI 2): the fused path's modulator (ofdm_tx / ofdm_rx). */
    int32_t modulator;
} ofdm_desc;

/*
 * Whole-stream statistics of the fused transmitter (ABI 3), one device record per run, zeroed
 * by the caller and accumulated by every ofdm_tx of the run.  The AWGN power is the mean of |y|^2
 * over the whole serial stream (noise/models.py:14); so that it -- and sigma -- does not depend on
 * how a run is batched or sharded over GPUs, the sum is kept EXACTLY: every lane's share of one
 * OFDM symbol is rounded once to 2^-40 fixed point and added as 32-bit limbs to 64-bit integers,
 * power_fx[0] + 2^32 power_fx[1] (units of 2^-40).  Records of several ranks combine by adding
 * the limbs (any order: integer arithmetic), then power_fx[1] += power_fx[0] >> 32,
 * power_fx[0] &= 2^32 - 1, power_sum = power_fx[1] 2^-8 + power_fx[0] 2^-40 (IEEE double).
 */
typedef struct ofdm_stats {
    double power_sum;     /* sum |y|^2 over all N+cp samples, = value of power_fx            */
    double x_power_sum;   /* sum |x|^2 over the modulated samples incl. the guard          */
    double x_peak;        /* max |x|^2 (simulation/models.py:519-522)                       */
    int64_t power_fx[2];  /* sum |y|^2 in 2^-40 fixed point, 32-bit limbs (see above)       */
} ofdm_stats;

typedef struct ofdm_plan_info {
    int32_t n_fft, cp, precision, equalizer, n_taps;
    int32_t bits_per_ofdm_symbol; /* sum of bits over active subcarriers            */
    int32_t bits_per_subcarrier;  /* uniform b in fixed mode, -1 in adaptive mode   */
    int32_t adaptive;
    double channel_gain_mean;     /* mean |H|^2 (equalization/models.py:46)          */
} ofdm_plan_info;

int ofdm_abi_version(void);
const char* ofdm_last_error(void);

int ofdm_plan_create(ofdm_plan_t* plan, const ofdm_desc* desc, void* stream);
int ofdm_plan_destroy(ofdm_plan_t plan);
int ofdm_plan_get_info(ofdm_plan_t plan, ofdm_plan_info* info);

/* The plan's channel response H = fft(h_raw, N) (or the explicit desc.H) and, if
   gains != NULL, |H|^2 (ChannelModel.get_frequency_response / get_gains,
   channel/models.py:26-35).  H: device complex128 [N]; gains: device double [N]. */
int ofdm_plan_response(ofdm_plan_t plan, void* stream, double* H, double* gains);

/* ---------------------------------------------------------------- operators
 * Drop-in arithmetic for the reference's operator objects.                    */

/* In-place batched FFT of `batch` contiguous rows of N (norm="ortho").
   Replaces np.fft.fft / np.fft.ifft(axis=1, norm="ortho") in
   modulation/models.py:32 and :46-48. */
int ofdm_fft(ofdm_plan_t plan, void* stream, void* data, int64_t batch, int32_t inverse);

/* QAMConstellationMapper.encode (constellation/models.py:220-249) and
   AdaptiveConstellationMapper.encode (constellation/adaptive.py:130-201):
   n_bytes packed bytes -> n_out complex symbols.  Fixed mode: symbol e uses bits
   [e*b, e*b+b), bits past the input are zero (padding :235-237).  Adaptive mode:
   n_out = S*N, subcarrier k of OFDM symbol s uses bits at s*sum(b)+off[k]; inactive
   subcarriers are 0+0j. */
int ofdm_map(ofdm_plan_t plan, void* stream, const uint8_t* bytes, int64_t n_bytes,
             int64_t n_out, void* symbols);

/* QAMConstellationMapper.decode (constellation/models.py:251-295): nearest LUT point
   by brute-force |z - C_m| argmin (first index on ties, NNClassifier :19-27), bits
   packed MSB-first; fixed mode writes ceil(n*b/8) bytes (tail zero-padded), adaptive
   mode floor(S*sum(b)/8) bytes (constellation/adaptive.py:257-265). */
int ofdm_demap(ofdm_plan_t plan, void* stream, const void* z, int64_t n, uint8_t* bytes);

/* QAMConstellationMapper.decode (constellation/models.py:251-295) or
   AdaptiveConstellationMapper.decode (constellation/adaptive.py:203-265) followed by
   Simulation.run's error count (simulation/models.py:596-606), fused: Z is (n_sym, N)
   equalised symbols in the plan precision, tx_bits the packed bits of those symbols (OFDM
   symbol s from bit s*bits_per_ofdm_symbol, MSB first).  Nearest point per subcarrier as
   ofdm_demap; counters[0] += bit errors (every bit in fixed mode, whole bytes of the run in
   adaptive mode, as the reference's decode), counters[1] += symbol errors.  counters: 2 device
   uint64 accumulated atomically. */
int ofdm_demap_count(ofdm_plan_t plan, void* stream, const void* Z, const uint8_t* tx_bits,
                     int64_t n_sym, uint64_t* counters);

/* NNClassifier.classify (constellation/models.py:19-27) for an arbitrary LUT of M
   complex128 points: idx[i] = argmin_m |z_i - lut_m| (first on ties).  z is complex128. */
int ofdm_nn_classify(void* stream, const double* lut, int32_t m, const void* z, int64_t n,
                     int64_t* idx);

/* Throughput-mode noise radius (ABI 4; ABI 5: stream version 3, the radius takes the whole word):
   radius[i] = sqrt(32 - log2(float(words[i] | 1))),
   evaluated exactly as the fused receivers evaluate it for every lane word (the float32 hardware
   log2 / square root: the one step of the stream definition, csrc/ofdm_device.hpp noise_radius,
   that IEEE arithmetic does not pin).  AWGNoiseModel.add_noise's Gaussian (noise/models.py:19-21)
   in throughput mode is sigma sqrt(2 ln 2) radius (cos, sin)(phase); the checker
   (oracle/philox_streams.py) takes these radii to restate the receivers' noise bit for bit.
   words: device uint32 [n]; radius: device float [n]. */
int ofdm_noise_radius(void* stream, const uint32_t* words, int64_t n, float* radius);

/* OFDMModulator.modulate (modulation/models.py:27-39): x[s] = [cp | ifft(X[s], ortho)]
   (zero padding: [ifft(X[s], ortho) | 0...0]), X is (n_sym, N), x is (n_sym, N+cp). */
int ofdm_modulate(ofdm_plan_t plan, void* stream, const void* X, int64_t n_sym, void* x);

/* OFDMModulator.demodulate (modulation/models.py:41-55): strip cp (zero padding: fold
   the tail onto the head, prefix/models.py:74-101), fft(ortho), per-row equalise
   (equalization/models.py:22-68).  yt is (n_sym, N+cp), Z (n_sym, N). */
int ofdm_demodulate(ofdm_plan_t plan, void* stream, const void* yt, int64_t n_sym,
                    double snr_db, void* Z);

/* IEqualizator.equalize applied to n_rows rows of N (equalization/models.py:22-68). */
int ofdm_equalize(ofdm_plan_t plan, void* stream, const void* Y, int64_t n_rows,
                  double snr_db, void* Z);

/* ChannelModel.transmit convolution (channel/models.py:46-55): y = conv(s, h/|h|)[:len].
   If power_sum != NULL, *power_sum (device double) += sum |y|^2. */
int ofdm_channel(ofdm_plan_t plan, void* stream, const void* s, int64_t len, void* y,
                 double* power_sum);

/* AWGNoiseModel.add_noise (noise/models.py:13-22) with caller-supplied standard normals
   (the reference's legacy-RNG draws, real array first):
   y += sqrt((power_sum/len) / 10^(snr/10) / 2) * (nr + j*ni).  power_sum is a device
   double holding sum |y|^2 over the len samples (from ofdm_channel or ofdm_power). */
int ofdm_awgn(ofdm_plan_t plan, void* stream, void* y, int64_t len, const double* nr,
              const double* ni, const double* power_sum, double snr_db);

/* *power_sum += sum |y|^2 over len samples (device double). */
int ofdm_power(ofdm_plan_t plan, void* stream, const void* y, int64_t len, double* power_sum);

/* ---------------------------------------------------------------- fused hot path
 * Simulation.run's data path (simulation/models.py:454-606) in two kernels.
 *
 * Bit source: `bits` != NULL -> packed tx bytes of the WHOLE run (OFDM symbol s
 * starts at bit s*bits_per_ofdm_symbol), e.g. the reference's PCG64 bytes
 * (parity mode).  bits == NULL -> throughput mode: bits and noise from the
 * counter-based lane streams keyed by (seed, global symbol) (stream version 3 since ABI 5:
 * Philox4x32-10 seeding MWC64X; definition in csrc/ofdm_device.hpp, restated in
 * oracle/philox_streams.py).  Caller bits on the bench shapes (complex128 OFDM, cyclic prefix,
 * 64-QAM at N = 1024, adaptive square-QAM loading at N = 2048 or 256-QAM at N = 4096) run the
 * throughput kernels with the bit -- and in
 * ofdm_rx, with nr/ni and no z_out, the noise -- source swapped; other shapes the generic kernel.  n_sym = 0 is an empty call (returns 0, launches nothing).
 *
 * ofdm_tx: for global OFDM symbols [sym0, sym0+n_sym): map -> IFFT(ortho) (OFDM) or
 *   nothing (single carrier) -> cyclic prefix or zero guard -> linear convolution with
 *   the normalised CIR across symbol boundaries (channel/models.py:52-55).  Writes the
 *   channel-output samples of each symbol to y[(s-sym0)*ystride + n], ystride = N (the
 *   post-prefix samples) or N + cp with zero padding (all samples: the receiver
 *   overlap-adds the guard); y may be NULL (power pass only).  Accumulates into the device
 *   record stats (ofdm_stats): sum|y|^2 over all N+cp samples (noise/models.py:14) in exact
 *   fixed point, sum|x|^2 and max|x|^2 over the modulated samples incl. the guard
 *   (simulation/models.py:519-522).
 *
 * ofdm_rx: adds AWGN with sigma^2 = (stats->power_sum/total_samples)/10^(snr/10) (noise_on=0:
 *   no noise), strips the prefix (or overlap-adds the zero guard, prefix/models.py:69-101),
 *   FFT(ortho), equalises (MMSE noise variance per OFDM symbol, equalization/models.py:
 *   39-49), IFFT(ortho) for single carrier, decides the nearest constellation point
 *   (per-axis slicer for square QAM, brute force over the LUT otherwise) and compares
 *   against the tx bits: counters[0] += bit errors over global bit positions
 *   < n_valid_bits, counters[1] += symbol errors (simulation/models.py:596-606).
 *   Noise: nr/ni != NULL -> the reference's normals for the whole serial stream
 *   (sample s*(N+cp)+m); NULL -> the throughput-mode lane streams, Box-Muller.
 *   z_out (optional): the equalised symbols of the first z_keep OFDM symbols of this
 *   call, (z_keep, N) complex -- the results' received_symbols (simulation/models.py:618).
 */
int ofdm_tx(ofdm_plan_t plan, void* stream, const uint8_t* bits, uint64_t seed, int64_t sym0,
            int64_t n_sym, void* y, ofdm_stats* stats);

int ofdm_rx(ofdm_plan_t plan, void* stream, const void* y, const double* nr, const double* ni,
            uint64_t seed, const ofdm_stats* stats, int64_t total_samples, double snr_db,
            int32_t noise_on, const uint8_t* bits, int64_t sym0, int64_t n_sym,
            int64_t n_valid_bits, uint64_t* counters, void* z_out, int64_t z_keep);

#ifdef __cplusplus
}
#endif

#endif /* OFDM_HIP_H */
