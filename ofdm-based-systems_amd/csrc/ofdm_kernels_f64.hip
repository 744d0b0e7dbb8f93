// complex128 instantiation of the operator launchers (parity mode / operator API), plus the
// precision-independent support kernels; the fused TX / RX launchers are in
// ofdm_kernels_f64_tx.hip / ofdm_kernels_f64_rx.hip (parallel compile).
#define OFDM_SUPPORT_KERNELS 1
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_OPS(double)

hipError_t launch_finalize(const double* partials, int nblocks, int nfields, int max_mask,
                           double* stats, hipStream_t s) {
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kBlock), 0, s, partials, nblocks, nfields, max_mask, stats);
    return hipGetLastError();
}

hipError_t launch_finalize_tx(const double* partials, int nblocks, double* stats, hipStream_t s) {
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_finalize_tx, dim3(1), dim3(kBlock), 0, s, partials, nblocks, stats);
    return hipGetLastError();
}

hipError_t launch_nn_classify(const double* lut, int m, const double* z, int64_t n, int64_t* idx,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_nn_classify, dim3(clamp_grid((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       lut, m, z, n, idx);
    return hipGetLastError();
}

hipError_t launch_noise_radius(const uint32_t* w, int64_t n, float* r, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();  // stale errors were reported by their own calls
    hipLaunchKernelGGL(k_noise_radius, dim3(clamp_grid((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w, n, r);
    return hipGetLastError();
}
}  // namespace ofdm
