// complex64 (throughput mode) instantiation of the operator launchers; the fused TX / RX
// launchers are in ofdm_kernels_f32_tx.hip / ofdm_kernels_f32_rx.hip (parallel compile).
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_OPS(float)
}  // namespace ofdm
