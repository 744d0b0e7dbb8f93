// complex64 instantiation of the fused RX launcher (every k_rx specialisation).
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_RX(float)
}  // namespace ofdm
