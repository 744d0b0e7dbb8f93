// complex64 instantiation of the fused TX launcher (every k_tx specialisation).
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_TX(float)
}  // namespace ofdm
