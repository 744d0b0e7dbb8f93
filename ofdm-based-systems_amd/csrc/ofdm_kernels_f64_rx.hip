// complex128 instantiation of the fused RX launcher (generic and throughput k_rx).
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_RX(double)
}  // namespace ofdm
