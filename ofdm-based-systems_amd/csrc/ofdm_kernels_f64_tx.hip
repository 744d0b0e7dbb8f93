// complex128 instantiation of the fused TX launcher (generic and throughput k_tx).
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE_TX(double)
}  // namespace ofdm
