// complex64 (throughput mode) instantiation of every kernel launcher.
#include "ofdm_kernels_inst.hpp"

namespace ofdm {
OFDM_INSTANTIATE(float)
}  // namespace ofdm
