"""MI355X-native drop-in for the OFDM modem path of JomarJunior/ofdm-based-systems.

Same module layout and operator API as the reference package
(``ofdm_based_systems.<operator>.models``); the arithmetic runs in the gfx950 HIP
kernels of ``_lib/libofdm_hip.so`` (C ABI: ``include/ofdm_hip.h``).
"""

__version__ = "0.1.0"
