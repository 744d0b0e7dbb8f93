"""bits_generation operators (mirrors ofdm_based_systems.bits_generation of the reference)."""
