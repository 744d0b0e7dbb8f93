"""prefix operators (mirrors ofdm_based_systems.prefix of the reference)."""
