"""configuration operators (mirrors ofdm_based_systems.configuration of the reference)."""
