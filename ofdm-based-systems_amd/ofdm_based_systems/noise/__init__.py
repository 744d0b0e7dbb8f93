"""noise operators (mirrors ofdm_based_systems.noise of the reference)."""
