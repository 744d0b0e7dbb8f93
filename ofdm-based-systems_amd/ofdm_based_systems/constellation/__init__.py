"""constellation operators (mirrors ofdm_based_systems.constellation of the reference)."""
