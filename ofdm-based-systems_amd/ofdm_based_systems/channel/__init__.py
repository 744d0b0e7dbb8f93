"""channel operators (mirrors ofdm_based_systems.channel of the reference)."""
