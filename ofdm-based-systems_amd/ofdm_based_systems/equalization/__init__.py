"""equalization operators (mirrors ofdm_based_systems.equalization of the reference)."""
