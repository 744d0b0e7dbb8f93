"""modulation operators (mirrors ofdm_based_systems.modulation of the reference)."""
