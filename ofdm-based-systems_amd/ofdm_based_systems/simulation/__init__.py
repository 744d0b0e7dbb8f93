"""simulation operators (mirrors ofdm_based_systems.simulation of the reference)."""
