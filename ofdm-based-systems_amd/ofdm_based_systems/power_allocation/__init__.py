"""power_allocation operators (mirrors ofdm_based_systems.power_allocation of the reference)."""
