"""serial_parallel operators (mirrors ofdm_based_systems.serial_parallel of the reference)."""
