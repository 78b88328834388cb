"""Drop-ins for the reference package ``code/SIM_code/Utility`` (legacy kernel / Kronecker signatures)."""
