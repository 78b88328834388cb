"""CPU oracle (test infrastructure only) -- see oracle/nmgp_oracle.py header."""
