"""CPU oracle package — test infrastructure only (see fm_oracle.py header)."""
