"""CPU oracle (test infrastructure only -- see hashnerf_oracle.py header)."""
