"""CPU oracle (test infrastructure only; see oracle/rs_oracle.c)."""
