"""CPU oracle (test infrastructure only): see vx_oracle.h / oracle.py."""
