"""TEST INFRASTRUCTURE ONLY -- the CPU checker.  See oracle/gclmul_oracle.c."""
