"""CPU oracle of the reference codec path — test infrastructure only (see gcodec_oracle.c)."""
