"""CPU oracle package (test infrastructure only)."""
