"""CPU oracle for the ComE SGNS hot path -- test infrastructure only (see oracle/oracle.py)."""
