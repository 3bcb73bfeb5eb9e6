"""CPU parity oracle (TEST INFRASTRUCTURE ONLY) -- see oracle/oracle.py."""
