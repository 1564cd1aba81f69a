"""CPU oracle for the IKF scan-matching core — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  Parity status: unpinned by reference outputs (the
reference cannot be built here and ships no tests); see slio_oracle.cpp.
"""
