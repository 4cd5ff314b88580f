"""Parity oracle (test infrastructure only): CPU restatement of the reference MEPOL path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
