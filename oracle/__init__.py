"""Test infrastructure: CPU oracle for the RX per-frame transform (see pn_oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
