"""ORACLE (test infrastructure only): CPU fp32 restatement of the reference MGN path.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Pinned bit-exactly to golden vectors from the reference's own code (tests/golden/).
"""
