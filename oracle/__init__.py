"""CPU oracle — test infrastructure only (see each module's header).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
