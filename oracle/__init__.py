"""ORACLE -- test infrastructure only (see gine_cpu.py).  Imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product path."""
