"""TEST INFRASTRUCTURE ONLY (the parity oracle). Importable from tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() — never from the product package avsr_amd/."""
