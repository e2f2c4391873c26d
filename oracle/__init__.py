"""TEST INFRASTRUCTURE ONLY — the parity oracle for halo's rx parse path.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package (halo_amd) never imports this.
"""
