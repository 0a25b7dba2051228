"""ORACLE — test infrastructure only (see oracle/kruskal.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker. The product package (distributed_ghs_implementation_amd) never imports
it; tests/test_no_oracle_in_product.py enforces that.
"""
