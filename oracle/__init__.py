"""ORACLE — test infrastructure only (CPU restatement + reference-built checkers).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product (funasr_amd) never imports it.
"""
