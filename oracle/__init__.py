"""TEST INFRASTRUCTURE ONLY — the CPU oracle for rogtk_amd's hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package. The product (rogtk_amd) never imports it.
"""
