"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see ws_oracle.py header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product (gev_amd/) never does.
"""
