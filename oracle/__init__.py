"""CPU oracle for the LGM render path -- TEST INFRASTRUCTURE ONLY (see raster_oracle.c header).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package."""
