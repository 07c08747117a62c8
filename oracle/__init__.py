"""CPU oracle for the batched pusher-slider NMPC hot path (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker.  Parity against acados is UNPINNED (see
qsp_oracle.c header and DESIGN.md).
"""
