"""ORACLE — test infrastructure only.

CPU restatements of the reference hot path used as the parity checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never imported by the product
package (ebsd-vae_amd/latice), which has no CPU fallback.
"""
