"""CPU oracle for the KGMT hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, as the parity checker or as the timed CPU baseline.  The product
package ``cudasbmp_amd`` never imports it.
"""
