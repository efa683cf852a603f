"""ORACLE package — test infrastructure only.

CPU restatements of the reference's hot path (BundleSDF nerf_runner.py and its
mycuda extensions) used as the parity checker by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg. The product
package bundlesdf_amd never imports anything from here.
"""
