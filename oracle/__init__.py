"""CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / reported CPU baseline.  The product path
(libspi_hip.so and the starpu-inference-server_amd package) never imports it.
"""
