"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's NCF hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker (or as the timed CPU
baseline).  The product path in ``movierecommender-tf-trt_amd/movierec`` never
imports it: without the HIP library the product raises.
"""
