"""Oracle package: CPU restatements of the reference's BLS12-381 hot path.

TEST INFRASTRUCTURE ONLY.  Imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, as the
checker -- never by the product package ``teku_amd``.
"""
