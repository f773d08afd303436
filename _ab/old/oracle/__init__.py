"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (Stamatios-Korres/recommendation_Gans),
used as the parity checker.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import anything from here; the product
package (``recommendation_gans_amd``) never does, and fails loudly when its HIP
library is missing instead of falling back to this code.

Pinning: every function here is checked against golden vectors produced by
importing the reference itself in the build container (tests/golden/make_golden.py,
fixtures in tests/golden/*.npz; tests/test_oracle_golden.py).
"""
