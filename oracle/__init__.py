"""ORACLE — test infrastructure only, never product code.

CPU restatement of the reference inference path (yazdayy/sound-event-detection,
``/root/reference``) used as the parity checker for the HIP path in
``sound-event-detection_amd/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import anything from this package, and
only as the checker / the timed CPU baseline — the product path never calls it.

Pinning: ``oracle/make_golden.py`` imports the reference itself (Python, run in
the build container with the test-only ``oracle/refshim`` stand-ins for the
absent librosa / sed_eval / h5py / prettytable) and writes the committed
fixtures in ``tests/golden/``; ``tests/test_oracle_golden.py`` checks this
restatement against them.
"""
