"""CPU oracle: a restatement of the reference's hot-path algorithms.

TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline. The product path
(long_context_biomedical_imaging_amd/) never imports it and has no CPU fallback.

Pinned by: tests/golden/*.npz, produced by tools/gen_golden.py from the reference source itself
(imported in the build container with third-party stand-ins, tools/ref_standins.py), and checked in
tests/test_oracle_golden.py.
"""
