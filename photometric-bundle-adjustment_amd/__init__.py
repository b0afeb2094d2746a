"""MI355X photometric bundle-adjustment residual/Jacobian engine (package root).

The compute path is the HIP library ``csrc/libpba.so`` reached through the C ABI in ``include/pba.h``;
``engine.py`` is the Python-side binding used by tests and bench.  Importing this package does not load
the library; creating an :class:`engine.Engine` does, and fails loudly if it is missing.
"""
