"""pipsort_amd — MI355X-native posterior-calculation engine for PIPSORT.

The product is the C-ABI library lib/libpipsort_engine.so (HIP kernels for
gfx950, include/pipsort_engine.h) and the drop-in bin/PIPSORT executable.
This package adds the ctypes binding (engine.py) and the SYN-v1 locus
generator (synth.py) used by tests and bench.py.
"""
from .engine import (EngineError, PostCal, Seam, Accumulators, device_count, load_library,  # noqa: F401
                     seam_from_arrays, psd_shift, lowrank_study, sym_eigen, LIB_PATH, PIPSORT_BIN)

__all__ = ["EngineError", "PostCal", "Seam", "Accumulators", "device_count", "load_library",
           "seam_from_arrays", "psd_shift", "lowrank_study", "sym_eigen", "LIB_PATH", "PIPSORT_BIN"]
