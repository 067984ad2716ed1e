"""fhecore: MI355X-native (gfx950) FHE polynomial-arithmetic core (Python host layer).

See include/fhecore.h for the C ABI and DESIGN.md for the kernels.  Reference-compatible
module-level names live one directory up (arithmetic.py, primitive.py, polynomial.py).
"""
from ._capi import FheError, LIB_PATH, load  # noqa: F401
from .context import Context, Graph, default_params, gen_moduli, to_device, to_host  # noqa: F401

__all__ = ["Context", "FheError", "Graph", "LIB_PATH", "default_params", "gen_moduli", "load", "to_device",
           "to_host"]
