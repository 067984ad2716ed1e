"""The reference's own module name, leading space included (/root/reference/ polynomial.py:1-5),
so that a caller's ``importlib.import_module(" polynomial")`` works unchanged with this directory
on ``sys.path`` in place of the reference's.  Everything lives in ``polynomial.py``; this file
only re-exports it (``poly_add`` plus the star-import chain ``primitive`` -> ``arithmetic``)."""
from polynomial import *  # noqa: F401,F403
from polynomial import poly_add  # noqa: F401  (explicit: the reference's one L2 entry point)
