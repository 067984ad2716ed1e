"""Drop-in for the reference's ``' polynomial'`` module (/root/reference/ polynomial.py:1-5).

The reference file name starts with a space.  Both names work with this directory on sys.path:
``import polynomial`` (this file) and the reference's own ``importlib.import_module(' polynomial')``
(`` polynomial.py`` beside it, leading space included, re-exports this module).
"""
from primitive import *  # noqa: F401,F403
from arithmetic import vec_add


def poly_add(a, b, MOD):
    """Ciphertext add: component-wise vec_add over (c0, c1, ...) (' polynomial.py':3-5).

    The reference computes vec_add(a[0], b[0], MOD) and vec_add(a[1], b[1], MOD) but discards
    both and returns None; this returns the tuple it evidently meant (documented divergence).
    """
    assert len(a) == len(b)
    return tuple(vec_add(x, y, MOD) for x, y in zip(a, b))
