"""Drop-in for the reference's ``primitive`` module (/root/reference/primitive.py:1-4).

It re-exports the arithmetic layer by star import, like the reference, so
``from primitive import *`` yields vec_add / vec_sub / vec_mul / NTT / iNTT (and ``np``).
"""
from arithmetic import *  # noqa: F401,F403


def XXX():
    """The reference's placeholder (primitive.py:3-4): prints "XXX"."""
    print("XXX")
