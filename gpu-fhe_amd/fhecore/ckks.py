"""CKKS canonical-embedding encoder: complex slot vectors <-> integer
polynomials of Z[X]/(X^N + 1) at scale delta, and their RNS residues.

This is the host-side data boundary of the library (like ``to_device``), not part of the §8 hot
path: encoding is one float64 FFT of length 2N (numpy) per plaintext.  Slot j sits at the root
zeta_j = exp(i pi 5^j / N) (j < N/2), the ordering under which the Galois element 5^r rotates
the slots by r (fhecore Context.galois_elt / rotate):

    encode:  m_k = round(delta * (2/N) Re(sum_j z_j zeta_j^-k))        (k < N)
    decode:  z_j = sum_k m_k zeta_j^k / delta,  m = CRT-centred residues
"""
from __future__ import annotations

import math

import numpy as np


class Encoder:
    def __init__(self, n: int):
        self.n = n
        self.slots = n // 2
        two_n = 2 * n
        self.pos = np.empty(self.slots, dtype=np.int64)  # 5^j mod 2N
        e = 1
        for j in range(self.slots):
            self.pos[j] = e
            e = e * 5 % two_n

    def encode(self, z, delta: float) -> np.ndarray:
        """z: complex [N/2] -> int64 coefficients [N] (|delta m| must stay below 2^62)."""
        z = np.asarray(z, dtype=np.complex128)
        if z.shape != (self.slots,):
            raise ValueError(f"encode: expected {self.slots} slots")
        a = np.zeros(2 * self.n, dtype=np.complex128)
        a[self.pos] = z
        m = (2.0 / self.n) * np.fft.fft(a)[: self.n].real
        c = np.rint(m * delta)
        if np.abs(c).max(initial=0) >= 2.0 ** 62:
            raise OverflowError("encode: scaled coefficients exceed 2^62")
        return c.astype(np.int64)

    def decode(self, coeffs, delta: float) -> np.ndarray:
        """Signed integer coefficients [N] (ints or floats) -> complex slots [N/2]."""
        b = np.zeros(2 * self.n, dtype=np.complex128)
        b[: self.n] = np.asarray(coeffs, dtype=np.float64)
        return (2 * self.n) * np.fft.ifft(b)[self.pos] / delta


def to_rns(coeffs, moduli) -> np.ndarray:
    """Signed int64 coefficients [N] -> residues [L, N] (uint64)."""
    c = np.asarray(coeffs, dtype=np.int64)
    return np.stack([np.mod(c, np.int64(q)).astype(np.uint64) if q < 2 ** 63 else
                     np.array([int(v) % q for v in c], dtype=np.uint64) for q in moduli])


def from_rns(x, moduli) -> np.ndarray:
    """Residues [l, N] -> CRT-centred integers, returned as float64 (exact integers are Python
    ints internally; the float is what decode needs)."""
    moduli = [int(q) for q in moduli]
    Q = math.prod(moduli)
    x = np.asarray(x)
    acc = np.zeros(x.shape[-1], dtype=object)
    for i, q in enumerate(moduli):
        hat = Q // q
        acc = acc + x[i].astype(object) * (hat * pow(hat % q, -1, q) % Q)
    acc = acc % Q
    return np.array([float(v - Q) if v > Q // 2 else float(v) for v in acc])
