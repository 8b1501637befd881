"""CPU ORACLE — test infrastructure only, never the product path.

Only ``tests/`` may import this module, and only as the checker.  The shipped sampler is the HIP
kernel behind ``include/drcvar_sampling.h`` (``csrc/drcvar_sampling.hip``); it never calls into
``oracle/``.

NumPy restatement of the device obstacle-sample generator, which replaces the reference's host
draws ``simulation/obstacles.py:43-77`` (``np.random.multivariate_normal(zeros(2), noise_cov)`` per
sample and step, step 0 the nominal start, ``:63``).  The reference's stream (sequential MT19937)
is not reproducible in parallel, so the device generator defines its own: for the sample with
global index ``g = (o * T + t) * N + i``

* Philox4x32-10 (Salmon et al., SC'11; multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments
  0x9E3779B9 / 0xBB67AE85) on counter ``(g lo, g hi, stream lo, stream hi)`` and key ``seed``;
* ``u1 = ((x0:x1) >> 12 + 1/2) / 2^52`` in (0, 1) (exact); angle ``2 pi (x2:x3) / 2^64``;
* Box-Muller ``z = sqrt(-2 log u1) (cos, sin)``; sample ``nominal + L z``.

``log_unit`` and ``cos_sin_turn`` restate the kernel's own series (atanh series of
``s = f / (2 + f)``; quadrant from the top bits, Taylor series on [-pi/4, pi/4]) so the tests can
check them against numpy's ``log`` / ``cos`` / ``sin`` and the kernel against this mirror.  The
kernel contracts its polynomial steps into FMAs; numpy rounds each product, so the two agree to a
few ulp, not bit for bit.
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 rounds on uint32 counter arrays; returns the four output words (uint64
    arrays holding 32-bit values).  Mirrors ``philox4x32_10`` in csrc/drcvar_sampling.hip."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK32 for c in (c0, c1, c2, c3))
    for r in range(10):
        ka, kb = np.uint64((k0 + r * _W0) & 0xFFFFFFFF), np.uint64((k1 + r * _W1) & 0xFFFFFFFF)
        p0, p1 = _M0 * c0, _M1 * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ ka
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ kb
        c0, c1, c2, c3 = n0, p1 & _MASK32, n2, p0 & _MASK32
    return c0, c1, c2, c3


def uniform52(hi, lo):
    """(top 52 bits + 1/2) / 2^52: exact, in [2^-53, 1 - 2^-53] (the kernel's ``uniform52``)."""
    v = ((hi << np.uint64(32)) | lo) >> np.uint64(12)
    return (v.astype(np.float64) + 0.5) * 2.0 ** -52


def log_unit(x):
    """log x for 0 < x <= 1, the kernel's series (``log_unit``)."""
    m, e = np.frexp(np.asarray(x, dtype=np.float64))
    lo = m < 0.70710678118654752440
    m = np.where(lo, m + m, m)
    e = np.where(lo, e - 1, e).astype(np.float64)
    f = m - 1.0
    s = f / (2.0 + f)
    z = s * s
    p = np.full_like(z, 2.0 / 21.0)
    for k in (19, 17, 15, 13, 11, 9, 7, 5, 3):
        p = p * z + 2.0 / k
    logm = (s * z) * p + (s + s)
    ln2_hi, ln2_lo = float.fromhex("0x1.62e42fefa3800p-1"), float.fromhex("0x1.ef35793c76730p-45")
    return e * ln2_hi + (e * ln2_lo + logm)


def cos_sin_turn(whi, wlo):
    """(cos, sin)(2 pi w / 2^64) for w = whi:wlo, the kernel's ``cos_sin_turn``."""
    w = (np.asarray(whi, dtype=np.uint64) << np.uint64(32)) | np.asarray(wlo, dtype=np.uint64)
    q = ((w + np.uint64(1 << 61)) >> np.uint64(62)).astype(np.uint64)
    rem = (w - (q << np.uint64(62))).view(np.int64) >> np.int64(11)
    x = rem.astype(np.float64) * (6.28318530717958647692 * 2.0 ** -53)
    z = x * x
    ps = np.full_like(z, -1.0 / 1307674368000.0)
    for c in (1.0 / 6227020800.0, -1.0 / 39916800.0, 1.0 / 362880.0, -1.0 / 5040.0, 1.0 / 120.0,
              -1.0 / 6.0):
        ps = ps * z + c
    s = (x * z) * ps + x
    pc = np.full_like(z, 1.0 / 20922789888000.0)
    for c in (-1.0 / 87178291200.0, 1.0 / 479001600.0, -1.0 / 3628800.0, 1.0 / 40320.0,
              -1.0 / 720.0, 1.0 / 24.0, -0.5):
        pc = pc * z + c
    c = z * pc + 1.0
    q = q.astype(np.int64)
    swap = (q & 1).astype(bool)
    a, b = np.where(swap, s, c), np.where(swap, c, s)
    return np.where((q + 1) & 2, -a, a), np.where(q & 2, -b, b)


def sample_trajectories(nominal, n_samples: int, chol, seed: int, stream_offset: int = 0,
                        zero_first_step: bool = True):
    """[O, T, N, 2] samples the device generator produces for ``nominal`` [O, T, 2] and the lower
    Cholesky factor ``chol`` (l00, l10, l11)."""
    nominal = np.asarray(nominal, dtype=np.float64)
    O, T = nominal.shape[:2]
    l00, l10, l11 = chol
    g = np.arange(O * T * n_samples, dtype=np.uint64)
    x0, x1, x2, x3 = philox4x32_10(g & _MASK32, g >> np.uint64(32),
                                   np.uint64(stream_offset & 0xFFFFFFFF),
                                   np.uint64((stream_offset >> 32) & 0xFFFFFFFF),
                                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    rad = np.sqrt(-2.0 * log_unit(uniform52(x0, x1)))
    cs, sn = cos_sin_turn(x2, x3)
    z0, z1 = rad * cs, rad * sn
    out = np.empty((O, T, n_samples, 2))
    nom = np.repeat(nominal.reshape(O * T, 1, 2), n_samples, axis=1).reshape(-1, 2)
    out.reshape(-1, 2)[:, 0] = nom[:, 0] + l00 * z0
    out.reshape(-1, 2)[:, 1] = nom[:, 1] + (l10 * z0 + l11 * z1)
    if zero_first_step and T:
        out[:, 0] = nominal[:, 0, None, :]
    return out
