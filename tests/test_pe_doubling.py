"""The device positional encoding's double-angle recurrence (lnerf_composite.h comp::encode_coord,
round 5) against the reference's per-frequency float64 sin/cos (pos_encoding.py:54-66, rounded to
float32 once): a numpy restatement of the recurrence on random coordinates in the range the
sampler produces, checked per value. After q doublings the float64 error is ABSOLUTE, about
2^(q+1) float64 ulps of 1 (2^(q+1-53); the step cos 2y = (c - s)(c + s) cancels where cos 2y ~ 0 and
sin 2y inherits that), not relative. So:
  * on random coordinates the rounded float32 values differ from the direct ones only where the
    exact value sits within that distance of a float32 rounding boundary: at most one float32 ulp,
    and rarely;
  * next to a zero of sin / cos (coordinates at k pi / 2^(q+1)) a tiny value can be many float32
    ulps of ITSELF away, but never more than 2^(q+1-53) + one float32 ulp absolute -- at F = 10 about
    2^-43, ~2^-19 of float32's resolution of the encoding's unit scale, so no MLP output can see it
    (CPU-only)."""
import numpy as np


def encode_doubling(x, F):
    """comp::encode_coord: one float64 sincos, then sin 2y = 2 sin y cos y, cos 2y = (c - s)(c + s)."""
    s, c = np.sin(x), np.cos(x)
    out_s, out_c = [], []
    for _ in range(F):
        out_s.append(s.astype(np.float32))
        out_c.append(c.astype(np.float32))
        s, c = 2.0 * s * c, (c - s) * (c + s)
    return out_s, out_c


def test_doubling_matches_per_frequency_sincos():
    rng = np.random.default_rng(7)
    # RAYS-mode points o + d t at t in [2, 6] for unit-scale cameras, plus small coordinates
    x = np.concatenate([rng.uniform(-8.0, 8.0, 400_000), rng.uniform(-1e-3, 1e-3, 100_000)])
    F = 10   # the most kr / k1 encode in LDS (k0 = 3 + 6 F <= 64)
    got_s, got_c = encode_doubling(x, F)
    differing = 0
    for q in range(F):
        arg = np.ldexp(x, q)
        for got, want in ((got_s[q], np.sin(arg).astype(np.float32)), (got_c[q], np.cos(arg).astype(np.float32))):
            d = got != want
            differing += int(d.sum())
            if d.any():
                # never more than one float32 ulp
                ulp = np.spacing(np.abs(want[d]).astype(np.float32))
                assert (np.abs(got[d].astype(np.float64) - want[d]) <= ulp).all(), q
    assert differing <= 50, differing   # of 10^7 values (measured: a handful)


def test_doubling_absolute_bound_at_zeros_of_sin_cos():
    """adversarial coordinates at (and one float64 ulp beside) k pi / 2^(q+1), where sin or
    cos of 2^q x crosses zero: the error bound is absolute, 2^(q+1) float64 ulps of 1 before the
    float32 rounding (measured worst: 0.75 of it)."""
    F = 10
    k = np.arange(1, 20000, dtype=np.float64)
    xs = []
    for q in range(F + 1):
        base = k * np.pi / 2.0 ** (q + 1)
        xs += [base, np.nextafter(base, 0.0), np.nextafter(base, np.inf)]
    x = np.concatenate(xs)
    x = x[x <= 16.0]
    x = np.concatenate([x, -x])
    got_s, got_c = encode_doubling(x, F)
    many_ulps = 0
    for q in range(F):
        arg = np.ldexp(x, q)
        bound = 2.0 ** (q + 1 - 53)
        for got, exact in ((got_s[q], np.sin(arg)), (got_c[q], np.cos(arg))):
            want = exact.astype(np.float32)
            err = np.abs(got.astype(np.float64) - want.astype(np.float64))
            ulp = np.spacing(np.abs(want)).astype(np.float64)
            assert (err <= bound + ulp).all(), (q, float((err - ulp).max()), bound)
            many_ulps += int((err > 4 * ulp).sum())
    # the relative statement of round 5 does not hold here: tiny values many ulps off do occur
    assert many_ulps > 0
