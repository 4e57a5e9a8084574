"""The device positional encoding's double-angle recurrence (lnerf_composite.h comp::encode_coord,
round 5) against the reference's per-frequency float64 sin/cos (pos_encoding.py:54-66, rounded to
float32 once): a numpy restatement of the recurrence on random coordinates in the range the
sampler produces, checked per value. After q doublings the float64 error is ~2^(q+1) ulp, so the
rounded float32 values may differ from the direct ones only where the exact value sits within that
distance of a float32 rounding boundary: at most one float32 ulp, and rarely (CPU-only)."""
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
