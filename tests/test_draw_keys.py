"""Host checks of two round-6 restatements the engine relies on for exact selections (numpy float64 is the same IEEE
arithmetic as the device's):

* ma_qh_draw (transport.h): the high-half bound k_ma takes from a Philox word instead of converting the draw,
  ma_qh_draw(hi) <= ma_qh(q) <= ma_qh_draw(hi) + 1 for q = z * (2^32 - 1), z = artis_rng_word_unit(lo, hi)
  (include/artis_rng.h), and when the bound is one low, q lies less than 3 above the multiple of 65536 it names --
  the two facts the exactness argument in transport.h uses;
* wave_select_continuum_nu (transport.h): select_continuum_nu's serial loop (ratecoeff.cc:628-684, the oracle's
  form) against the running sums + binary search the wave uses, bit for bit."""
import numpy as np

KEY_SCALE = 4294967295.0  # MA_KEY_SCALE (physics.h)


def _q(x):
    z = (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return z * KEY_SCALE


def _qh(q):
    return (q.astype(np.uint64) & np.uint64(0xFFFFFFFF)) >> np.uint64(16)


def _qh_draw(hi):
    return np.where(hi < 2, np.uint64(0), hi - np.uint64(2)) >> np.uint64(16)


def test_ma_qh_draw_bound():
    rng = np.random.default_rng(6)
    x = rng.integers(0, 2**63, size=2_000_000, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, 2_000_000,
                                                                                          dtype=np.uint64)
    # adversarial words: hi at and just above every 65536 boundary region, lo at its extremes
    k = rng.integers(0, 65536, size=200_000, dtype=np.uint64)
    hi = (k << np.uint64(16)) + rng.integers(0, 4, size=200_000, dtype=np.uint64)
    lo = rng.choice(np.array([0, 1, 2**21 - 1, 2**21, 2**32 - 2**11, 2**32 - 1], dtype=np.uint64), size=200_000)
    x = np.concatenate([x, (hi << np.uint64(32)) | lo, np.array([0, 1, 2**64 - 1, 2**32, 2**33], dtype=np.uint64)])
    h = x >> np.uint64(32)
    q = _q(x)
    qh, qd = _qh(q), _qh_draw(h)
    assert (qd <= qh).all() and (qh <= qd + np.uint64(1)).all()
    low = qd < qh
    assert low.any()  # the adversarial words reach the case
    assert (q[low] - (qh[low] << np.uint64(16)).astype(np.float64) < 3.0).all()


def _serial(pieces, zrand, nu_threshold, deltanu):
    npieces = len(pieces)
    total = 0.0
    for p in pieces:
        total += p
    alpha_old = alpha = total
    head = 0.0
    i = 1
    while i < npieces:
        alpha_old = alpha
        head += pieces[i - 1]
        alpha = total - head
        if zrand >= alpha / total:
            break
        i += 1
    return nu_threshold + (i - 1) * deltanu + (total * zrand - alpha_old) / (alpha - alpha_old) * deltanu


def _shared(pieces, zrand, nu_threshold, deltanu):
    npieces = len(pieces)
    P = [0.0]
    for p in pieces:
        P.append(P[-1] + p)
    total = P[npieces]
    lo, hi = 1, npieces
    while lo < hi:
        mid = (lo + hi) >> 1
        if zrand >= (total - P[mid]) / total:
            hi = mid
        else:
            lo = mid + 1
    i = lo
    k = npieces - 1 if i == npieces else i
    alpha_old, alpha = total - P[k - 1], total - P[k]
    return nu_threshold + (i - 1) * deltanu + (total * zrand - alpha_old) / (alpha - alpha_old) * deltanu


def test_fb_running_sum_search_matches_serial_loop():
    rng = np.random.default_rng(7)
    for trial in range(3000):
        n = int(rng.choice([2, 3, 5, 64, 100, 255, 256]))
        pieces = rng.random(n) * 10.0 ** rng.uniform(-30, 5)
        if trial % 3 == 0:
            pieces[rng.random(n) < 0.3] = 0.0  # zero pieces (cross-sections below threshold)
        if trial % 7 == 0:
            pieces[:] = 0.0  # total 0: both forms take the loop to its end
        for z in (0.0, 1e-300, rng.random(), rng.random(), 1.0 - 2.0**-53):
            with np.errstate(invalid="ignore", divide="ignore"):  # (total 0: 0 / 0 on both sides)
                a = _serial(list(pieces), z, 3.2e15, 1.7e13)
                b = _shared(list(pieces), z, 3.2e15, 1.7e13)
            assert (a == b) or (np.isnan(a) and np.isnan(b)), (n, z, a, b)
