"""The engine skips the log of col_excitation_ratecoeff's Gaunt factor (macroatom.h:107-150) above x = E/kT = 0.57
(physics.h MA_GAUNT_NOLOG, col_exc_core / te_col_exc / te_col_exc_fast): Gamma = max(g_bar, 0.276 e^x (-gamma_E -
ln x)) is g_bar there whatever the log's value, so the skipped and the full expression give the same Gamma bit for
bit.  This checks the premise in double precision over the whole range the skip covers: -0.5772156649 - log(x) < 0
(so the test term is negative, or -inf where e^x overflows) for every x > 0.57, and the full expression's Gamma is
g_bar there."""
import numpy as np

MA_GAUNT_NOLOG = 0.57
G_BAR = 0.2


def gamma_full(x):
    with np.errstate(over="ignore", invalid="ignore"):
        test = 0.276 * np.exp(x) * (-0.5772156649 - np.log(x))
    return np.where(G_BAR > test, G_BAR, test)


def gamma_skip(x):
    with np.errstate(over="ignore", invalid="ignore"):
        test = np.where(x > MA_GAUNT_NOLOG, -1.0, 0.276 * np.exp(x) * (-0.5772156649 - np.log(x)))
    return np.where(G_BAR > test, G_BAR, test)


def test_log_term_negative_above_threshold():
    # every double in the first ulps above the threshold, then a dense log-spaced sweep up to overflow of exp
    x0 = np.nextafter(MA_GAUNT_NOLOG, np.inf)
    first = x0 + np.arange(4096) * np.spacing(x0)
    sweep = np.geomspace(x0, 1e6, 2_000_000)
    for x in (first, sweep):
        assert (-0.5772156649 - np.log(x) < 0).all()
        assert (gamma_full(x) == G_BAR).all()


def test_skip_matches_full_expression_everywhere():
    # below the threshold the skip evaluates the full expression; above it both give g_bar
    x = np.concatenate([np.geomspace(1e-12, 0.57, 100_000), np.geomspace(0.57, 1e4, 100_000),
                        np.array([0.5615, 0.5616, 0.57, np.nextafter(0.57, 1.0), 710.0, 1e300])])
    full, skip = gamma_full(x), gamma_skip(x)
    assert np.array_equal(full.view(np.uint64), skip.view(np.uint64))
    # the region where the log matters lies below the threshold: Gamma exceeds g_bar only for small x
    assert (full[x > MA_GAUNT_NOLOG] == G_BAR).all() and (full[x < 0.1] > G_BAR).any()
