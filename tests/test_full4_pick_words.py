"""FULL4's pick words on doubles: sub-moves 2 and 3 take
w2 = r1 * 0x85EBCA6B and w3 = r2 * 0xC2B2AE35 (mod 2^32, narde_rules.h
turn_words; the oracle restates the same), deterministic functions of the
words of sub-moves 0 and 1 rather than fresh Philox output.  The parity tests
cannot see a correlation this would add to the random policy (both sides
compute it), so this test checks the law itself: for uniform 32-bit r (what
Philox4x32-10 delivers), the picks mulhi(r, n0) and mulhi(r * c, n2) must be
independent and each uniform, for the list sizes a doubles turn has.  A
chi-square test of independence over 2^22 draws per (n0, n2) pair."""
import numpy as np
import pytest

C2, C3 = 0x85EBCA6B, 0xC2B2AE35


def _picks(r, c, n0, n2):
    w2 = (r.astype(np.uint64) * np.uint64(c)) & np.uint64(0xFFFFFFFF)
    p0 = (r.astype(np.uint64) * np.uint64(n0)) >> np.uint64(32)
    p2 = (w2 * np.uint64(n2)) >> np.uint64(32)
    return p0.astype(np.int64), p2.astype(np.int64)


def _chi2_independence(p0, p2, n0, n2):
    table = np.zeros((n0, n2), np.float64)
    np.add.at(table, (p0, p2), 1.0)
    row, col = table.sum(1, keepdims=True), table.sum(0, keepdims=True)
    exp = row * col / table.sum()
    chi2 = float(((table - exp) ** 2 / exp).sum())
    return chi2, (n0 - 1) * (n2 - 1)


@pytest.mark.parametrize("c", [C2, C3])
@pytest.mark.parametrize("n0,n2", [(2, 2), (3, 5), (4, 4), (7, 11), (12, 9), (15, 15), (24, 2)])
def test_subsequent_picks_independent_of_first(c, n0, n2):
    rng = np.random.default_rng(n0 * 100 + n2 + (c & 7))
    r = rng.integers(0, 2 ** 32, size=1 << 22, dtype=np.uint64).astype(np.uint32)
    p0, p2 = _picks(r, c, n0, n2)
    chi2, dof = _chi2_independence(p0, p2, n0, n2)
    # chi-square with dof degrees of freedom: mean dof, sd sqrt(2 dof); 6 sd
    assert chi2 < dof + 6 * np.sqrt(2 * dof), (chi2, dof)
    # and each pick uniform over its list
    for p, n in ((p0, n0), (p2, n2)):
        cnt = np.bincount(p, minlength=n).astype(np.float64)
        e = len(p) / n
        assert float(((cnt - e) ** 2 / e).sum()) < (n - 1) + 6 * np.sqrt(2 * (n - 1))
