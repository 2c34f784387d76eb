"""The dual ratio test's tightening walk over the smallest keys only
(or-tools_amd/csrc/kernels/simplex_kernels.hip, dual_tighten_* kernels),
restated in numpy and checked against the walk over the fully sorted keys
(dual_flip_walk_kernel, the round-5 path): whenever the selection returns a
tightened bound it is the full walk's, and otherwise it returns B, the bound
the full walk's own fallbacks return. Random breakpoints with ties, +/-0
ratios, boxed and non-boxed columns, and selection sizes from 1 up.

The walk (entering_variable.cc:163-207 in pop order) flips boxed breakpoints
while the variation stays positive and accepts the first one that does not
flip; a ratio tie ends it at B because the pop order would then also depend
on magnitudes."""
import numpy as np
import pytest

NONE = np.uint64(0xFFFFFFFFFFFFFFFF)


def order_bits(x):
    b = np.float64(x).view(np.uint64)
    return np.uint64(~int(b) & 0xFFFFFFFFFFFFFFFF) if int(b) >> 63 else np.uint64(int(b) | (1 << 63))


def bits(x):
    return int(np.float64(x).view(np.uint64))


def full_walk(ratio, harris, delta, variation, best):
    """dual_flip_walk_kernel over the slots sorted by key (stable)."""
    keys = [int(order_bits(r)) for r in ratio]
    order = sorted(range(len(ratio)), key=lambda i: keys[i])
    prev = 0.0
    n = len(order)
    for i in range(n):
        r = ratio[order[i]]
        if i > 0 and r == prev:
            break
        prev = r
        d = delta[order[i]]
        if variation > 0.0 and d > 0.0:
            variation -= d
            if variation > 0.0:
                continue
        if i + 1 < n and ratio[order[i + 1]] == r:
            break
        h = bits(harris[order[i]])
        return min(h, best)
    return best


def threshold(keys, target):
    """The two histogram passes: the top 12 bits, then the next 12 inside
    the chosen bin, to the first bin where the count from below reaches
    min(target, n)."""
    n = len(keys)
    tgt = min(target, n)
    top = [k >> 52 for k in keys]
    h0 = np.bincount(top, minlength=4096)
    cum = np.cumsum(h0)
    b0 = int(np.searchsorted(cum, tgt))
    below0 = int(cum[b0] - h0[b0])
    mid = [(k >> 40) & 0xFFF for k in keys if (k >> 52) == b0]
    h1 = np.bincount(mid, minlength=4096)
    cum1 = below0 + np.cumsum(h1)
    b1 = int(np.searchsorted(cum1, tgt))
    t = (b0 << 52) | (b1 << 40) | ((1 << 40) - 1)
    return t, int(cum1[b1])


def selection_walk(ratio, harris, delta, variation, best, target, cap=2048):
    """dual_tighten_walk_kernel: gather the keys <= T, sort, walk; B when the
    walk leaves the gathered keys or accepts the last of them while more
    lie past T."""
    keys = [int(order_bits(r)) for r in ratio]
    t, count = threshold(keys, target)
    if count > cap:
        return best, "cap"
    sel = sorted((i for i in range(len(keys)) if keys[i] <= t), key=lambda i: keys[i])
    assert len(sel) == count
    n, total = len(sel), len(keys)
    prev = 0.0
    for i in range(n):
        r = ratio[sel[i]]
        if i > 0 and r == prev:
            return best, "tie"
        prev = r
        d = delta[sel[i]]
        if variation > 0.0 and d > 0.0:
            variation -= d
            if variation > 0.0:
                continue
        if i + 1 < n:
            if ratio[sel[i + 1]] == r:
                return best, "tie"
        elif n < total:
            return best, "edge"
        return min(bits(harris[sel[i]]), best), "accepted"
    return best, "exhausted"


def _case(rng, n, tie_rate, zero_rate):
    ratio = rng.exponential(1.0, n)
    if tie_rate > 0:
        pool = ratio[: max(1, n // 8)]
        ties = rng.random(n) < tie_rate
        ratio[ties] = rng.choice(pool, ties.sum())
    zeros = rng.random(n) < zero_rate
    ratio[zeros] = np.where(rng.random(zeros.sum()) < 0.5, 0.0, -0.0)
    mag = rng.uniform(0.1, 2.0, n)
    harris = np.maximum(1e-9 / mag, ratio + 1e-7 / mag)
    boxed = rng.random(n) < 0.8
    delta = np.where(boxed, rng.exponential(0.05, n) * mag, 0.0)
    variation = float(rng.exponential(1.0))
    best = bits(float(np.max(harris)) * 2.0)
    return ratio, harris, delta, variation, best


@pytest.mark.parametrize("seed", range(40))
def test_selection_walk_matches_full_walk(seed):
    rng = np.random.default_rng(seed)
    outcomes = set()
    for n, tie_rate, zero_rate in [(5, 0.0, 0.0), (50, 0.0, 0.1), (600, 0.0, 0.0),
                                   (600, 0.05, 0.02), (3000, 0.0, 0.0), (3000, 0.01, 0.05)]:
        ratio, harris, delta, variation, best = _case(rng, n, tie_rate, zero_rate)
        ref = full_walk(ratio, harris, delta, variation, best)
        for target in (1, 3, 16, 512):
            got, how = selection_walk(ratio, harris, delta, variation, best, target)
            outcomes.add(how)
            if how == "accepted":
                assert got == ref, (n, target)
            else:
                assert got == best  # the untightened bound: always safe
            if how in ("tie", "exhausted") and len(ratio) <= target:
                assert got == ref  # every key gathered: the full walk's own ending
    assert "accepted" in outcomes


def test_threshold_keeps_at_least_the_target():
    rng = np.random.default_rng(7)
    for n in (1, 2, 17, 513, 5000):
        keys = [int(order_bits(r)) for r in rng.exponential(1.0, n)]
        for target in (1, 5, 512):
            t, count = threshold(keys, target)
            below = sum(1 for k in keys if k <= t)
            assert below == count >= min(target, n)
