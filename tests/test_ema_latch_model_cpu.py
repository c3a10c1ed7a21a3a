"""CPU model of the EMA+OLS walk's latched positions (k_tile.hip ema_tile_kernel: `latch64` and
the coupling fixpoint) against the sequential flat / long / short machine of
docs/oracle_spec.md, on random 64-bar tiles whose condition words obey the nesting the kernel
relies on (entry-long A and exit-long X disjoint, B and Y disjoint, A implies Y, B implies X),
with carried positions and forced exits. The GPU parity tests check the kernel itself."""
import random

M = (1 << 64) - 1


def latch64(S, R, q):
    """State after every bar of a set/reset latch (S, R disjoint), q = state before bar 0."""
    A = ~R & M
    s1 = (A + S) & M
    cout = s1 < A
    sm = (s1 + q) & M
    cout |= sm < s1
    return (((sm ^ A ^ S) >> 1) | (int(cout) << 63)) & M


def latched(Aw, Bw, Xw, Yw, fb, pos):
    RL, RS = Xw | fb, Yw | fb
    lin, sin = int(pos > 0), int(pos < 0)
    Ap, Bp = Aw, Bw
    while True:
        Lw, Sw = latch64(Ap, RL, lin), latch64(Bp, RS, sin)
        An = Aw & ~(((Sw << 1) & M) | sin) & M
        Bn = Bw & ~(((Lw << 1) & M) | lin) & M
        if (An, Bn) == (Ap, Bp):
            return Lw, Sw
        Ap, Bp = An, Bn


def sequential(Aw, Bw, Xw, Yw, fb, pos):
    L = S = 0
    for b in range(64):
        bit = lambda w: (w >> b) & 1  # noqa: E731
        if pos == 0:
            pos = 1 if bit(Aw) else (-1 if bit(Bw) else 0)
        elif (bit(Xw) if pos > 0 else bit(Yw)) or bit(fb):
            pos = 0
        L |= int(pos > 0) << b
        S |= int(pos < 0) << b
    return L, S


def _tile(rnd):
    """Condition words of one tile: per bar the close sits under the lower band, under / at /
    over the EMA or over the upper band, with a random OLS slope sign; ~5 % of bars outside the
    decision range, and sometimes the series' last bar (forced exit) inside the tile."""
    Aw = Bw = Xw = Yw = 0
    for b in range(64):
        r, slope = rnd.choice([-2, -1, 0, 1, 2]), rnd.choice([-1, 0, 1])
        if rnd.random() < 0.05:
            continue
        if r == -2 and slope >= 0:
            Aw |= 1 << b
        elif r == 2 and slope <= 0:
            Bw |= 1 << b
        if r >= 0:
            Xw |= 1 << b
        if r <= 0:
            Yw |= 1 << b
    bl = rnd.choice([64, 70, rnd.randrange(0, 64)])
    fb = 0
    if bl < 64:
        fb, keep = 1 << bl, (1 << bl) - 1
        Aw, Bw, Xw, Yw = Aw & keep, Bw & keep, Xw & keep, Yw & keep
    return Aw, Bw, Xw, Yw, fb, rnd.choice([-1, 0, 1])


def test_latched_positions_match_sequential_machine():
    rnd = random.Random(1)
    for i in range(30000):
        t = _tile(rnd)
        assert latched(*t) == sequential(*t), (i, t)
