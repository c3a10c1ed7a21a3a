"""Offline check of the EMA walk's latched positions (k_tile.hip latch64 + coupling fixpoint)
against the sequential flat/long/short machine on random tiles whose masks obey the nesting the
kernel relies on (A and X disjoint, B and Y disjoint, A implies Y, B implies X)."""
import random
M = (1 << 64) - 1
def latch(S, R, q):
    A = ~R & M; s1 = (A + S) & M; cout = s1 < A; sm = (s1 + q) & M; cout |= sm < s1
    return (((sm ^ A ^ S) >> 1) | (int(cout) << 63)) & M
def fix(Aw, Bw, Xw, Yw, fb, pos):
    RL, RS = Xw | fb, Yw | fb; lin, sin = int(pos > 0), int(pos < 0)
    Ap, Bp = Aw, Bw
    while True:
        Lw = latch(Ap, RL, lin); Sw = latch(Bp, RS, sin)
        An = Aw & ~(((Sw << 1) & M) | sin) & M; Bn = Bw & ~(((Lw << 1) & M) | lin) & M
        if An == Ap and Bn == Bp: break
        Ap, Bp = An, Bn
    return Lw, Sw
def seq(Aw, Bw, Xw, Yw, fb, pos):
    L = S = 0
    for b in range(64):
        a, bb, x, y, f = (Aw >> b) & 1, (Bw >> b) & 1, (Xw >> b) & 1, (Yw >> b) & 1, (fb >> b) & 1
        if pos == 0:
            pos = 1 if a else (-1 if bb else 0)
        elif pos > 0:
            if x or f: pos = 0
        else:
            if y or f: pos = 0
        L |= int(pos > 0) << b; S |= int(pos < 0) << b
    return L, S
rnd = random.Random(1)
for it in range(200000):
    # close vs ema relation per bar: r in {below lo, below e, equal, above e, above hi}
    Aw = Bw = Xw = Yw = 0
    for b in range(64):
        r = rnd.choice([-2, -1, 0, 1, 2]); slope = rnd.choice([-1, 0, 1])
        vm = rnd.random() < 0.95
        if not vm: continue
        if r == -2 and slope >= 0: Aw |= 1 << b
        if r == 2 and slope <= 0 and not (Aw >> b) & 1: Bw |= 1 << b
        if r >= 0: Xw |= 1 << b
        if r <= 0: Yw |= 1 << b
    bl = rnd.choice([64, 70, rnd.randrange(0, 64)])
    fb = (1 << bl) if bl < 64 else 0
    if bl < 64:  # bars >= bl are outside vm
        keep = (1 << bl) - 1
        Aw &= keep; Bw &= keep; Xw &= keep; Yw &= keep
    pos = rnd.choice([-1, 0, 1])
    assert fix(Aw, Bw, Xw, Yw, fb, pos) == seq(Aw, Bw, Xw, Yw, fb, pos), it
print("ok")
