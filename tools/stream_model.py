"""A lane-level Python model of the ordered-stream kernels (ramcloud_amd/csrc/
stream.h: k_stream_prep, k_stream, k_stream_fix) for small batches.

It follows the kernels' data flow step for step -- spans of 128-byte steps
per 8-lane group, lane u holding dwords u, u+8, u+16, u+24 of a step, the
byte rotation by the group's half-wave index, the position table
X^(128 - q)(b), the carry injected into bytes 0..3, the masked sums at entry
boundaries (whole dwords plus the remainder bytes), the re-base at entry
starts with the initial state X^d(0xFFFFFFFF), the unshift X^p(X^-128(.)),
the per-lane entry windows of 8 slots and their refill, and the cross-span
fix-up -- so that a mismatch on the GPU can be localised against it.  Used by
tests/test_stream_model.py against the oracle (design check, not a product
path).

    python tools/stream_model.py      # a few random batches vs the oracle
"""
import sys

POLY = 0x82F63B78
ONE = 0x80000000


def mulmod(a, b):
    p = 0
    for i in range(32):
        if a & (ONE >> i):
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


def xpow8(n):
    r, sq = ONE, 0x00800000
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


XINV = ((POLY & 0x7FFFFFFF) << 1) | 1


def xinv8pow(n):
    inv8 = ONE
    for _ in range(8):
        inv8 = mulmod(inv8, XINV)
    r, sq = ONE, inv8
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


class Tables:
    def __init__(self):
        c = [xpow8(m) for m in range(129)]
        # pos[q][b] = X^(128 - q)(b)
        self.pos = [[mulmod(b, c[128 - q]) for b in range(256)] for q in range(128)]
        ci = xinv8pow(128)
        self.inv = [[mulmod(b << (8 * k), ci) for b in range(256)] for k in range(4)]
        self.ff = [mulmod(0xFFFFFFFF, c[dd]) for dd in range(129)]


def grp_xor(vals):
    r = 0
    for v in vals:
        r ^= v
    return r


def model(data, base_off, off, lens, nspan, finalize=True, T=None):
    """CRCs of entries (off[i], lens[i]) of `data` (bytes) as k_stream computes
    them; base_off is where offsets count from.  Returns (out, refused)."""
    T = T or Tables()
    n = len(off)
    B = base_off
    S_ = [B + o for o in off]
    E_ = [S_[i] + lens[i] for i in range(n)]
    R0, R1 = S_[0], E_[-1]
    A0 = R0 & ~127
    R1 = max(R1, A0)
    ns = max((R1 - A0 + 127) // 128, 1)
    sps = (ns + nspan - 1) // nspan
    L = 128 * sps
    nsp = (ns + sps - 1) // sps
    # k_stream_prep
    first_ev = [None] * nspan
    for i in range(n):
        lo = 0
        if i > 0:
            Ep = E_[i - 1]
            if S_[i] < Ep or S_[i] - Ep >= 4096:
                return None, True
            lo = (Ep - A0 + L - 1) // L if Ep > A0 else 0
        hi = (E_[i] - A0 + L - 1) // L if E_[i] > A0 else 0
        if i == n - 1:
            hi = nsp
        for s in range(lo, min(hi, nsp)):
            first_ev[s] = n if (i == n - 1 and s * L + A0 >= E_[i]) else i
    out = [None] * n
    span_t = [0] * nspan
    xe_val = [0] * nspan
    xe_idx = [None] * nspan

    def byte_at(a):
        return data[a] if 0 <= a < len(data) and a < R1 else 0

    def dword(a):
        return sum(byte_at(a + k) << (8 * k) for k in range(4))

    BIG = 0x7FFFFFFF
    for span in range(nspan):
        if span * sps >= ns:
            continue
        g4 = (span % 8) & 3
        sg = A0 + span * L
        e0 = first_ev[span]

        def rel(x):
            r = x - sg
            return -1 if r < 0 else (L + 1 if r > L + 1 else r)

        def window(e0):
            Sr = [[BIG] * 8 for _ in range(8)]
            Er = [[BIG] * 8 for _ in range(8)]
            for u in range(8):
                for m in range(8):
                    e = e0 + u + 8 * m
                    if e < n:
                        Sr[u][m], Er[u][m] = rel(S_[e]), rel(E_[e])
            return Sr, Er

        Sr, Er = window(e0)
        if span == 0:   # empty entries exactly at A0
            for i in range(e0):
                out[i] = 0 if finalize else 0xFFFFFFFF
        cnt = [0] * 8
        Sd = [u == 0 and Sr[0][0] <= 0 for u in range(8)]
        Ed = [False] * 8
        cross = [u == 0 and Sr[0][0] < 0 for u in range(8)]
        xe_done = False
        G = 0xFFFFFFFF if Sr[0][0] == 0 else 0
        for t in range(sps):
            w = [[dword(sg + 128 * t + 4 * (u + 8 * j)) for j in range(4)] for u in range(8)]
            w[0][0] ^= G
            vals = []   # vals[u][j][k]: lookup of rotated byte k of dword j
            for u in range(8):
                vu = []
                for j in range(4):
                    vj = []
                    for k in range(4):
                        kk = (k + g4) & 3
                        q = 4 * u + 32 * j + kk
                        vj.append(T.pos[q][(w[u][j] >> (8 * kk)) & 0xFF])
                    vu.append(vj)
                vals.append(vu)
            D = [[grp_xor(vals[u][j]) for j in range(4)] for u in range(8)]
            F = [grp_xor(D[u]) for u in range(8)]
            T0 = 128 * t
            C = 0
            while True:
                nb = [(Sr[u][0] if not Sd[u] else (Er[u][0] if not Ed[u] else BIG))
                      for u in range(8)]
                P = min(nb)
                if P == BIG and e0 + 64 < n and cnt[0] == 8:
                    e0 += 64
                    Sr, Er = window(e0)
                    cnt = [0] * 8
                    Sd = [False] * 8
                    Ed = [False] * 8
                    P = min(Sr[u][0] for u in range(8))
                if P > T0 + 128:
                    break
                p = P - T0
                Pd, r = p >> 2, p & 3
                acc = [0] * 8
                for u in range(8):
                    for j in range(4):
                        if u + 8 * j < Pd:
                            acc[u] ^= D[u][j]
                if r:
                    js, us = Pd >> 3, Pd & 7
                    m = (1 << (8 * r)) - 1
                    wsel = (w[us][js] & m) | ((G & ~m & 0xFFFFFFFF) if Pd == 0 else 0)
                    for k in range(4):
                        kk = (k + g4) & 3
                        acc[us] ^= T.pos[4 * Pd + kk][(wsel >> (8 * kk)) & 0xFF]
                V = grp_xor(acc)
                d8 = 128 - p
                isS = [not Sd[u] and Sr[u][0] == P for u in range(8)]
                isE = [(Sd[u] or isS[u]) and not Ed[u] and Er[u][0] == P for u in range(8)]
                for u in range(8):
                    idx = e0 + u + 8 * cnt[u]
                    if isE[u] and not isS[u]:
                        Y = V ^ C
                        raw = Y
                        if d8:
                            Z = grp_xor(T.inv[k][(Y >> (8 * k)) & 0xFF] for k in range(4))
                            raw = grp_xor(T.pos[128 - p + k][(Z >> (8 * k)) & 0xFF]
                                          for k in range(4)) if p >= 4 else mulmod(Z, xpow8(p))
                        if cross[u]:
                            xe_val[span], xe_idx[span] = raw, idx
                            xe_done = True
                        else:
                            out[idx] = (~raw & 0xFFFFFFFF) if finalize else raw
                    if isE[u] and isS[u]:
                        out[idx] = 0 if finalize else 0xFFFFFFFF
                if any(isS):
                    C = V ^ T.ff[d8]
                for u in range(8):
                    Sd[u] = Sd[u] or isS[u]
                    Ed[u] = Ed[u] or isE[u]
                    if Ed[u]:
                        Sr[u] = Sr[u][1:] + [BIG]
                        Er[u] = Er[u][1:] + [BIG]
                        cnt[u] += 1
                        Sd[u] = Ed[u] = cross[u] = False
            G = grp_xor(F) ^ C
        span_t[span] = G
        if not xe_done:
            xe_idx[span] = None
    # k_stream_fix
    for g in range(nspan):
        if g * sps >= ns or xe_idx[g] is None:
            continue
        i = xe_idx[g]
        sg = A0 + g * L
        h = (S_[i] - A0) // L
        assert 0 <= h < g
        st = span_t[h]
        for m in range(h + 1, g):
            st = mulmod(st, xpow8(L)) ^ span_t[m]
        raw = mulmod(st, xpow8(E_[i] - sg)) ^ xe_val[g]
        out[i] = (~raw & 0xFFFFFFFF) if finalize else raw
    return out, False


def crc32c(b, state=0xFFFFFFFF):
    for x in b:
        state ^= x
        for _ in range(8):
            state = (state >> 1) ^ (POLY if state & 1 else 0)
    return state


def main():
    import random
    rnd = random.Random(1)
    T = Tables()
    for trial in range(20):
        n = rnd.randint(1, 40)
        lens = [rnd.choice([0, 1, 3, 4, 5, 100, 127, 128, 129, 300, 1000]) for _ in range(n)]
        gaps = [rnd.choice([0, 0, 0, 1, 7, 200]) for _ in range(n)]
        pos, off = rnd.randint(0, 130), []
        for i in range(n):
            pos += gaps[i]
            off.append(pos)
            pos += lens[i]
        data = bytes(rnd.getrandbits(8) for _ in range(pos + 64))
        got, refused = model(data, 0, off, lens, nspan=rnd.choice([1, 2, 3, 8, 16]), T=T)
        want = [(~crc32c(data[o:o + ln])) & 0xFFFFFFFF for o, ln in zip(off, lens)]
        bad = [i for i in range(n) if got[i] != want[i]]
        print(f"trial {trial}: n={n} bad={bad[:5]}")
        if bad:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
