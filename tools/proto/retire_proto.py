"""CPU prototype of px_psa.hip's prefix doubling with RETIRED groups, checked
against a naive suffix sort.  Sequential: every step takes its keys from the ranks at the
step's start (as k_dbl_key does) and a group retires when it keeps one key K whose target
group (the one starting at slot K - 1) had exactly its size at the step's start.  Retired
members carry (id | RET) ranks; a rank read through a link is g + (rank(q + D) - T); links
are shortened before each step and the retired groups copy their root's final order at the
end.  Order: suffixes of a doc compare byte-wise, a doc's end is smaller than any byte, and
equal suffixes (both ending together) keep position order.

    python tools/proto/retire_proto.py [trials]
"""
import random
import sys

RET = 1 << 31


def naive_sa(T, dist):
    n = len(T)
    return sorted(range(n), key=lambda p: (bytes(T[p:p + dist[p]]) + b"", p) if False else (list(T[p:p + dist[p]]) + [-1], p))


def doubling(T, dist, syms=3, retire=True):
    n = len(T)
    sym = lambda p, s: T[p + s] + 1 if s < dist[p] else 0  # noqa: E731
    key0 = [tuple(sym(p, s) for s in range(syms)) for p in range(n)]
    sa = sorted(range(n), key=lambda p: (key0[p], p))
    rank = [0] * n
    gsz = {}  # group start -> size (live groups of >= 2)
    r = 0
    while r < n:
        e = r
        complete = key0[sa[r]][-1] == 0
        while not complete and e + 1 < n and key0[sa[e + 1]] == key0[sa[r]]:
            e += 1
        for j in range(r, e + 1):
            rank[sa[j]] = r
        if e > r:
            gsz[r] = e - r + 1
        r = e + 1
    ent = []   # [g, size, T, D]
    h = syms
    retired_total = 0
    def shorten():
        # a link to a range that one retired group now covers exactly follows that group's link
        for i, (g, size, Tt, D) in enumerate(ent):
            q0 = sa[g]
            x = rank[q0 + D]
            while x & RET:
                g2, s2, T2, D2 = ent[x & ~RET]
                if g2 != Tt or s2 != size:
                    break  # (the target split and only part of it retired: member by member)
                Tt, D = T2, D + D2
                x = rank[q0 + D]
            ent[i][2], ent[i][3] = Tt, D

    while gsz:
        shorten()

        def live(q):
            acc = 0
            x = rank[q]
            while x & RET:
                g, _, Tt, D = ent[x & ~RET]
                acc += g - Tt
                q += D
                x = rank[q]
            return acc + x

        keys = {}
        for g, size in gsz.items():
            for j in range(g, g + size):
                p = sa[j]
                keys[j] = live(p + h) + 1 if h < dist[p] else 0
        size0 = dict(gsz)
        new_gsz = {}
        new_rank = {}
        for g, size in sorted(gsz.items()):
            ks = [keys[j] for j in range(g, g + size)]
            if all(k == ks[0] for k in ks) and ks[0] != 0:
                K = ks[0]
                if retire and K - 1 != g and size0.get(K - 1) == size:
                    idx = len(ent)
                    ent.append([g, size, K - 1, h])
                    for j in range(g, g + size):
                        new_rank[sa[j]] = idx | RET
                    retired_total += size
                    continue
                new_gsz[g] = size
                continue
            order = sorted(range(size), key=lambda i: (ks[i], i))  # stable by key
            mem = [sa[g + i] for i in order]
            kk = [ks[i] for i in order]
            for i in range(size):
                sa[g + i] = mem[i]
            i = 0
            while i < size:
                e = i
                while kk[i] != 0 and e + 1 < size and kk[e + 1] == kk[i]:
                    e += 1
                for j in range(i, e + 1):
                    new_rank[sa[g + j]] = g + i
                if e > i:
                    new_gsz[g + i] = e - i + 1
                i = e + 1
        for p, x in new_rank.items():
            rank[p] = x
        gsz = new_gsz
        h *= 2
    # resolve: every live suffix is final now, so each retired member's rank through its
    # links is its final slot (computed for all before any is written)
    shorten()

    def live_final(q):
        acc = 0
        x = rank[q]
        while x & RET:
            g, _, Tt, D = ent[x & ~RET]
            acc += g - Tt
            q += D
            x = rank[q]
        return acc + x
    fin = []
    for g, size, _, _ in ent:
        for j in range(size):
            q = sa[g + j]
            fin.append((q, live_final(q)))
    for q, f in fin:
        rank[q] = f
        sa[f] = q
    return sa, retired_total


def corpus(rng):
    alpha = rng.choice([b"ab", b"abc", b"abcd<>/", bytes(range(32, 127))])
    tmpl = bytes(rng.choice(alpha) for _ in range(rng.randint(20, 200)))
    docs = []
    for _ in range(rng.randint(2, 12)):
        body = bytes(rng.choice(alpha) for _ in range(rng.randint(0, 60)))
        cut = rng.randint(0, len(tmpl))
        docs.append(tmpl[:cut] + body + tmpl[cut:] + (tmpl if rng.random() < 0.3 else b""))
    return [d for d in docs if d]


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = random.Random(5)
    ret_any = 0
    for t in range(trials):
        docs = corpus(rng)
        T = b"".join(docs)
        dist = []
        for d in docs:
            dist += list(range(len(d), 0, -1))
        want = naive_sa(T, dist)
        got, nret = doubling(T, dist)
        base, _ = doubling(T, dist, retire=False)
        assert base == want, f"trial {t}: doubling without retirement differs"
        assert got == want, f"trial {t}: retired doubling differs ({nret} retired)"
        ret_any += nret > 0
    print(f"ok: {trials} corpora, {ret_any} with retired groups")


if __name__ == "__main__":
    main()
