"""Reinsert scenarios (PiXiuCtrl.cpp:12-29, 63-69, 88-114) — TEST INFRASTRUCTURE ONLY.

Each scenario is a list of batches, ("set", keys, vals) or ("del", keys), over one
instance (records_per_shard = 0).  They fill a chunk to its 65,535 slots so that the
reference's reinsert is well defined (PiXiuStr.cpp:189-193), then trigger it:

* rotation     — 2/3 of the chunk deleted while it is live; the next setitem closes it
                 under half live and re-inserts the rest (PiXiuCtrl.cpp:13-24);
* glob_delete  — deletes on a closed chunk drive it under half live; the next delitem
                 re-inserts it through Glob_Reinsert_Chunk (PiXiuCtrl.cpp:64-67);
* glob_replace — setitems replacing keys of a closed chunk do the same through the
                 CritBit replace (CritBitTree.cpp:32-38) and the setitem trigger
                 (PiXiuCtrl.cpp:26-29), inside one batch, followed by more deletes;
* direct       — PiXiuCtrl::reinsert(PiXiuChunk *&) called by the client on a closed chunk
                 that is 85 % live (no trigger would fire: need_reinsert is false, and
                 Glob_Reinsert_Chunk never points at it, which keeps the reference defined).

``run_scalar`` drives one record at a time through the oracle or the reference;
``state`` / ``digest`` reduce the end state to what both can report: every touched key's
presence, compat getitem bytes, slot and compressed bytes.
"""
from __future__ import annotations

import hashlib
import random

FULL = 65535


def key(i: int) -> bytes:
    return b"r%06d" % i


def _val(rng: random.Random, i: int) -> bytes:
    n = rng.randrange(0, 14)
    return bytes(rng.choice(b"abcdeXYZ") for _ in range(n)) + (b"%d" % (i % 97) if n else b"")


def scenarios() -> dict:
    out = {}
    rng = random.Random(19950207)
    ks = [key(i) for i in range(FULL + 10)]
    vs = [_val(rng, i) for i in range(FULL + 10)]
    out["rotation"] = [
        ("set", ks[:FULL], vs[:FULL]),
        ("del", [ks[i] for i in range(FULL) if i % 3]),
        ("set", ks[FULL:], vs[FULL:]),
    ]
    rng = random.Random(7)
    n = FULL + 100
    ks = [key(i) for i in range(n + 10)]
    vs = [_val(rng, i) for i in range(n + 10)]
    out["glob_delete"] = [
        ("set", ks[:n], vs[:n]),
        ("del", [ks[i] for i in range(0, 40000)]),
        ("set", ks[n:], vs[n:]),
    ]
    rng = random.Random(11)
    n = FULL + 10
    ks = [key(i) for i in range(n + 200)]
    vs = [_val(rng, i) for i in range(n + 200)]
    mixed_k, mixed_v = [], []
    nxt = n
    for i in range(40000):  # replace keys of the closed chunk, new keys interleaved
        mixed_k.append(ks[i])
        mixed_v.append(_val(rng, i + 7))
        if i % 400 == 0:
            mixed_k.append(ks[nxt])
            mixed_v.append(vs[nxt])
            nxt += 1
    out["glob_replace"] = [
        ("set", ks[:n], vs[:n]),
        ("set", mixed_k, mixed_v),
        ("del", [ks[i] for i in range(40000, 41000)]),
        ("set", ks[nxt:nxt + 10], vs[nxt:nxt + 10]),
    ]
    rng = random.Random(13)
    n = FULL + 10
    ks = [key(i) for i in range(n + 40)]
    vs = [_val(rng, i) for i in range(n + 40)]
    out["direct"] = [
        ("set", ks[:n], vs[:n]),
        ("del", [ks[i] for i in range(0, FULL, 7)]),
        ("reinsert", 0),
        ("set", ks[n:n + 20], vs[n:n + 20]),
        ("del", [ks[i] for i in range(FULL, FULL + 6)]),
        ("set", ks[n + 20:], vs[n + 20:]),
    ]
    return out


def touched(ops) -> list:
    seen = set()
    for op in ops:
        if op[0] != "reinsert":
            seen.update(op[1])
    return sorted(seen)


def run_scalar(impl, ops) -> list:
    """impl: object with set(k, v) -> rc and delete(k) -> rc.  Returns every record's rc."""
    rets = []
    for op in ops:
        if op[0] == "set":
            for k, v in zip(op[1], op[2]):
                r = impl.set(k, v)
                rets.append(int(r[0] if isinstance(r, tuple) else r))
        elif op[0] == "reinsert":
            rets.append(int(impl.reinsert(op[1])))
        else:
            for k in op[1]:
                rets.append(int(impl.delete(k)))
    return rets


def digest(rets, state) -> dict:
    """state: list of (key, present, get_bytes|None, idx|None, comp|None) in key order."""
    h = hashlib.sha256()
    for k, present, g, idx, comp in state:
        h.update(k + b"|%d|" % present)
        if present:
            h.update(b"%d|" % len(g) + g + b"|%d|" % idx + comp)
    return {
        "records": len(rets),
        "rets_sha256": hashlib.sha256(bytes(r & 0xFF for r in rets)).hexdigest(),
        "replaced": sum(1 for r in rets if r == 1),
        "live": sum(1 for s in state if s[1]),
        "state_sha256": h.hexdigest(),
    }


def ops_sha256(ops) -> str:
    h = hashlib.sha256()
    for op in ops:
        h.update(op[0].encode())
        if op[0] == "reinsert":
            h.update(b"%d" % op[1])
            continue
        for k in op[1]:
            h.update(b"%d:" % len(k) + k)
        if op[0] == "set":
            for v in op[2]:
                h.update(b"%d:" % len(v) + v)
    return h.hexdigest()


def reference_state(ref, keys) -> list:
    out = []
    for k in keys:
        g = ref.get(k)
        loc = ref.locate_comp(k)
        out.append((k, g is not None, g, loc[0] if loc else None, loc[1] if loc else None))
    return out


def oracle_state(sh, keys) -> list:
    """Also returns the chunk number of every live key (4th field of the extra list)."""
    out, where = [], []
    for k in keys:
        g = sh.get(k)
        loc = sh.locate(k)
        out.append((k, g is not None, g, loc[1] if loc else None, sh.comp(*loc) if loc else None))
        where.append(loc)
    return out, where
