"""Deterministic synthetic corpora for the five BASELINE.json configs.

SURVEY.md §8(d) specifies the shapes; every generator draws from a counter-based
splitmix64 stream seeded with ``0x5049585500 + config`` so the same corpus is
rebuilt bit-for-bit on any host (no datasets travel; there is no network).

A corpus is a CSR pair of byte buffers: ``keys[koff[i]:koff[i+1]]`` and
``vals[voff[i]:voff[i+1]]`` for record ``i``.
"""
from __future__ import annotations

import dataclasses
import functools
import os

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
SEED_BASE = 0x5049585500

# 40-token HTML/URL vocabulary (visible ASCII only: the README corpus had its
# invisible characters stripped, README.md:51).
VOCAB = [
    "<div", "</div>", "<a", "href=", '"http://', "www.", ".com/", "class=", '"nav"',
    "<span>", "</span>", "<li>", "</li>", "<ul>", "</ul>", "<p>", "</p>", "<img",
    "src=", '.jpg"', "/>", "<script", "</script>", "var", "function(){", "return",
    "question/", "zhihu", "qq", "news", "index", ".htm", "title", "content", "&amp;",
    "id=", "?", "=", ";", "{",
]


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """n outputs of splitmix64 at counter positions start+1 .. start+n."""
    with np.errstate(over="ignore"):
        x = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (
            np.arange(start + 1, start + n + 1, dtype=np.uint64) * GAMMA)
        z = (x ^ (x >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


class Stream:
    """Sequential view of one splitmix64 stream."""

    def __init__(self, config: int, tag: int):
        self.seed = (SEED_BASE + config + tag * 0x1_0000_0000_0000) & 0xFFFFFFFFFFFFFFFF
        self.pos = 0

    def u64(self, n: int) -> np.ndarray:
        out = splitmix64(self.seed, n, self.pos)
        self.pos += n
        return out

    def uniform(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))

    def randint(self, lo: int, hi: int, n: int) -> np.ndarray:
        """integers in [lo, hi)"""
        return (lo + (self.u64(n) % np.uint64(hi - lo))).astype(np.int64)


@dataclasses.dataclass
class Corpus:
    config: int
    keys: np.ndarray  # uint8
    koff: np.ndarray  # int64, n+1
    vals: np.ndarray  # uint8
    voff: np.ndarray  # int64, n+1

    @property
    def n(self) -> int:
        return len(self.koff) - 1

    def key(self, i: int) -> bytes:
        return self.keys[self.koff[i]:self.koff[i + 1]].tobytes()

    def val(self, i: int) -> bytes:
        return self.vals[self.voff[i]:self.voff[i + 1]].tobytes()

    @property
    def raw_bytes(self) -> int:
        return int(self.koff[-1] + self.voff[-1])

    def slice(self, a: int, b: int) -> "Corpus":
        return Corpus(self.config,
                      self.keys[self.koff[a]:self.koff[b]], self.koff[a:b + 1] - self.koff[a],
                      self.vals[self.voff[a]:self.voff[b]], self.voff[a:b + 1] - self.voff[a])


def _csr(parts: list) -> tuple:
    lens = np.fromiter((len(p) for p in parts), dtype=np.int64, count=len(parts))
    off = np.zeros(len(parts) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy() if parts else np.zeros(0, np.uint8)
    return buf, off


class _TokenTable:
    """Concatenated token bytes with offsets, for vectorised token -> byte expansion."""

    def __init__(self, tokens: list):
        enc = [t.encode() if isinstance(t, str) else t for t in tokens]
        self.lens = np.array([len(t) for t in enc], np.int64)
        self.offs = np.zeros(len(enc), np.int64)
        np.cumsum(self.lens[:-1], out=self.offs[1:])
        self.blob = np.frombuffer(b"".join(enc), np.uint8)

    def expand(self, ids: np.ndarray) -> np.ndarray:
        lens = self.lens[ids]
        total = int(lens.sum())
        starts = np.zeros(len(ids), np.int64)
        np.cumsum(lens[:-1], out=starts[1:])
        idx = np.arange(total, dtype=np.int64) + np.repeat(self.offs[ids] - starts, lens)
        return self.blob[idx]


_VOCAB = _TokenTable(VOCAB)


@functools.lru_cache(maxsize=None)
def _numbers(hi: int) -> _TokenTable:
    return _TokenTable([str(i) for i in range(hi)])


def _zipf_ids(st: Stream, n: int, k: int) -> np.ndarray:
    w = 1.0 / np.arange(1, k + 1)
    cdf = np.cumsum(w) / w.sum()
    return np.searchsorted(cdf, st.uniform(n), side="right").clip(0, k - 1)


@functools.lru_cache(maxsize=None)
def _mixed_table(num_hi: int) -> tuple:
    """Vocabulary tokens then decimal numbers 0..num_hi-1, padded to a 2-D table."""
    toks = [t.encode() for t in VOCAB] + [str(i).encode() for i in range(num_hi)]
    width = max(len(t) for t in toks)
    tab = np.zeros((len(toks), width), np.uint8)
    lens = np.array([len(t) for t in toks], np.int64)
    for i, t in enumerate(toks):
        tab[i, :len(t)] = np.frombuffer(t, np.uint8)
    mask = np.arange(width)[None, :] < lens[:, None]
    return tab, mask, lens


def _soup(st: Stream, nbytes: int, num_hi: int, num_frac: float) -> np.ndarray:
    """>= nbytes of vocabulary tokens (Zipf-ish) mixed with decimal numbers."""
    tab, mask, lens = _mixed_table(num_hi)
    out = []
    have = 0
    while have < nbytes:
        m = max(64, (nbytes - have) // 4)
        is_num = st.uniform(m) < num_frac
        vid = _zipf_ids(st, m, len(VOCAB))
        nid = st.randint(0, num_hi, m)
        ids = np.where(is_num, len(VOCAB) + nid, vid)
        buf = tab[ids][mask[ids]]
        out.append(buf)
        have += len(buf)
    return np.concatenate(out)[:nbytes]


def config1(n: int = 1000, part: int = 0) -> Corpus:
    st = Stream(1, part * 1_000_000)
    ids = st.randint(0, 100_000_000, n)
    keys = [b"http://www.zhihu.com/question/%08d_%d" % (int(ids[i]), i + part * n) for i in range(n)]
    lens = st.randint(60, 80, n)
    vals = []
    for i in range(n):
        body = _soup(st, int(lens[i]), 1000, 0.2)
        vals.append(b"::" + body.tobytes())
    kb, ko = _csr(keys)
    vb, vo = _csr(vals)
    return Corpus(1, kb, ko, vb, vo)


def config2(n: int = 100_000, part: int = 0) -> Corpus:
    st = Stream(2, part * 1_000_000)
    keys = [b"rec/%08d" % (i + part * n) for i in range(n)]
    soup = _soup(st, 1000 * n, 1000, 0.2)
    kb, ko = _csr(keys)
    vo = np.arange(n + 1, dtype=np.int64) * 1000
    return Corpus(2, kb, ko, soup, vo)


def _templates() -> list:
    st = Stream(3, 99)
    return [_soup(st, 8192, 100_000, 0.1) for _ in range(16)]


def _config3_block(args) -> np.ndarray:
    b, count, soup_len, part = args
    return _soup(Stream(3, 1000 + b + part * 1_000_000), soup_len * count, 100_000, 0.1)


def config3(n: int = 10_000, value_len: int = 60_000, workers: int = 0, part: int = 0) -> Corpus:
    """HTML-shape pages: a fixed 8 KB boilerplate (one of 16) + tag/word soup + ids.
    Blocks of 256 pages draw from independent streams, so they can be built in parallel."""
    st = Stream(3, part * 1_000_000)
    tmpl = _templates()
    mmdd = st.randint(0, 365, n)
    tid = st.randint(0, 16, n)
    keys = []
    for i in range(n):
        d = int(mmdd[i])
        keys.append(b"http://www.qq.com/a/2017%02d%02d/%06d.htm" % (d // 31 + 1, d % 31 + 1, i + part * n))
    vals = np.empty(n * value_len, np.uint8)
    soup_len = value_len - 8192
    block = 256
    jobs = [(b, min(n, (b + 1) * block) - b * block, soup_len, part) for b in range((n + block - 1) // block)]
    if workers == 0:
        workers = min(8, os.cpu_count() or 1) if len(jobs) > 4 else 1
    if workers > 1:
        import concurrent.futures as cf
        with cf.ProcessPoolExecutor(workers) as ex:
            soups = list(ex.map(_config3_block, jobs))
    else:
        soups = [_config3_block(j) for j in jobs]
    for (b, count, _, _), soup in zip(jobs, soups):
        for k in range(count):
            i = b * block + k
            o = i * value_len
            vals[o:o + 8192] = tmpl[int(tid[i])]
            vals[o + 8192:o + value_len] = soup[k * soup_len:(k + 1) * soup_len]
    kb, ko = _csr(keys)
    vo = np.arange(n + 1, dtype=np.int64) * value_len
    return Corpus(3, kb, ko, vals, vo)


def config4(n: int = 1_000_000, rec_len: int = 256, part: int = 0) -> Corpus:
    st = Stream(4, part * 1_000_000)
    keys = [b"k%07d" % (i + part * n) for i in range(n)]
    kb, ko = _csr(keys)
    vlen = rec_len - 8
    u = st.uniform(n * vlen)
    letters = (ord("A") + st.randint(0, 16, n * vlen)).astype(np.uint8)
    vals = np.where(u < 0.10, np.uint8(251), letters).astype(np.uint8)
    vo = np.arange(n + 1, dtype=np.int64) * vlen
    return Corpus(4, kb, ko, vals, vo)


def config5(n: int = 10_000, total: int = 65_531, part: int = 0) -> Corpus:
    """Max-size binary records (no byte 251) with planted repeats of earlier records."""
    st = Stream(5, part * 1_000_000)
    keys = [b"bin%07d" % (i + part * n) for i in range(n)]
    kb, ko = _csr(keys)
    vlen = total - 10
    vals = np.empty(n * vlen, np.uint8)
    for i in range(n):
        o = i * vlen
        p = 0
        while p < vlen:
            r = st.u64(4)
            if i > 0 and (int(r[0]) >> 11) * (1.0 / (1 << 53)) < 0.25:
                ln = 32 + int(r[1] % np.uint64(2017))
                ln = min(ln, vlen - p)
                j = i - 1 - int(r[2] % np.uint64(min(64, i)))
                s = int(r[3] % np.uint64(vlen - ln + 1))
                vals[o + p:o + p + ln] = vals[j * vlen + s:j * vlen + s + ln]
            else:
                ln = 256 + int(r[1] % np.uint64(1793))
                ln = min(ln, vlen - p)
                b = (st.u64(ln) % np.uint64(255)).astype(np.uint8)
                b[b >= 251] += 1  # U(0..255) minus {251}
                vals[o + p:o + p + ln] = b
            p += ln
    vo = np.arange(n + 1, dtype=np.int64) * vlen
    return Corpus(5, kb, ko, vals, vo)


def tiny_keys(n: int) -> Corpus:
    """n key-only records "s%06d" (exercises the 65,535-slot chunk rotation)."""
    kb, ko = _csr([b"s%06d" % i for i in range(n)])
    return Corpus(0, kb, ko, np.zeros(0, np.uint8), np.zeros(n + 1, np.int64))


GENERATORS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}
FULL_SIZES = {1: 1000, 2: 100_000, 3: 10_000, 4: 1_000_000, 5: 10_000}


def make(config: int, n: int | None = None, part: int = 0) -> Corpus:
    """Corpus of `config`; `part` selects an independent, same-shaped corpus with
    disjoint keys (one per rank in weak-scaling runs).  part 0 is the canonical corpus."""
    n = FULL_SIZES[config] if n is None else n
    return GENERATORS[config](n, part=part)
