"""TEST/DESIGN PROTOTYPE ONLY: tools/proto/pool_proto.cpp (MemPool accounting from a
suffix array) against the oracle's walk (pxo_pool_trace), pools / used after every doc.
  g++ -O2 -shared -fPIC -o /tmp/pp/libpool.so tools/proto/pool_proto.cpp
  python tools/proto/pool_check.py /tmp/pp/libpool.so"""
import ctypes as C
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _oracle import Oracle, _csr, _p, assemble  # noqa: E402
from pixiu_amd import synth  # noqa: E402

lib = C.CDLL(sys.argv[1])
orc = Oracle()


def check(name, docs):
    n = len(docs)
    db, do = _csr(docs)
    ch = np.zeros(n, np.uint32)
    po = np.zeros(n, np.int32)
    uo = np.zeros(n, np.int32)
    rc = orc.lib.pxo_pool_trace(C.c_int(n), _p(db), _p(do), _p(ch), _p(po), _p(uo))
    assert rc == 0, rc
    m = int(np.searchsorted(ch, 1)) if ch[-1] > 0 else n  # docs of the first chunk
    pp = np.zeros(n, np.int32)
    uu = np.zeros(n, np.int32)
    st = np.zeros(8, np.uint64)
    t0 = time.time()
    lib.pool_proto(C.c_int(m), _p(db), _p(do), C.c_int(1), C.c_int(5), _p(pp), _p(uu), _p(st))
    bad = [i for i in range(m) if (pp[i], uu[i]) != (po[i], uo[i])]
    print(f"{name}: {m}/{n} docs, {int(do[m])} B, pools {po[m-1]} used {uo[m-1]}, leaves {st[0]} splits {st[1]} "
          f"one-sided {st[2]} climb steps {st[3]} ({st[3]/max(st[2],1):.2f}/climb, max {st[5]}) cand {st[4]} "
          f"{time.time()-t0:.1f}s -> {'OK' if not bad else 'MISMATCH at doc %d: %s vs %s' % (bad[0], (pp[bad[0]], uu[bad[0]]), (po[bad[0]], uo[bad[0]]))}")
    return not bad


ok = True
for cfg, nrec in (((2, 1500), (3, 25), (4, 5000), (5, 20)) if len(sys.argv) <= 2 else ()):
    cp = synth.make(cfg, nrec)
    ok &= check(f"config {cfg}", [assemble(cp.key(i), cp.val(i)) for i in range(cp.n)])
rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 7)
for trial in range(int(sys.argv[3]) if len(sys.argv) > 3 else 60):
    alpha = rng.choice([b"ab", b"abc", b"ab\xfb", b"a\xfb\x00\x02", b"abcd", bytes(range(256))])
    docs = []
    for _ in range(rng.randint(1, 60)):
        k = bytes(rng.choice(alpha) for _ in range(rng.randint(1, 12)))
        v = bytes(rng.choice(alpha) for _ in range(rng.randint(0, 400)))
        docs.append(assemble(k, v))
    ok &= check(f"fuzz {trial}", docs)
print("ALL OK" if ok else "FAILURES")
