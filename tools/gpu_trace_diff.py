"""Debug aid: for fuzz cases whose GPU output differs from the oracle, compare the
per-byte encoder message streams (trace build) and report the first divergence."""
import ctypes as C, os, random, sys
os.environ["PIXIU_AMD_LIB"] = os.path.join(os.path.dirname(__file__), "..", "pixiu_amd", "libpixiu_amd_trace.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pixiu_amd as px
from _oracle import Oracle, assemble
from test_gpu_parity import _gen, ALPHAS

lib = px.load_library()
lib.px_debug_trace_take.argtypes = [C.c_void_p, C.c_uint32]
orc = Oracle()
buf = (C.c_int * (1 << 22))()

def gpu_trace():
    n = lib.px_debug_trace_take(buf, 1 << 22)
    return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]

def oracle_trace(keys, vals):
    orc.lib.pxo_trace_take(buf, 1 << 22)
    sh = orc.new()
    for k, v in zip(keys, vals):
        sh.set(k, v)
    n = orc.lib.pxo_trace_take(buf, 1 << 22)
    return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]

shown = 0
for seed in [int(x) for x in sys.argv[1:]] or [1, 2, 3]:
    rng = random.Random(seed)
    for trial in range(25):
        alpha = rng.choice(ALPHAS)
        n = rng.randint(1, 30)
        keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
        gpu_trace()
        with px.Store() as st:
            res = st.set_batch(keys, vals, check=False)
        g = gpu_trace()
        o = oracle_trace(keys, vals)
        gg = [(a, b) for a, b, _ in g]
        oo = [(a, b) for a, b, _ in o]
        if gg == oo:
            continue
        j = next((j for j in range(min(len(gg), len(oo))) if gg[j] != oo[j]), min(len(gg), len(oo)))
        # locate doc and position
        docs = [assemble(k, v) for k, v in zip(keys, vals)]
        acc, d = 0, 0
        while d < len(docs) and acc + len(docs[d]) <= j:
            acc += len(docs[d]); d += 1
        print(f"seed {seed} trial {trial} alpha {alpha[:6]!r}: first divergence at msg {j} (doc {d} pos {j-acc}) "
              f"gpu {gg[j] if j < len(gg) else None} oracle {oo[j] if j < len(oo) else None} status {res['status'].tolist()[:d+1]}")
        print("   gpu ctx", gg[max(0, j - 6):j + 3])
        print("   orc ctx", oo[max(0, j - 6):j + 3])
        if shown == 0:
            print("   doc bytes around:", list(docs[d][max(0, j - acc - 10):j - acc + 5]) if d < len(docs) else None)
        shown += 1
print("divergent trials:", shown)
