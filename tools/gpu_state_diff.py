"""Debug aid: first divergence of the per-position Ukkonen state (trace build vs oracle)."""
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
def take(f):
    n = f(buf, 1 << 22)
    return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]
def split(tr):
    st, msg = [], []
    i = 0
    while i < len(tr):
        if tr[i][0] <= -100:
            st.append(tr[i] + tr[i + 1] + tr[i + 2]); i += 3
        else:
            msg.append(tr[i][:2]); i += 1
    return st, msg
shown = 0
for seed in [int(x) for x in sys.argv[1:]] or [1, 2, 3]:
    rng = random.Random(seed)
    for trial in range(25):
        alpha = rng.choice(ALPHAS); n = rng.randint(1, 30)
        keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
        take(lib.px_debug_trace_take)
        with px.Store() as st:
            st.set_batch(keys, vals, check=False)
        gs, gm = split(take(lib.px_debug_trace_take))
        take(orc.lib.pxo_trace_take)
        sh = orc.new()
        for k, v in zip(keys, vals): sh.set(k, v)
        os_, om = split(take(orc.lib.pxo_trace_take))
        if gs == os_ and gm == om: continue
        j = next((j for j in range(min(len(gs), len(os_))) if gs[j] != os_[j]), None)
        print(f"seed {seed} trial {trial}: state divergence at step {j}")
        hdr = "(-100-counter, act_node, act_doc, act_direct, act_off, remainder, n_nodes, pools, used)"
        print("  ", hdr)
        if j is not None:
            for q in range(max(0, j - 3), j + 2):
                print("   gpu", gs[q] if q < len(gs) else None)
                print("   orc", os_[q] if q < len(os_) else None)
        shown += 1
        if shown >= 4: sys.exit(0)
