"""Debug aid: k_gst_encode per-category counters and cycles (prof build)."""
import ctypes as C, os, sys
os.environ["PIXIU_AMD_LIB"] = os.path.join(os.path.dirname(__file__), "..", "pixiu_amd", "libpixiu_amd_prof.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import pixiu_amd as px
from pixiu_amd import synth
NAMES = ["bytes", "ff_calls", "ff_bytes", "pass", "iters", "lookups", "probes", "root", "walk", "link", "canon_lvl",
         "t_total", "t_ff", "t_derive", "t_walk", "t_split", "t_grow", "t_canon", "t_end", "t_root", "t_enc", "keymiss", "t_key", "t_look", "d_batch", "d_laneit", "d_serial", "d_commit", "d_flagged", "d_short", "d_push", "d_t_total", "d_t_lane", "g_nosplit", "g_t_leaf", "g_t_split", "g_t_add",
         "e_look", "e_off1", "e_off2", "e_off3", "e_off4p", "k_cached", "k_load1", "k_loadn"]
lib = px.load_library()
lib.px_debug_prof_take.argtypes = [C.c_void_p, C.c_uint32]
cfg, n, rps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cp = synth.make(cfg, n)
buf = (C.c_ulonglong * 64)()
lib.px_debug_prof_take(buf, 64)
with px.Store(records_per_shard=rps) as st:
    st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    ms = st.stats()["last_set_stage_ms"]
k = lib.px_debug_prof_take(buf, 64)
v = dict(zip(NAMES, buf[:k]))
b = max(v["bytes"], 1)
print(f"config {cfg} n {n} rps {rps}: kernel {ms:.1f} ms")
for name in NAMES:
    if name.startswith("d_"):
        continue
    x = v[name]
    per = x / b
    print(f"  {name:10s} {x:16d}  per byte {per:10.3f}" + (f"  ({x / max(v['t_total'],1) * 100:5.1f}% of wave time)" if name.startswith("t_") and name != "t_total" or name == "t_total" else ""))
