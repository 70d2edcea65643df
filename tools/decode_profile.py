"""Debug aid: k_decode batch/serial counters (prof build), one config batch."""
import ctypes as C, os, sys
os.environ["PIXIU_AMD_LIB"] = os.path.join(os.path.dirname(__file__), "..", "pixiu_amd", "libpixiu_amd_prof.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import pixiu_amd as px
from pixiu_amd import synth
import re
from decode_profile_names import IDX
NAMES = ["d_batch", "d_laneit", "d_serial", "d_commit", "d_flagged", "d_short", "d_push", "d_t_total", "d_t_lane",
         "df_none", "df_topref", "df_cap", "df_nolink", "df_over", "df_lper", "df_depth", "df_range", "df_badrec",
         "d_topb", "d_subb", "d_topc", "d_maxit", "d_t_assign", "d_rounds", "d_spill"]
lib = px.load_library()
lib.px_debug_prof_take.argtypes = [C.c_void_p, C.c_uint32]
cfg, n, rps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
waves = int(sys.argv[4]) if len(sys.argv) > 4 else 0
cp = synth.make(cfg, n)
keys_host = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
out_cap = int(2 * cp.raw_bytes + 256 * n + (1 << 20))
out = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
buf = (C.c_ulonglong * 128)()
with px.Store(records_per_shard=rps, decode_waves=waves) as st:
    lib.px_debug_prof_take(buf, 128)
    st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    lib.px_debug_prof_take(buf, 128)
    # the set batch's decodes: key prefixes and the span build (k_decode_addr)
    v = {name: buf[IDX[name]] for name in NAMES}
    print(f"config {cfg} n {n} rps {rps}: set batch decodes (key prefixes + span tables)")
    for name in NAMES:
        print(f"  {name:10s} {v[name]:16d}  per record {v[name] / n:12.1f}")
    print(f"  lane iterations per batch {v['d_laneit'] / max(v['d_batch'], 1):.2f}, committed per batch {v['d_commit'] / max(v['d_batch'], 1):.2f}")
    print(f"  lane-phase share of wave time {v['d_t_lane'] / max(v['d_t_total'], 1) * 100:.1f}%")
    print(f"  assignment share of wave time {v['d_t_assign'] / max(v['d_t_total'], 1) * 100:.1f}%")
    rc, off, ln, sts, need = st.get_batch_device(keys_host, out.data_ptr(), out_cap, px.COMPAT)
    ms = st.stats()["last_decode_kernel_ms"]
k = lib.px_debug_prof_take(buf, 128)
v = {name: buf[IDX[name]] for name in NAMES}
print(f"config {cfg} n {n} rps {rps} waves {waves}: decode kernel {ms:.2f} ms, expanded {int(np.asarray(ln).sum())} B")
for name in NAMES:
    print(f"  {name:10s} {v[name]:16d}  per query {v[name] / n:12.1f}")
print(f"  lane iterations per batch {v['d_laneit'] / max(v['d_batch'], 1):.2f}, committed per batch {v['d_commit'] / max(v['d_batch'], 1):.2f}")
print(f"  lane-phase share of wave time {v['d_t_lane'] / max(v['d_t_total'], 1) * 100:.1f}%")
