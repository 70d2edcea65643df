"""Debug aid: decoder counters (prof build) of the set batch of tests/test_gpu_spans.py's
deep reference chains: frames spilled past the LDS lane stack (d_spill) and walks sent to
the serial machine for depth (df_depth)."""
import ctypes as C, os, sys
os.environ["PIXIU_AMD_LIB"] = os.path.join(os.path.dirname(__file__), "..", "pixiu_amd", "libpixiu_amd_prof.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch  # noqa: F401  (probes the device before the library initialises HIP)
import pixiu_amd as px
from decode_profile_names import counters


def _chain_docs(seed, n, size):  # (the same docs as tests/test_gpu_spans.py's)
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 256, size, dtype=np.uint8)
    vals = [v.tobytes()]
    for _ in range(n - 1):
        v = np.insert(v, int(rng.integers(0, len(v) + 1)), np.uint8(rng.integers(0, 256)))
        vals.append(v.tobytes())
    return [b"c%04d" % i for i in range(n)], vals


n, rps = int(sys.argv[1]) if len(sys.argv) > 1 else 96, int(sys.argv[2]) if len(sys.argv) > 2 else 48
keys, vals = _chain_docs(11, n, 1500)
lib = px.load_library()
lib.px_debug_prof_take.argtypes = [C.c_void_p, C.c_uint32]
buf = (C.c_ulonglong * 128)()
with px.Store(records_per_shard=rps) as st:
    lib.px_debug_prof_take(buf, 128)
    st.set_batch(keys, vals)
    lib.px_debug_prof_take(buf, 128)
    v = counters(buf)
    print(f"chain docs n {n} rps {rps}: set batch decodes")
    for k in ("d_batch", "d_serial", "d_push", "d_spill", "df_depth", "df_lper", "df_topref", "df_cap"):
        print(f"  {k:10s} {v[k]:12d}")
