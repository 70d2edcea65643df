"""The PX_PROFILE counter indices, read from px_kernels.hip's enum (debug tools only)."""
import os
import re

_src = open(os.path.join(os.path.dirname(__file__), "..", "pixiu_amd", "csrc", "px_kernels.hip")).read()
_enum = re.search(r"enum \{ (P_BYTES.*?) P_N \};", _src, re.S).group(1)
IDX = {n.strip()[2:].lower(): i for i, n in enumerate(_enum.replace("\n", " ").split(",")) if n.strip()}


def counters(buf):
    return {name: buf[i] for name, i in IDX.items()}
