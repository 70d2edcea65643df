"""Static instruction mix of one kernel in a gfx950 assembly listing, split by loop
depth (the compiler's "Loop: Header=... Depth=N" block annotations): a cheap proxy
for dynamic instruction counts while iterating on a kernel.
  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S px_kernels.hip -o k.s
  python tools/isa_mix.py k.s k_gst_encode"""
import collections, re, sys

path, want = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % want, l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
depth = 0
by = collections.defaultdict(collections.Counter)
for l in lines[start + 1:end]:
    s = l.strip()
    if re.match(r"^[\w.$]+:", s):  # block label: depth from its annotation
        m = re.search(r"Depth=(\d+)", s)
        depth = int(m.group(1)) if m else 0
        continue
    if s.startswith(";") and "Depth=" in s and ("Loop:" in s or "This" in s):
        m = re.search(r"Depth=(\d+)", s)
        depth = int(m.group(1))
        continue
    if not s or s.startswith((".", ";")):
        continue
    op = s.split()[0]
    cat = ("wait" if op.startswith("s_waitcnt") else "br" if "branch" in op else "spill" if op in ("v_readlane_b32", "v_writelane_b32")
           else "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "lds" if op.startswith("ds_") else "other")
    by[depth][cat] += 1
cats = ["salu", "valu", "spill", "br", "wait", "vmem", "lds", "other"]
print("depth " + " ".join(f"{c:>6}" for c in cats) + "  total")
for d in sorted(by):
    print(f"{d:5d} " + " ".join(f"{by[d][c]:6d}" for c in cats) + f"  {sum(by[d].values()):6d}")
tot = collections.Counter()
for d in by: tot.update(by[d])
print("  all " + " ".join(f"{tot[c]:6d}" for c in cats) + f"  {sum(tot.values()):6d}")
m = re.search(r"\.sgpr_spill_count:\s*(\d+)", "\n".join(lines[end:end + 4000]))
