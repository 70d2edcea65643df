"""Attribute a kernel's static instructions to source lines (from the .loc
directives of a `-g` assembly listing), weighted by loop depth, to find the
source lines that expand into the most scalar/vector instructions.
  hipcc --offload-arch=gfx950 -O3 -g -std=c++17 --cuda-device-only -S px_kernels.hip -o kg.s
  python tools/isa_lines.py kg.s k_gst_encode [min_depth]"""
import collections, re, sys

path, want = sys.argv[1], sys.argv[2]
min_depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lines = open(path).read().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % want, l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
depth, loc = 0, ("?", 0)
by = collections.defaultdict(collections.Counter)
for l in lines[start + 1:end]:
    s = l.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
    if m:
        loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    if re.match(r"^[\w.$]+:", s) or (s.startswith(";") and "Depth=" in s):
        m = re.search(r"Depth=(\d+)", s)
        depth = int(m.group(1)) if m else (0 if re.match(r"^[\w.$]+:", s) else depth)
        continue
    if not s or s.startswith((".", ";")) or depth < min_depth:
        continue
    op = s.split()[0]
    cat = "spill" if op in ("v_readlane_b32", "v_writelane_b32") else op[:2]
    by[loc][cat] += 1
tot = sorted(by.items(), key=lambda kv: -sum(kv[1].values()))
for (f, ln), c in tot[:45]:
    print(f"{f}:{ln:<5d} total {sum(c.values()):4d}  s_ {c['s_']:4d}  v_ {c['v_']:4d}  spill {c['spill']:3d}")
