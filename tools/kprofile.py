"""Static code-size profile of a decode kernel: instructions per source
function (from the -gline-tables-only .loc lines of the ISA).
usage: python tools/kprofile.py ISA.s [kernel-substring]"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "quantized_decoder_polar_codes_amd", "csrc")
fn_at = {}
for f in os.listdir(CS):
    if not f.endswith((".hip", ".hpp")):
        continue
    cur = "?"
    starts = []
    for i, line in enumerate(open(os.path.join(CS, f)), 1):
        m = re.match(r"^(?:template\s*<.*>\s*)?(?:__global__|__device__|static __device__)[^(]*?(\w+)\s*\(", line)
        if m:
            cur = m.group(1)
        elif re.match(r"^(?:__global__|__device__)", line):
            cur = line.split("(")[0].split()[-1]
        starts.append(cur)
    fn_at[f] = starts
src = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "lut_fast_kernel"
files, cur, inside = {}, None, False
cnt = collections.Counter()
for line in open(src):
    if re.match(r"^_Z\w+:", line):
        inside = want in line
        continue
    if line.startswith(".Lfunc_end"):
        inside = False
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', line)
    if m:
        files[m.group(1)] = os.path.basename(m.group(2))
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
    if m:
        f, ln = files.get(m.group(1), "?"), int(m.group(2))
        cur = f"{f}:{fn_at[f][ln - 1] if f in fn_at and 0 < ln <= len(fn_at[f]) else ln}"
        continue
    s = line.strip()
    if inside and s and not s.startswith((".", ";", "_", "/")) and not s.endswith(":"):
        cnt[cur] += 1
tot = sum(cnt.values())
print(f"{tot} instructions")
for k, v in cnt.most_common(40):
    print(f"{v:7d} {100 * v / tot:5.1f}%  {k}")
