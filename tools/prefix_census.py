"""Share of the f/g table lookups done while a frame has 1, 2, 4 or L live list
paths (SCL traversal of SCLLUTDecoder.cpp; FastSCL with IdentifyNodes' special
nodes), for the frozen-prefix stages of the fast engine.
usage: python tools/prefix_census.py [N K L]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantized_decoder_polar_codes_amd import codes as C  # noqa: E402

N, K, L = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (1024, 512, 8)
n = N.bit_length() - 1
_, mb, fm, _ = C.construct_pw(N, K)
nt = C.identify_nodes(N, mb)
print(f"N={N} K={K} L={L}: first information leaves {list(mb[:4])}")


def census(fast):
    ops, live = [], [1]

    def rec(d, node):
        t = nt[(1 << d) + node - 1] if fast else -1
        if fast and d > 0 and t in (0, 1, 2, 3):
            ops.append(("special", N >> d, live[0]))
            if t in (1, 2):  # R1: one fork per layer; REP: one fork
                live[0] = min(L, live[0] * (2 ** min(N >> d, 3) if t == 1 else 2))
            return
        if d == n:
            ops.append(("leaf", 1, live[0]))
            if fm[node] == 0:
                live[0] = min(L, live[0] * 2)
            return
        ops.append(("fg", (N >> d) // 2, live[0]))
        rec(d + 1, 2 * node)
        ops.append(("fg", (N >> d) // 2, live[0]))
        rec(d + 1, 2 * node + 1)

    rec(0, 0)
    return ops


for fast in (False, True):
    ops = census(fast)
    tot = sum(w for k, w, _ in ops if k == "fg")
    for lv in sorted({lv for _, _, lv in ops}):
        s = sum(w for k, w, l in ops if k == "fg" and l == lv)
        print(f"{'FastSCL' if fast else 'SCL':8s} live paths {lv}: f/g lookups per path {s:6d} ({100 * s / tot:4.1f} %)")
