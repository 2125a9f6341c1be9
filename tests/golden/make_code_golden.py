"""Generate tests/golden/codes_pw_nodes.npz: the reference's own host inputs
for the decoders -- the 5G-NR code construction and the node labels -- pinning
codes.construct_pw / codes.identify_nodes.

Runs the reference's Python in this container (it does not travel):
  PolarCodesUtils/CodeConstruction.py:65-84  PolarCodeConstructor.PW
  PolarCodesUtils/IdentifyNodes.py:13-150    NodeIdentifier.run
with a numpy-2 adapter for code written against numpy 1.x: `np.int` (removed
in numpy 1.24) is bound to `int` while the reference runs, and the
constructor's `np.loadtxt(QPath, delimiter="\\n")` (rejected by numpy 2,
CodeConstruction.py:68) is replaced by setting `Q1` exactly as that line
computes it, from the reference's own `reliable sequence.txt`.  The drivers
call NodeIdentifier with use_new_node=False (mainQuantizedDecoder_LLRDomain.py:68);
both settings are stored.

Usage:  python tests/golden/make_code_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

CASES = [(N, K) for N in (16, 32, 64, 128, 256, 512, 1024)
         for K in sorted({1, N // 8, N // 4, N // 2 - 3, N // 2, 3 * N // 4, N - 1})]


def main():
    sys.path.insert(0, REF)
    from PolarCodesUtils.CodeConstruction import PolarCodeConstructor
    from PolarCodesUtils.IdentifyNodes import NodeIdentifier

    seq = np.loadtxt(os.path.join(REF, "reliable sequence.txt")).astype(int)
    had = hasattr(np, "int")
    np.int = int  # numpy-2 adapter (see module doc)
    try:
        out = {"cases": np.array(CASES, dtype=np.int32)}
        for N, K in CASES:
            c = PolarCodeConstructor.__new__(PolarCodeConstructor)
            c.N, c.K = N, K
            c.Q1 = seq[seq < N]  # CodeConstruction.py:69
            frozenbits, msgbits, fmask, mmask = c.PW()
            out[f"frozen_{N}_{K}"] = fmask.astype(np.int8)
            for new in (False, True):
                nt = NodeIdentifier(N, K, frozenbits, msgbits, use_new_node=new).run()
                out[f"nodes{int(new)}_{N}_{K}"] = nt.astype(np.int8)
    finally:
        if not had:
            del np.int
    np.savez_compressed(os.path.join(HERE, "codes_pw_nodes.npz"), **out)
    print(f"{len(CASES)} codes written")


if __name__ == "__main__":
    main()
