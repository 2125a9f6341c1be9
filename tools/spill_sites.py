"""Dev tool: where the register allocator's spill code sits in a decode kernel.

Compiles one unit (default qpd_fast_fscl1.hip, the FastSCL-LUT bench kernel) to
gfx950 assembly with line tables and attributes every scratch load / store and
every SGPR-spill reload (`v_readlane_b32 sN, vM, <lane>`) of the lut_fast_kernel
functions to the source line of the next located instruction (spill code itself
carries line 0).  The per-loop totals come from the compiler's own remarks
(`-Rpass-missed=regalloc`).  CPU only.

usage: python tools/spill_sites.py [unit.hip] [-Dflags...]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quantized_decoder_polar_codes_amd", "csrc")


def main(argv):
    unit = "qpd_fast_fscl1.hip"
    if argv and argv[0].endswith(".hip"):
        unit, argv = argv[0], argv[1:]
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "u.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
               "-I", CSRC, "-gline-tables-only", "--offload-device-only", "-S", os.path.join(CSRC, unit), "-o", asm,
               "-Rpass-missed=regalloc"] + argv
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            sys.exit(p.stderr[-2000:])
        print("allocator remarks (loops with spills / reloads):")
        for line in p.stderr.splitlines():
            if "remark" in line and ("spills" in line or "reloads" in line):
                print("  " + re.sub(r"\s*\[-Rpass-missed=regalloc\]", "", line.replace(CSRC + "/", "")))
        files, pend, sites, infn = {}, [], collections.Counter(), False
        for line in open(asm):
            if line.startswith("_ZN3qpd15lut_fast_kernel") and ":" in line:
                infn = True
                continue
            if infn and line.startswith(".Lfunc_end"):
                infn = False
            m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', line)
            if m:
                files[m.group(1)] = os.path.basename(m.group(2))
                continue
            if not infn:
                continue
            m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
            if m:
                if int(m.group(2)) and pend:
                    where = f"{files.get(m.group(1), '?')}:{m.group(2)}"
                    for k in pend:
                        sites[(where, k)] += 1
                    pend = []
                continue
            s = line.strip()
            if s.startswith("scratch_load"):
                pend.append("scratch load")
            elif s.startswith("scratch_store"):
                pend.append("scratch store")
            elif re.match(r"v_readlane_b32 s\d+, v\d+, \d+\s*$", s):
                pend.append("sgpr reload")
    print("spill code by the source line it precedes:")
    for (where, k), n in sites.most_common(30):
        print(f"  {n:5d}  {k:14s} {where}")


if __name__ == "__main__":
    main(sys.argv[1:])
