"""Golden vectors for the MinDistortion LUT generator (quantized_decoder_polar_codes_amd/lutgen.py,
csrc/qpd_lutgen.cpp), produced by the REFERENCE's own Python code imported from /root/reference:

* QuantizeDensityEvolution/MinDistortionQuantizer.py:28-99  find_OptLS_quantizer (the pure-Python
  twin of the C++ LLRQuantizer::find_OptLS_quantizer, LLRQuantizer.cpp:67-165);
* QuantizeDensityEvolution/QLLRDensityEvolution_MinDistortion.py:73-126  LLRQuantizerSC.run;
* utils.py:30-45  channel_llr_density_table;
* the GenerateLookUpTable_LLRDomain.py:36-52 channel design steps, restated inline below (a script body).

The reference generator calls the C++ LLRQuantizer (pybind11 + OpenCV), which cannot be built here
(SURVEY.md §8(c)).  As SURVEY.md §8(c) prescribes, the module path it imports
(`quantizers.quantizer.LLROptLSQuantizer`) is served, for this script only, by a three-line adapter
that calls the reference's own Python twin and returns the C++ 4-tuple
(density[1,K], quanta[1,K], lut[1,M], distortion).  The generator under test is therefore pinned in
its `sum_order="numpy"` mode (numpy pairwise sums, as the Python twin); the default "cpp" mode differs
only in summation order inside the DP.

Usage:  python tests/golden/make_lutgen_golden.py     (needs /root/reference; writes lutgen_*.npz)
"""
import importlib.util
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    mdq = _load("ref_MinDistortionQuantizer", os.path.join(REF, "QuantizeDensityEvolution", "MinDistortionQuantizer.py"))
    utils = _load("ref_utils", os.path.join(REF, "utils.py"))

    class LLRQuantizer:  # adapter: the C++ signature/return shape over the reference's Python twin
        def find_OptLS_quantizer(self, density, quanta, M, K):
            d, q, lut = mdq.find_OptLS_quantizer(np.asarray(density).reshape(-1), np.asarray(quanta).reshape(-1), K)
            return d[None], q[None], lut[None], None

    pkg = types.ModuleType("quantizers")
    sub = types.ModuleType("quantizers.quantizer")
    leaf = types.ModuleType("quantizers.quantizer.LLROptLSQuantizer")
    leaf.LLRQuantizer = LLRQuantizer
    sys.modules.update({"quantizers": pkg, "quantizers.quantizer": sub, "quantizers.quantizer.LLROptLSQuantizer": leaf})
    de = _load("ref_QLLRDE", os.path.join(REF, "QuantizeDensityEvolution", "QLLRDensityEvolution_MinDistortion.py"))

    # (1) the DP quantizer on random inputs (ascending unique quanta, as every caller passes)
    rng = np.random.default_rng(42)
    cases = {}
    for i, (M, K) in enumerate([(5, 5), (9, 4), (20, 4), (57, 16), (130, 16), (300, 16), (512, 16), (64, 2)]):
        q = np.sort(rng.normal(0, 4, size=M))
        q = np.unique(q)
        d = rng.random(q.size) ** 3
        d /= d.sum()
        od, oq, lut = mdq.find_OptLS_quantizer(d, q, K)
        cases[f"q{i}_density"], cases[f"q{i}_quanta"], cases[f"q{i}_K"] = d, q, K
        cases[f"q{i}_out_density"], cases[f"q{i}_out_quanta"], cases[f"q{i}_out_lut"] = od, oq, lut
    np.savez_compressed(os.path.join(HERE, "lutgen_optls.npz"), n_cases=8, **cases)
    print("lutgen_optls.npz: 8 DP cases")

    # (2) whole designs (GenerateLookUpTable_LLRDomain.py:36-60 with the Python twin)
    for N, v, snr in [(8, 8, 2.0), (16, 16, 3.0), (32, 16, 3.0)]:
        t = time.time()
        sigma = np.sqrt(1 / 10 ** (snr / 10))
        e = 2 / sigma ** 2
        dd = np.sqrt(2 * e)
        pyx, x_discrete, quanta = utils.channel_llr_density_table(128, -e - 3 * dd, e + 3 * dd, e, -e, dd)
        cd, cq, _, _ = LLRQuantizer().find_OptLS_quantizer(pyx, quanta, 128, v)
        llr_density, llr_quanta, lut_fs, lut_gs = de.LLRQuantizerSC(N, v).run(channel_llr_density=cd,
                                                                           channel_llr_quanta=cq)
        lut_f = np.stack([np.asarray(lut_fs[p][0]) for p in range(N - 1)]).astype(np.uint8)
        lut_g = np.stack([np.asarray(lut_gs[p][0]) for p in range(N - 1)]).astype(np.uint8)
        name = f"lutgen_n{N}_v{v}_snr{snr:.0f}.npz"
        np.savez_compressed(os.path.join(HERE, name), N=N, v=v, design_snr_db=snr, channel_density=cd.reshape(-1),
                            channel_quanta=cq.reshape(-1), lut_f=lut_f, lut_g=lut_g, llr_density=llr_density,
                            llr_quanta=llr_quanta)
        print(f"{name}: {time.time() - t:.1f}s")


if __name__ == "__main__":
    main()
