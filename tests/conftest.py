import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqpd.so on cuda:0)")
    config.addinivalue_line("markers", "host_engine: a gpu test that exercises the host engine on purpose "
                                       "(the kernels-only fixture below leaves QPD_HOST_ENGINE alone)")


ENGINE_NAMES = {0: "none", 1: "gpu", 2: "host"}  # qpd_info.last_engine (enum qpd_ran, include/qpd.h)


@pytest.fixture(autouse=True)
def _gpu_tests_run_the_kernels(request, monkeypatch):
    """Every -m gpu test runs the HIP kernels: host-buffer calls of a few frames
    would otherwise go to the host engine (qpd_decode_host below
    qpd_info.host_max_frames), and a "GPU" parity case would test C++.  Decoders
    read QPD_HOST_ENGINE when they are created.  Tests of the host engine itself
    carry the host_engine marker and choose their engine explicitly."""
    if request.node.get_closest_marker("gpu") is None or request.node.get_closest_marker("host_engine") is not None:
        return
    monkeypatch.setenv("QPD_HOST_ENGINE", "gpu")


def golden_files(pattern="*.npz"):
    """Decoder fixtures.  The default pattern gives the LUT and SC decoders'
    fixtures; the LUT-generator (lutgen_*.npz) and float-domain (float_*.npz)
    fixtures and the code-construction pin (codes_*.npz) have their own tests
    and are returned only when asked for."""
    own = ("lutgen_", "float_", "codes_")
    return sorted(p for p in glob.glob(os.path.join(GOLDEN_DIR, pattern))
                  if pattern.startswith(own) or not os.path.basename(p).startswith(own))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_packed(g):
    from quantized_decoder_polar_codes_amd.lut import PackedLUT

    return PackedLUT(N=int(g["N"]), v=int(g["v"]), lut_f=g["lut_f"], f_base=g["f_base"], f_step=int(g["f_step"]),
                     lut_g=g["lut_g"], g_base=g["g_base"], g_step=int(g["g_step"]),
                     vcl=np.ascontiguousarray(g["vcl"]))


@pytest.fixture(scope="session")
def native_lib():
    from quantized_decoder_polar_codes_amd import build

    build.build_native()
    from quantized_decoder_polar_codes_amd import _lib

    return _lib.load()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.lib()
    return oracle


def frame_lanes(info, frame):
    """Where a frame runs in the kernels: (task, frame set, lanes).  Fast
    engine: a task is frames_per_wave consecutive frames, set s holds
    64 / lanes_per_frame of them, frame slot k of a set owns lanes
    [k * lanes_per_frame, (k + 1) * lanes_per_frame)."""
    fpw_task = int(info["frames_per_wave"])
    gs = int(info["lanes_per_frame"])
    per_set = max(1, 64 // gs)
    slot = frame % fpw_task
    k = slot % per_set
    return frame // fpw_task, slot // per_set, (k * gs, (k + 1) * gs - 1)


def assert_engine(dec, engine):
    """The decoder's last decode call ran on `engine` ("gpu": the kernels; "host":
    the host engine); None skips the check."""
    if dec is None or engine is None:
        return
    ran = ENGINE_NAMES.get(int(dec.info()["last_engine"]), "?")
    assert ran == engine, f"the last decode ran on the {ran} engine, this check is for the {engine} engine"


def assert_frames_equal(got, want, dec=None, label="", redecode=None, inputs=None, engine="gpu"):
    """Bit-exact frame comparison that explains a mismatch instead of only
    counting it: for each differing frame (up to 8) the task / frame set /
    lanes it ran on, the differing bit positions and both bit strings; with
    `redecode(rows) -> bits` the differing frames are decoded again, alone, in
    a fresh decoder, which separates a deterministic difference (same result
    alone) from one that depended on the run.  Everything is also written as
    JSON to $QPD_DIAG_DIR (default gpurun_out/), which gpurun copies back.
    With `dec`, the decoder's last decode must have run on `engine` (default
    the GPU kernels; None: no check)."""
    import json

    assert_engine(dec, engine)

    got = np.asarray(got)
    want = np.asarray(want)
    assert got.shape == want.shape, (got.shape, want.shape)
    bad = np.flatnonzero((got != want).reshape(len(got), -1).any(1))
    if bad.size == 0:
        return
    info = dec.info() if dec is not None else None
    rec = {"label": label, "frames": int(len(got)), "differing": bad.tolist(), "info": info, "detail": []}
    alone = redecode(bad) if redecode is not None else None
    lines = [f"{label}: {bad.size}/{len(got)} frames differ"]
    for i, f in enumerate(bad[:8]):
        pos = np.flatnonzero(got[f] != want[f])
        d = {"frame": int(f), "bits_differ": pos.tolist(),
             "got": "".join(map(str, got[f].astype(int))), "want": "".join(map(str, want[f].astype(int)))}
        where = ""
        if info is not None:
            t, s, ln = frame_lanes(info, int(f))
            d.update(task=t, set=s, lanes=list(ln))
            where = f" (task {t}, set {s}, lanes {ln[0]}-{ln[1]})"
        if alone is not None:
            d["alone_equals_want"] = bool(np.array_equal(alone[i], want[f]))
            d["alone_equals_got"] = bool(np.array_equal(alone[i], got[f]))
        if inputs is not None:
            d["input"] = np.asarray(inputs[f]).tolist()
        rec["detail"].append(d)
        lines.append(f"  frame {f}{where}: {pos.size} bits differ at {pos[:24].tolist()}"
                     + ("" if alone is None else f"; alone in a fresh decoder: "
                        f"{'= oracle' if d['alone_equals_want'] else ('= this run' if d['alone_equals_got'] else 'a third result')}"))
    out_dir = os.environ.get("QPD_DIAG_DIR", os.path.join(ROOT, "gpurun_out"))
    try:
        os.makedirs(out_dir, exist_ok=True)
        safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in label)[:120] or "mismatch"
        with open(os.path.join(out_dir, f"parity_fail_{safe}.json"), "w") as fh:
            json.dump(rec, fh, indent=1)
    except OSError:
        pass
    pytest.fail("\n".join(lines))
