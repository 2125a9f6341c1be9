"""BASELINE config 5's collective path on the device: an RCCL ("nccl") process
group of world size 1 on cuda:0 (loopback TCP store), through which
bench.rank_job and montecarlo.run_point run exactly as they do on the driver's
8-GPU node.  The counters, the block the driver's stop rule ends at
(mainQuantizedDecoder_LLRDomain.py:130-203, `Nblkerrs > 1000`) and the
throughput line's BER/BLER must equal the group-less run on the same frames.
More ranks than GPUs cannot share one device under RCCL; the N-rank sharding
itself is covered on CPU with gloo (tests/test_bench.py, test_montecarlo.py).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N, K, L, EBN0 = 1024, 512, 8, 2.0


@pytest.fixture(scope="module")
def rccl(native_lib):
    import torch
    import torch.distributed as dist

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def make():
    import bench

    base = bench.workload(N, K, L, "SCL-LUT", 0, EBN0, device=0)  # one table design, one decoder

    def mk(frame0, frames):
        msg, sym = base.src(frame0, frames) if frames else (None, None)
        return bench.Workload(base.dec, base.src, base.packed, base.fm, base.nt, msg, sym, frame0)

    return mk


def test_rccl_all_reduce_on_device(rccl):
    import torch
    import torch.distributed as dist

    t = torch.tensor([3, 5, 7], dtype=torch.int64, device="cuda:0")
    dist.all_reduce(t, group=rccl)
    m = torch.tensor([1.5], dtype=torch.float64, device="cuda:0")
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=rccl)
    torch.cuda.synchronize()
    assert t.tolist() == [3, 5, 7] and m.item() == 1.5


@pytest.mark.parametrize("stop", [1000, None])
def test_run_point_through_rccl_equals_groupless(stop, rccl, make):
    """The driver's loop (fused generate + decode + device counters), with and
    without its stop rule, through the RCCL group and without one."""
    from quantized_decoder_polar_codes_amd import montecarlo as MC

    wl = make(0, 0)
    dec, src = wl.dec, wl.src
    F, B = 60_000, 8192
    res = {}
    for name, grp in (("rccl", rccl), ("none", None)):
        res[name] = MC.run_point(src, dec.decode_batch, dec.K, EBN0, B, F, stop, A=dec.out_bits, group=grp,
                                 count_device=src.device, gen_decode=src.decode_frames)
    a, b = res["rccl"], res["none"]
    assert (a.bit_errors, a.block_errors, a.blocks, a.frames_decoded, a.stopped_early) == \
        (b.bit_errors, b.block_errors, b.blocks, b.frames_decoded, b.stopped_early)
    if stop is not None:  # at 2 dB the point stops inside the 60 000 frames (BLER ~ 6.7e-2)
        assert a.stopped_early and a.block_errors == stop + 1 and a.blocks < F
    else:
        assert a.blocks == F and a.block_errors > 0


def _args(argv):
    import bench

    return bench.parse(argv + ["--N", str(N), "--K", str(K), "--L", str(L), "--ebn0", str(EBN0)])


def _ctx(rank_group):
    import torch

    import bench

    return bench.Ctx(0, 1, torch.device("cuda", 0), rank_group)


def test_bench_mc_mode_through_rccl(rccl, make):
    """bench.py --mc-frames (config C5's per-rank body) through the RCCL group:
    the same counters and stop block as the group-less run."""
    import bench

    out = {}
    for name, grp in (("rccl", rccl), ("none", None)):
        args = _args(["--mc-frames", "40000", "--frames", "8192", "--mc-stop", "1000"])
        out[name], _ = bench.rank_job(args, _ctx(grp), make)
    a, b = out["rccl"], out["none"]
    for k in ("bit_errors", "block_errors", "blocks", "frames_decoded", "stopped_early", "ber", "bler"):
        assert a[k] == b[k], k
    assert a["stopped_early"] and a["block_errors"] == 1001


def test_bench_throughput_line_through_rccl(rccl, make):
    """The throughput body (resident frames, timed steps, counter and wall
    all-reduces over RCCL, end-to-end Monte-Carlo leg): BER/BLER and frame
    counts equal the group-less run; the bench's parity leg runs on it."""
    import bench

    out = {}
    for name, grp in (("rccl", rccl), ("none", None)):
        args = _args(["--frames", "16384", "--steps", "2", "--warmup", "1"])
        out[name], wl = bench.rank_job(args, _ctx(grp), make)
    a, b = out["rccl"], out["none"]
    for k in ("ber", "bler", "frames_counted", "n_gpus"):
        assert a[k] == b[k], k
    assert a["value"] > 0 and a["monte_carlo_e2e"]["value"] > 0
    # the parity leg the bench runs on rank 0 at any world size (small sample)
    args = _args(["--frames", "16384", "--cpu-baseline-seconds", "2", "--cpu-workers", "4"])
    bench.parity_and_baseline(args, wl, a)
    ps = a["parity_sample"]
    assert ps["frames"] > 0 and all(v for k, v in ps.items() if k.startswith("bit_exact_vs_"))
