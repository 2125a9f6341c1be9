"""bench.py's own multi-rank path on CPU (gloo): frame sharding by global frame
id, the counter and wall all-reduces, n_gpus / value reporting, the end-to-end
rate and the Monte-Carlo mode (BASELINE config 5) -- with a stand-in decoder,
since the real one needs the GPU (its parity is tests/test_gpu_*.py)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

N, K = 16, 8


def frame_bits(frame0, B):
    """Deterministic 'channel' per global frame id: the stand-in decoder's
    output bits; the message is all zeros, so the errors are these ones."""
    gid = np.arange(frame0, frame0 + B, dtype=np.uint64)[:, None]
    j = np.arange(N, dtype=np.uint64)[None, :]
    h = ((gid * np.uint64(0x9E3779B97F4A7C15)) ^ (j * np.uint64(0xBF58476D1CE4E5B9))) >> np.uint64(59)
    return (h == 0).astype(np.int32)  # ~1/32 of the positions


class FakeDecoder:
    """decode_batch(sym) -> the first K symbols as bits (CPU torch)."""

    def __init__(self):
        self.N, self.K, self.out_bits = N, K, K

    def decode_batch(self, sym):
        return sym[:, :K].to(dtype=__import__("torch").uint8)


def fake_make(seen_ranges):
    import torch

    def src(frame0, B):
        seen_ranges.append((frame0, B))
        return torch.zeros((B, K), dtype=torch.uint8), torch.from_numpy(frame_bits(frame0, B))

    def make(frame0, frames):
        dec = FakeDecoder()
        msg, sym = src(frame0, frames) if frames else (None, None)
        return bench.Workload(dec, src, None, None, None, msg, sym, frame0)

    return make


def expected(frame_ranges):
    bits = np.concatenate([frame_bits(f0, B)[:, :K] for f0, B in frame_ranges])
    return int(bits.sum()), int((bits.sum(1) > 0).sum()), len(bits)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, argv, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = bench.parse(argv)
        ctx = bench.Ctx(rank, world, torch.device("cpu"), dist.group.WORLD)
        ranges = []
        res, wl = bench.rank_job(args, ctx, fake_make(ranges))
        q.put((rank, res, ranges))
    finally:
        dist.destroy_process_group()


def run_world(world, argv):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, ranges = q.get(timeout=120)
        out[rank] = (res, ranges)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world", [1, 2])
def test_bench_rank_job_shards_and_reduces(world):
    F, steps = 96, 3
    out = run_world(world, ["--frames", str(F), "--steps", str(steps), "--warmup", "1", "--N", str(N), "--K", str(K)])
    res = out[0][0]
    assert all(out[r][0] is None for r in range(1, world))  # only rank 0 reports
    # rank r decoded global frames [r*F, (r+1)*F): disjoint, covering [0, world*F)
    first = sorted(out[r][1][0] for r in range(world))
    assert first == [(r * F, F) for r in range(world)]
    bit, blk, frames = expected(first)
    assert res["n_gpus"] == world and res["frames_counted"] == frames == world * F
    assert res["ber"] == bit / (frames * K) and res["bler"] == blk / frames
    assert res["value"] == pytest.approx(world * F * steps / (res["ms_per_step"] * steps / 1e3))
    assert res["metric"] == bench.METRIC and res["scaling"] == "weak"
    # the end-to-end leg generated new frames on every rank (beyond the resident ones)
    e2e = res["monte_carlo_e2e"]
    assert e2e["value"] > 0
    for r in range(world):
        later = out[r][1][1:]
        assert len(later) == 1 + steps and all(B == F and f0 >= (1 << 40) for f0, B in later)


@pytest.mark.parametrize("world,stop", [(1, 0), (2, 0), (2, 20)])
def test_bench_monte_carlo_mode_matches_single_process(world, stop):
    """--mc-frames: the sharded Monte-Carlo point gives the counters of the
    driver loop over global frames [0, F), whatever the rank count."""
    from quantized_decoder_polar_codes_amd import montecarlo as MC

    F, B = 1000, 64
    argv = ["--mc-frames", str(F), "--frames", str(B), "--N", str(N), "--K", str(K), "--mc-stop", str(stop)]
    res = run_world(world, argv)[0][0]
    want = MC.run_point(lambda f0, n: (np.zeros((n, K), np.uint8), frame_bits(f0, n)[:, :K].astype(np.uint8)),
                        lambda s: s, K, 2.0, B, F, stop if stop else None)
    assert (res["bit_errors"], res["block_errors"], res["blocks"], res["stopped_early"]) == \
        (want.bit_errors, want.block_errors, want.blocks, want.stopped_early)
    assert res["n_gpus"] == world and res["value"] > 0


def test_launch_cmd_is_torchrun_with_loopback():
    args = bench.parse(["--gpus", "8", "--steps", "3"])
    cmd = bench.launch_cmd(args, ["--gpus", "8", "--steps", "3"], 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
