"""BASELINE config C5 at its own size on the device: one Monte-Carlo point of
10^8 N=1024 K=512 SCL-LUT (L=8) frames (mainQuantizedDecoder_LLRDomain.py:130-203,
MaxBlock = 10^8, no early stop), through an RCCL ("nccl") process group, and
the same point split the way the driver's 8-rank job splits it
(montecarlo.run_point: rank r takes the r-th slice of every step of
8 x batch frames), the ranks run one after the other on this GPU.  The
ranks' counters must sum to the RCCL run's, frame for frame.  With the
driver's stop rule (`Nblkerrs > 1000`), the 8 ranks' slices in lock step must
stop at the same block as the one-rank run, with the crossing frame in a rank
other than 0's.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N, K, L, EBN0 = 1024, 512, 8, 2.0
FRAMES = 10 ** 8
WORLD = 8
BATCH = 1 << 21  # frames per rank per step of the shards (bench.py used 2^21 through round 6 r06r)


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
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def point():
    import bench

    wl = bench.workload(N, K, L, "SCL-LUT", 0, EBN0, device=0)
    return wl.dec, wl.src


def _run(dec, src, batch, max_blocks, stop, **kw):
    from quantized_decoder_polar_codes_amd import montecarlo as MC

    return MC.run_point(src, dec.decode_batch, dec.K, EBN0, batch, max_blocks, stop, A=dec.out_bits,
                        count_device=src.device, gen_decode=src.decode_frames, **kw)


def test_c5_full_point_rccl_equals_eight_rank_shards(rccl, point):
    import torch

    dec, src = point
    a = _run(dec, src, BATCH, FRAMES, None, group=rccl)
    torch.cuda.synchronize()
    assert a.blocks == FRAMES and a.frames_decoded == FRAMES and not a.stopped_early
    parts = [_run(dec, src, BATCH, FRAMES, None, shard=(r, WORLD)) for r in range(WORLD)]
    torch.cuda.synchronize()
    assert sum(p.frames_decoded for p in parts) == FRAMES
    assert all(p.frames_decoded > 0 for p in parts)
    assert sum(p.bit_errors for p in parts) == a.bit_errors
    assert sum(p.block_errors for p in parts) == a.block_errors
    # the driver's MaxBlock BER / BLER (:194-196) at 2 dB: BLER about 6.7e-2
    assert 0.03 < a.bler < 0.12 and a.ber == a.bit_errors / (K * FRAMES)


def test_c5_stop_rule_crossing_outside_rank0(point):
    dec, src = point
    batch = 1024
    one = _run(dec, src, WORLD * batch, FRAMES, 1000)
    eight = _run(dec, src, batch, FRAMES, 1000, virtual_world=WORLD)
    assert one.stopped_early and eight.stopped_early
    assert (one.blocks, one.bit_errors, one.block_errors, one.ber, one.bler) == \
        (eight.blocks, eight.bit_errors, eight.block_errors, eight.ber, eight.bler)
    assert one.block_errors == 1001
    assert (one.blocks % (WORLD * batch)) // batch != 0  # the crossing frame is in another rank's slice
