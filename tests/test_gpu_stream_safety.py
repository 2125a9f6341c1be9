"""One decoder handle across streams and host threads (SURVEY.md §8(b):
"thread-safe per handle per stream"; the reference's decode is one synchronous
call under the GIL, py_SCLLUTDecoder.cpp:15).

A decoder owns work buffers (global slab, pre-pass rows, task-queue counter,
error word, host staging), so calls on different streams must not overlap.
The library orders them itself (qpd_capi.hip: order_on / mark_on, a per-handle
mutex).  Each test issues work that WOULD overlap without that ordering -- a
large decode still running on one stream when the next call starts on another
-- and checks every result against the oracle or a separately decoded copy.
The task-queue counter is never reset (qpd_common.hpp: wave_take); a counter
started just below 2^32 checks the wrap-around deterministically.
"""
import threading

import numpy as np
import pytest

from conftest import assert_frames_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qpd(native_lib):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import quantized_decoder_polar_codes_amd as Q

    return Q


def _code(N, K):
    from quantized_decoder_polar_codes_amd import codes as C

    _, mb, fm, mm = C.construct_pw(N, K)
    return fm, C.identify_nodes(N, mb).astype(np.int32)


@pytest.mark.parametrize("kind", ["SCL-LUT", "FastSCL-LUT", "SC-LUT"])
def test_device_decode_then_host_decode_without_sync(kind, qpd, oracle_mod):
    """decode_batch(torch, side stream) immediately followed by decode(numpy)
    and decode_batch(numpy) on the same decoder, no synchronization between."""
    import torch

    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 1024, 512, 8
    fm, nt = _code(N, K)
    p = LU.random_luts(N, 16, seed=31, distinct_mags=3)
    rng = np.random.default_rng(32)
    big = rng.integers(0, 16, size=(1 << 15, N), dtype=np.int32)  # ~1-3 ms of decode on the side stream
    small = rng.integers(0, 16, size=(12, N), dtype=np.int32)
    dec = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt)
    x = torch.from_numpy(big).cuda()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        dev = dec.decode_batch(x)  # asynchronous on `side`
    one = dec.decode(small[0])  # host path on the decoder's own stream, right away
    many = dec.decode_batch(small)
    side.synchronize()
    want = oracle_mod.decode_lut(kind, p, K, L, fm, small, node_type=nt)
    assert_frames_equal(one[None], want[:1], dec, f"stream-one-{kind}")
    assert_frames_equal(many, want, dec, f"stream-many-{kind}")
    ref = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt).decode_batch(big)  # a fresh decoder, synchronous
    assert_frames_equal(dev.cpu().numpy(), ref, dec, f"stream-big-{kind}")
    sample = np.arange(0, len(big), len(big) // 16)
    assert_frames_equal(ref[sample], oracle_mod.decode_lut(kind, p, K, L, fm, big[sample], node_type=nt), None,
                        f"stream-big-oracle-{kind}")


def test_two_streams_alternate_on_one_decoder(qpd):
    """Launches alternating between two streams with no host synchronization:
    each waits for the previous one (they share the slab and the queue)."""
    import torch

    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 512, 256, 8
    fm, nt = _code(N, K)
    p = LU.random_luts(N, 16, seed=41, distinct_mags=3)
    rng = np.random.default_rng(42)
    batches = [rng.integers(0, 16, size=(b, N), dtype=np.int32) for b in (20000, 7, 9000, 1, 15000, 333)]
    for kind in ("SCL-LUT", "FastSCL-LUT"):
        dec = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        xs = [torch.from_numpy(b).cuda() for b in batches]
        torch.cuda.synchronize()
        outs = []
        for i, x in enumerate(xs):
            with torch.cuda.stream(streams[i % 2]):
                outs.append(dec.decode_batch(x))
        torch.cuda.synchronize()
        fresh = qpd.from_packed(kind, p, K, fm, L=L, node_type=nt)
        for i, (b, o) in enumerate(zip(batches, outs)):
            assert_frames_equal(o.cpu().numpy(), fresh.decode_batch(b), dec, f"alternate-{kind}-{i}")


@pytest.mark.parametrize("engine", ["auto", "generic"])
def test_task_queue_counter_wraps(engine, qpd, monkeypatch):
    """The queue counter is never reset: launch bases advance by each launch's
    task count.  Started 40 below 2^32 it wraps during the second launch; a
    small grid (max_waves) makes every launch take most tasks from the queue."""
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 256, 128, 8
    fm, nt = _code(N, K)
    p = LU.random_luts(N, 16, seed=51, distinct_mags=3)
    rng = np.random.default_rng(52)
    batches = [rng.integers(0, 16, size=(b, N), dtype=np.int32) for b in (200, 333, 64, 1000, 1, 517)]
    ref = qpd.from_packed("FastSCL-LUT", p, K, fm, L=L, node_type=nt, engine=engine)
    want = [ref.decode_batch(b) for b in batches]
    monkeypatch.setenv("QPD_TASK_BASE0", str((1 << 32) - 40))
    for mw in (3, 0):
        dec = qpd.from_packed("FastSCL-LUT", p, K, fm, L=L, node_type=nt, engine=engine, max_waves=mw)
        for i, b in enumerate(batches):
            assert_frames_equal(dec.decode_batch(b), want[i], dec, f"wrap-{engine}-mw{mw}-{i}")


def test_host_threads_share_one_decoder(qpd, oracle_mod):
    """Host threads calling one decoder at once (ctypes releases the GIL):
    the handle's lock serializes them; every result is the oracle's."""
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K, L = 256, 128, 8
    fm, nt = _code(N, K)
    p = LU.random_luts(N, 16, seed=61, distinct_mags=3)
    rng = np.random.default_rng(62)
    inputs = [rng.integers(0, 16, size=(40 + 9 * t, N), dtype=np.int32) for t in range(4)]
    want = [oracle_mod.decode_lut("SCL-LUT", p, K, L, fm, x, node_type=nt) for x in inputs]
    dec = qpd.from_packed("SCL-LUT", p, K, fm, L=L, node_type=nt)
    errors = []

    def work(t):
        try:
            for _ in range(6):
                got = dec.decode_batch(inputs[t])
                if not np.array_equal(got, want[t]):
                    errors.append((t, int((got != want[t]).any(1).sum())))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def test_input_error_check_waits_for_device_work(qpd):
    """qpd_check_input_error waits for the decoder's own last launch (a torch
    stream) rather than the whole device, and clears the flag."""
    import torch

    from quantized_decoder_polar_codes_amd import _lib
    from quantized_decoder_polar_codes_amd import lut as LU

    N, K = 256, 128
    fm, nt = _code(N, K)
    dec = qpd.from_packed("SCL-LUT", LU.minsum_uniform_luts(N), K, fm, L=4)
    x = torch.randint(0, 16, (20000, N), dtype=torch.int32, device="cuda")
    x[19999, 5] = 99  # the last frame: seen only when the whole launch ran
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        dec.decode_batch(x)
    with pytest.raises(ValueError, match="outside"):
        _lib.check(_lib.load().qpd_check_input_error(dec._h))
    _lib.check(_lib.load().qpd_check_input_error(dec._h))  # cleared
