"""Monte-Carlo harness: the reference driver's counting/stop rule, frame
sharding across ranks (gloo, world_size 2, on CPU) and -- on the GPU -- the
frame generator keyed by global frame id."""
import os
import socket

import numpy as np
import pytest

from quantized_decoder_polar_codes_amd import montecarlo as MC


def driver_loop(errors, K, A, max_blocks, stop):
    """Literal restatement of mainQuantizedDecoder_LLRDomain.py:147-202 over a
    precomputed sequence of per-frame bit-error counts."""
    nbit = nblk = nblocks = 0
    for f in range(max_blocks):
        nbit += int(errors[f])
        nblk += int(errors[f] > 0)
        if nblk > stop:
            return nbit / (A * nblocks), nblk / nblocks, nbit, nblk, nblocks, True
        nblocks += 1
        if nblocks == max_blocks:
            return nbit / (K * nblocks), nblk / nblocks, nbit, nblk, nblocks, False
    raise AssertionError


K = 24


def synthetic_source(frame0, B):
    """Deterministic per-frame 'decoder errors': msg zeros, bits = hashed error pattern."""
    gid = np.arange(frame0, frame0 + B, dtype=np.uint64)
    h = (gid * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)
    nerr = np.where(h % np.uint64(7) == 0, (h % np.uint64(5)) + np.uint64(1), 0).astype(np.int64)
    bits = np.zeros((B, K), dtype=np.uint8)
    for i, k in enumerate(nerr):
        bits[i, :k] = 1
    return np.zeros((B, K), dtype=np.uint8), bits


def errors_of(n):
    msg, bits = synthetic_source(0, n)
    return (bits != msg).sum(1)


@pytest.mark.parametrize("batch,max_blocks,stop", [(7, 500, 20), (64, 500, 20), (1000, 500, 20), (13, 300, 10 ** 6),
                                                   (5, 50, 1), (1, 2, 10)])
def test_run_point_matches_driver_loop(batch, max_blocks, stop):
    want = driver_loop(errors_of(max_blocks), K, K, max_blocks, stop)
    got = MC.run_point(synthetic_source, lambda s: s, K, 1.0, batch, max_blocks, stop)
    assert (got.ber, got.bler, got.bit_errors, got.block_errors, got.blocks, got.stopped_early) == want


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, batch, max_blocks, stop, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = MC.run_point(synthetic_source, lambda s: s, K, 1.0, batch, max_blocks, stop, group=dist.group.WORLD)
        q.put((rank, (r.ber, r.bler, r.bit_errors, r.block_errors, r.blocks, r.stopped_early)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 16), (2, 100), (3, 9)])
def test_distributed_shards_give_identical_counts(world, batch):
    """world_size > 1 over gloo: every rank reports exactly the single-process
    result (the RCCL path of bench.py/simulate() uses the same code)."""
    import torch.multiprocessing as mp

    max_blocks, stop = 600, 25
    want = driver_loop(errors_of(max_blocks), K, K, max_blocks, stop)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, max_blocks, stop, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r] == want


@pytest.mark.parametrize("world,batch,max_blocks", [(8, 16, 1000), (8, 100, 1000), (3, 7, 250), (8, 1, 20)])
def test_shard_counters_sum_to_one_shot(world, batch, max_blocks):
    """No early stop (config C5's MaxBlock branch): the `world` ranks' shards
    run one after the other (shard=(rank, world)) sum to the one-shot counters,
    as the end-of-point all-reduce does, and cover every frame once."""
    want = driver_loop(errors_of(max_blocks), K, K, max_blocks, 10 ** 9)
    parts = [MC.run_point(synthetic_source, lambda s: s, K, 1.0, batch, max_blocks, None, shard=(r, world))
             for r in range(world)]
    assert sum(p.bit_errors for p in parts) == want[2]
    assert sum(p.block_errors for p in parts) == want[3]
    assert sum(p.frames_decoded for p in parts) == max_blocks
    for p in parts:  # each shard's rates are over its own frames
        assert p.blocks == p.frames_decoded
        assert p.bler == (p.block_errors / p.blocks if p.blocks else 0.0)
        assert p.ber == (p.bit_errors / (K * p.blocks) if p.blocks else 0.0)


@pytest.mark.parametrize("world,batch,max_blocks,stop", [(8, 16, 2000, 40), (8, 5, 600, 25), (3, 9, 600, 25),
                                                         (8, 64, 300, 10 ** 6)])
def test_virtual_world_matches_driver_loop(world, batch, max_blocks, stop):
    """The ranks' slices of every step in lock step (virtual_world): the
    driver's counters and stop block, wherever the crossing frame falls."""
    want = driver_loop(errors_of(max_blocks), K, K, max_blocks, stop)
    got = MC.run_point(synthetic_source, lambda s: s, K, 1.0, batch, max_blocks, stop, virtual_world=world)
    assert (got.ber, got.bler, got.bit_errors, got.block_errors, got.blocks, got.stopped_early) == want


def test_virtual_world_crossing_outside_rank0():
    """A case whose stop crossing lies in a slice other than rank 0's."""
    world, batch, max_blocks, stop = 8, 16, 2000, 40
    want = driver_loop(errors_of(max_blocks), K, K, max_blocks, stop)
    assert want[5] and (want[4] % (world * batch)) // batch != 0  # the crossing block's rank
    got = MC.run_point(synthetic_source, lambda s: s, K, 1.0, batch, max_blocks, stop, virtual_world=world)
    assert got.blocks == want[4]


def test_mc_ref_philox_known_answer():
    """Philox4x32-10 known-answer vector (Random123 kat_vectors: counter=0, key=0)."""
    from mc_ref import philox

    r = philox(0, 0, 0, 0, 0, 0)
    assert [int(x) for x in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    m = 0xFFFFFFFF
    r = philox(m, m, m, m, m, m)
    assert [int(x) for x in r] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


# ---------------------------------------------------------------------------
# GPU: frame generator and end-to-end simulation
# ---------------------------------------------------------------------------

@pytest.mark.gpu
def test_gpu_frames_match_restatement_and_are_shard_invariant(native_lib):
    import torch

    import quantized_decoder_polar_codes_amd as Q
    from mc_ref import frames as ref_frames
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, Kc = 256, 128
    _, mb, fm, mm = C.construct_pw(N, Kc)
    dec = Q.from_packed("SC-LUT", LU.minsum_uniform_luts(N), Kc, fm)
    edges, lut = MC.uniform_channel_quantizer(16, 0.5)
    sigma = MC.sigma_for(2.0, Kc / N)
    src = MC.GpuFrames(dec, edges, lut, 16, sigma, seed=99)
    msg, sym = src(1000, 300)
    msg2, sym2 = src(1100, 50)  # a sub-range generated separately
    torch.cuda.synchronize()
    assert torch.equal(msg[100:150], msg2) and torch.equal(sym[100:150], sym2)
    rmsg, rsym, _ = ref_frames(N, Kc, mb, 99, 1000, 300, sigma, edges, lut, 16)
    assert (msg.cpu().numpy() == rmsg).all()  # integer path: exact
    # float64 noise: the device log/sin/cos may differ from glibc's in the last
    # ulp, which moves a symbol only if its LLR lies within ~1e-16 of an edge
    assert (sym.cpu().numpy() == rsym).all()


@pytest.mark.gpu
def test_gpu_simulate_batch_invariant_and_sane(native_lib):
    import quantized_decoder_polar_codes_amd as Q
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, Kc, L = 128, 64, 8
    _, mb, fm, mm = C.construct_pw(N, Kc)
    dec = Q.from_packed("SCL-LUT", LU.minsum_uniform_luts(N), Kc, fm, L=L)
    a = MC.simulate(dec, Kc, [1.0, 3.0, 5.0], batch=3000, max_blocks=20000, stop_blkerrs=200)
    b = MC.simulate(dec, Kc, [1.0, 3.0, 5.0], batch=777, max_blocks=20000, stop_blkerrs=200)
    for x, y in zip(a, b):
        assert (x.bit_errors, x.block_errors, x.blocks) == (y.bit_errors, y.block_errors, y.blocks)
    assert a[0].bler > a[1].bler > a[2].bler
    assert a[2].ber < 1e-2


@pytest.mark.gpu
def test_gpu_frames_with_crc_and_ca_simulation(native_lib):
    """CRC-aided decoders: the generator appends the CRC (bit-exact vs the
    restatement), noiseless frames decode to their messages, and a short
    simulation behaves."""
    import torch

    import oracle
    import quantized_decoder_polar_codes_amd as Q
    from mc_ref import frames as ref_frames
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU

    N, A, L = 256, 100, 8
    K = A + 24
    _, mb, fm, mm = C.construct_pw(N, K)
    dec = Q.from_packed("CA-SCL-LUT", LU.minsum_uniform_luts(N), K, fm, L=L, A=A)
    edges, lut = MC.uniform_channel_quantizer(16, 0.5)
    sigma = MC.sigma_for(2.0, A / N)
    src = MC.GpuFrames(dec, edges, lut, 16, sigma, seed=7)
    msg, sym = src(0, 200)
    torch.cuda.synchronize()
    assert msg.shape == (200, A)
    rmsg, rsym, _ = ref_frames(N, K, mb, 7, 0, 200, sigma, edges, lut, 16, A=A, crc=(24, oracle.CRC24_LOC))
    assert (msg.cpu().numpy() == rmsg).all()
    assert (sym.cpu().numpy() == rsym).all()
    quiet = MC.GpuFrames(dec, edges, lut, 16, 1e-3, seed=8)
    m2, s2 = quiet(0, 500)
    assert torch.equal(dec.decode_batch(s2), m2)
    res = MC.simulate(dec, A, [1.0, 4.0], batch=2000, max_blocks=10000, stop_blkerrs=300)
    assert res[0].bler > res[1].bler



@pytest.mark.gpu
@pytest.mark.parametrize("N,K,A,frame0,md", [(8, 4, None, 0, False), (16, 9, None, 5, False), (64, 40, 27, 3, False),
                                             (1024, 512, None, (1 << 33) + 17, True), (2048, 1000, 983, 11, True),
                                             (512, 300, 276, 0, True)])
def test_gpu_frames_bit_exact_vs_restatement(native_lib, N, K, A, frame0, md):
    """Every generator path bit-exact against the numpy restatement: N below one
    word and beyond 64 words, message lengths off the byte grid, CRC-aided
    messages, frame ids above 2^32 and the MinDistortion channel quantizer
    (non-uniform edges)."""
    import torch

    import oracle
    import quantized_decoder_polar_codes_amd as Q
    from mc_ref import frames as ref_frames
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lut as LU
    from quantized_decoder_polar_codes_amd import lutgen as LG

    _, mb, fm, mm = C.construct_pw(N, K) if N <= 1024 else (None, *_pw_big(N, K))
    kind = "CA-SCL-LUT" if A is not None else "SC-LUT"
    kw = {"L": 2, "A": A} if A is not None else {}
    dec = Q.from_packed(kind, LU.minsum_uniform_luts(N), K, fm, **kw)
    sigma = MC.sigma_for(1.5, (A or K) / N)
    if md:
        _, _, edges, lut = LG.channel_quantizer(sigma, 128, 16)
    else:
        edges, lut = MC.uniform_channel_quantizer(16, 0.5)
    src = MC.GpuFrames(dec, edges, lut, 16, sigma, seed=424242)
    B = 96
    msg, sym = src(frame0, B)
    torch.cuda.synchronize()
    crc = (24, oracle.CRC24_LOC) if A is not None else None
    rmsg, rsym, _ = ref_frames(N, K, mb, 424242, frame0, B, sigma, edges, lut, 16, A=A, crc=crc)
    assert (msg.cpu().numpy() == rmsg).all()
    assert (sym.cpu().numpy() == rsym).all()


def _pw_big(N, K):
    """A frozen set for N > 1024 (beyond the 5G sequence): the K largest-weight
    positions as information bits (any mask exercises the generator)."""
    w = np.array([bin(i).count("1") for i in range(N)])
    order = np.lexsort((np.arange(N), w))
    mb = np.sort(order[N - K:])
    fm = np.ones(N, dtype=np.int64)
    fm[mb] = 0
    return mb, fm, 1 - fm


@pytest.mark.gpu
@pytest.mark.parametrize("kind,N,K,L,engine", [("SCL-LUT", 1024, 512, 8, "auto"), ("FastSCL-LUT", 1024, 512, 8, "auto"),
                                               ("SC-LUT", 128, 32, 1, "auto"), ("CA-SCL-LUT", 256, 124, 8, "auto"),
                                               ("SCL-LUT", 256, 128, 4, "generic"),
                                               # output rows off the dword grid: the tail's byte path counts
                                               ("SC-LUT", 128, 33, 1, "auto"), ("CA-SCL-LUT", 256, 126, 8, "auto")])
def test_gpu_fused_generate_decode_equals_unfused(kind, N, K, L, engine, native_lib):
    """qpd_mc_decode (generation writes the decoder's root pre-pass rows on a
    fast-engine decoder, else its own symbol buffer) = qpd_mc_frames followed
    by decode_batch, bit for bit, and so are the Monte-Carlo counters of a
    fixed-seed point (the driver's stop rule and MaxBlock branch)."""
    import torch

    import quantized_decoder_polar_codes_amd as Q
    from quantized_decoder_polar_codes_amd import codes as C
    from quantized_decoder_polar_codes_amd import lutgen as LG

    _, mb, fm, mm = C.construct_pw(N, K)
    nt = C.identify_nodes(N, mb).astype(np.int32)
    d = LG.design(N, 16, 3.0)
    kw = {"A": K - 24} if kind.startswith("CA-") else {}
    dec = Q.from_packed(kind, d.packed(), K, fm, L=L, node_type=nt, engine=engine, **kw)
    sigma = MC.sigma_for(2.0, K / N)
    _, _, edges, clut = LG.channel_quantizer(sigma, 128, 16)
    src = MC.GpuFrames(dec, edges, clut, 16, sigma, seed=4321)
    msg_a, sym = src(5000, 3001)
    bits_a = dec.decode_batch(sym)
    msg_b, bits_b = src.decode_frames(5000, 3001)
    torch.cuda.synchronize()
    assert torch.equal(msg_a, msg_b)
    assert torch.equal(bits_a, bits_b)
    for stop in (None, 50):
        a = MC.run_point(src, dec.decode_batch, dec.K, 2.0, 1000, 7000, stop, A=dec.out_bits, count_device=src.device)
        b = MC.run_point(src, dec.decode_batch, dec.K, 2.0, 1000, 7000, stop, A=dec.out_bits, count_device=src.device,
                         gen_decode=src.decode_frames)
        assert (a.bit_errors, a.block_errors, a.blocks, a.stopped_early) == \
            (b.bit_errors, b.block_errors, b.blocks, b.stopped_early)
