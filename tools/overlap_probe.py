"""Probe: does splitting the bench batch over concurrent streams (one decoder
handle per stream: its own pre-pass rows, prefix records, slab and task queue)
hide the pre-pass / prefix kernels and the decode kernel's drain?

Times, best of 3 (HIP events on the current stream, joined across streams):
  one   -- one decoder, the whole batch (the bench's call)
  seqK  -- one decoder, K slices one after the other on one stream
  parK  -- K decoders, slice k on stream k (launched back to back)
and checks that the concatenated outputs equal the one-call output.
usage: python tools/overlap_probe.py [frames_log2=21] [K ...]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import quantized_decoder_polar_codes_amd as Q  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 21
Ks = [int(k) for k in sys.argv[2:]] or [2, 4]
kind = os.environ.get("PROBE_KIND", "SCL-LUT")
F = 1 << lg
wl = bench.workload(1024, 512, 8, kind, F, 2.0)
sym = wl.sym
decs = [wl.dec] + [Q.from_packed(kind, wl.packed, 512, wl.fm, L=8, node_type=wl.nt) for _ in range(max(Ks) - 1)]
streams = [torch.cuda.Stream() for _ in range(max(Ks))]
ref = wl.dec.decode_batch(sym)
torch.cuda.synchronize()
dig = lambda t: hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()[:12]  # noqa: E731


def timed(fn):
    best, out = 1e9, None
    for _ in range(4):
        cur = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        out = fn(cur)
        e1.record(cur)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best, out


def one(cur):
    return wl.dec.decode_batch(sym)


def seq(K):
    def f(cur):
        h = F // K
        return torch.cat([wl.dec.decode_batch(sym[k * h:(k + 1) * h]) for k in range(K)])
    return f


def par(K):
    def f(cur):
        h = F // K
        outs = []
        for k in range(K):
            s = streams[k]
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                o = decs[k].decode_batch(sym[k * h:(k + 1) * h])
                o.record_stream(cur)
                outs.append(o)
        for k in range(K):
            cur.wait_stream(streams[k])
        return torch.cat(outs)
    return f


cases = [("one", one)] + [(f"seq{K}", seq(K)) for K in Ks] + [(f"par{K}", par(K)) for K in Ks]
for name, fn in cases:
    ms, out = timed(fn)
    ok = "same" if torch.equal(out, ref) else "DIFFERENT " + dig(out)
    print(f"{kind:12s} 2^{lg} {name:6s} {ms:8.3f} ms {F / ms / 1e3:8.3f} Mframes/s  output {ok}", flush=True)
