"""Chunked, stream-overlapped QSGD-MaxNorm all-reduce.

One bucket is cut into C contiguous chunks.  The max-norm is global over the
whole bucket, so it is still computed once (absmax -> all_reduce MAX).  Then,
per chunk:
    encode(c)       on the compute stream                (HIP)
    all_reduce(c)   on RCCL's stream, after encode(c)    (int32 SUM of packed lanes)
    decode(c)       on a decode stream, after all_reduce(c)
so encode(c+1) runs while chunk c is on the wire and chunk c-1 decodes.

Stream dependencies (nothing waits on a whole stream inside a call):
    decode stream  <- event after the norm is final (absmax + MAX)
    decode(c)      <- the RCCL work handle of chunk c (W > 1), or an event
                      recorded right after encode(c) (W = 1)
    compute stream <- the decode stream, once, at the end of the call (the next
                      call's encode(c) must not overwrite chunk c's words
                      before this call's decode(c) has read them)
With the generator in torch mode the packed integers equal the unchunked
encode's (draws are consumed chunk by chunk, in element order).

The reference has no counterpart (it all-reduces one monolithic int8/int32
vector after the whole compress, reducer.py:528-533).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import codec as _hip_codec
from .rng import default_generator


class ChunkedQSGDAllReduce:
    """reduce(x) = decode(SUM over ranks of encode(x)) * 1/W, chunk-pipelined.

    world: the W the lanes are sized for; defaults to the group's size.
    collective: run the MAX / SUM collectives (default: world > 1).  False
    keeps the W-sized lanes without them (timing a rank's kernels on one GPU;
    the decoded floats then assume a SUM that did not happen).
    """

    def __init__(self, n: int, bits: int, device, chunks: int = 4, group=None, generator=None, codec=None,
                 world: int | None = None, collective: bool | None = None):
        self.n, self.bits, self.device = n, bits, torch.device(device)
        self.group = group
        if world is None:
            world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.world = int(world)
        self.collective = self.world > 1 if collective is None else bool(collective)
        self.codec = codec or _hip_codec
        self.gen = generator or default_generator
        chunks = max(1, min(chunks, n))
        step = -(-n // chunks)
        step = (step + 3) // 4 * 4  # chunk starts stay 16-byte aligned
        self.bounds = [(s, min(s + step, n)) for s in range(0, n, step)]
        self.lanes = [self.codec.qsgd_layout(e - s, bits, self.world) for s, e in self.bounds]
        self.words = [torch.empty(ln.plane_words, dtype=torch.int32, device=self.device) for ln in self.lanes]
        self.norm = torch.empty(1, dtype=torch.float32, device=self.device)
        self.dec_stream = torch.cuda.Stream(self.device)

    def bits_per_step(self) -> int:
        return 32 + sum(32 * w.numel() for w in self.words)

    def _max(self, norm: torch.Tensor):
        """MAX of the local norms (enqueued in line: every encode needs it)."""
        if self.collective:
            dist.all_reduce(norm, op=dist.ReduceOp.MAX, group=self.group)

    def _reduce(self, words: torch.Tensor):
        """Asynchronous SUM of one chunk's packed words; the work handle, or
        None when the words are final on the compute stream."""
        if self.collective:
            return dist.all_reduce(words, group=self.group, async_op=True)
        return None

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None, _trace: dict | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty_like(x)
        W = self.world
        compute = torch.cuda.current_stream(self.device)

        def mark(key, stream):  # timing events of trace(); nothing when not tracing
            if _trace is not None:
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                _trace.setdefault(key, []).append(e)

        mark("start", compute)
        self.codec.absmax(x, out=self.norm)
        self._max(self.norm)
        norm_ready = torch.cuda.Event()
        norm_ready.record(compute)
        self.dec_stream.wait_event(norm_ready)
        for (s, e), ln, wd in zip(self.bounds, self.lanes, self.words):
            rng = self.gen.reserve(e - s, 1, device=self.device, backend=self.codec)
            mark("encode_start", compute)
            self.codec.qsgd_encode(x[s:e], self.norm, self.bits, rng, W, out=wd, lanes=ln)
            mark("encode_end", compute)
            work = self._reduce(wd)
            if work is None:
                encoded = torch.cuda.Event()
                encoded.record(compute)
            if _trace is not None:  # a probe stream that waits for this chunk's SUM only
                with torch.cuda.stream(_trace["probe"]):
                    if work is not None:
                        work.wait()
                    else:
                        _trace["probe"].wait_event(encoded)
                    mark("sum_end", _trace["probe"])
            with torch.cuda.stream(self.dec_stream):
                if work is not None:
                    work.wait()  # the decode stream waits for this chunk's RCCL SUM; the host does not block
                else:
                    self.dec_stream.wait_event(encoded)
                mark("decode_start", self.dec_stream)
                self.codec.qsgd_decode(wd, e - s, self.norm, self.bits, W, 1.0 / W, out=out[s:e], lanes=ln)
                mark("decode_end", self.dec_stream)
        compute.wait_stream(self.dec_stream)
        for t in [x, out, self.norm, *self.words]:
            t.record_stream(self.dec_stream)
        return out

    def trace(self, x: torch.Tensor, out: torch.Tensor | None = None) -> dict:
        """One call with HIP timing events on every stream it uses: per chunk
        the end of its encode, of its SUM (seen from a probe stream that waits
        for that chunk's collective only), and the start / end of its decode,
        in ms from the call's start.  `decode_overlaps_next_sum`: decode(c)
        started before SUM(c+1) ended, for every c; `encode_overlaps_previous_sum`:
        encode(c+1) ran while SUM(c) was in flight, for every c (the overlap that
        matters when the SUM is the long pole)."""
        torch.cuda.synchronize(self.device)
        tr = {"probe": torch.cuda.Stream(self.device)}
        self(x, out, _trace=tr)
        torch.cuda.synchronize(self.device)
        t0 = tr["start"][0]
        ms = {k: [t0.elapsed_time(e) for e in tr[k]]
              for k in ("encode_start", "encode_end", "sum_end", "decode_start", "decode_end")}
        C = len(self.bounds)
        started = [ms["decode_start"][c] < ms["sum_end"][c + 1] for c in range(C - 1)]
        ended = [ms["decode_end"][c] < ms["sum_end"][c + 1] for c in range(C - 1)]
        # encode(c+1) against SUM(c): the SUMs run in order on one communicator, so
        # SUM(c) starts no earlier than max(encode_end(c), sum_end(c-1)); the overlap
        # is that interval's intersection with encode(c+1)'s
        ov = []
        for c in range(C - 1):
            s0 = max(ms["encode_end"][c], ms["sum_end"][c - 1] if c else 0.0)
            ov.append(max(0.0, min(ms["encode_end"][c + 1], ms["sum_end"][c]) - max(ms["encode_start"][c + 1], s0)))
        return {"chunks": C, "ms": ms, "decode_overlaps_next_sum": bool(started) and all(started),
                "decode_c_started_before_sum_c1_ended": started, "decode_c_ended_before_sum_c1_ended": ended,
                "encode_c1_overlap_sum_c_ms": ov,
                "encode_overlaps_previous_sum": bool(ov) and all(v > 0 for v in ov)}
