"""HIP-graph synthesis for small batches (serving latency; reference ``synthesize.py:128-150`` single mode, the
batch-1 path of ``notebooks/control.ipynb:778``).

A batch-1 text -> wav synthesis is ~350 kernel launches driven from Python: ~3 ms of host time against well under
1 ms of GPU work, so the latency is the host's.  Here the packed synthesis path (``FastSpeech2.infer_front`` /
``infer_back`` + ``Generator.infer_packed``) is captured in two HIP graphs and replayed:

  * graph 1, per input shape (B, text length, reference-mel length): style encoder, encoder, variance adaptor,
    duration rounding -> the mel lengths (device);
  * the one host sync of any FastSpeech2 synthesis: the B mel lengths come back to the host;
  * graph 2, per (graph-1 key, mel lengths): packed length regulator + decoder, mel_linear, PostNet and the
    packed HiFi-GAN down to the int16 waveform.

Every replay recomputes the whole text -> wav path from its inputs (copied into the graph's static input
tensors first); only launch overhead is removed.  A key is captured after ``warm`` eager runs on it (allocations,
workspaces, the vocoder's length tables settle); shapes seen for the first time run eagerly.  Captured graphs keep
their memory (pool), the vocoder tables they read (referenced by the entry) and every kernel workspace they
captured (``hip._GRAPHS_LIVE``: grown workspaces are retired, never freed).
"""
from __future__ import annotations

import collections
import time

import torch


def _multi_copy(pairs) -> bool:
    from ..ops import hip

    return hip.multi_copy(pairs)


class SynthGraphs:
    def __init__(self, model, vocoder, int16_scale=None, warm: int = 1, max_batch: int = 8, max_graphs: int = 64):
        self.model, self.voc = model, vocoder
        self.scale = int16_scale
        self.warm, self.max_batch, self.max_graphs = int(warm), int(max_batch), int(max_graphs)
        self.g1 = collections.OrderedDict()
        self.g2 = collections.OrderedDict()
        self.pool = None
        self.stream = None  # warm-up AND capture run on this one stream: the stream-keyed workspaces of the kernel
        #                     library (split-K partials) are allocated by the warm-up, never inside a capture
        self.stats = {"captures": 0, "replays": 0, "eager": 0, "capture_s": 0.0}

    def supported(self, texts) -> bool:
        return (texts.is_cuda and texts.shape[0] <= self.max_batch and self.model.packed_inference_ok(texts)
                and self.voc.packable())

    # ------------------------------------------------------------------ eager halves
    def _front(self, inp):
        return self.model.infer_front(*inp)

    def _back(self, front, lens):
        rows = self.model.infer_back(front, lens)
        return self.voc.infer_packed(rows, lens, int16_scale=self.scale)

    # ------------------------------------------------------------------ capture helpers
    def _capture(self, fn):
        from ..ops import hip

        hip.graphs_live()  # grown workspaces are retired from now on (graphs hold their addresses)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool, stream=self.stream):
            out = fn()
        torch.cuda.synchronize()
        self.stats["captures"] += 1
        self.stats["capture_s"] += time.perf_counter() - t0
        return g, out

    def _evict(self, table):
        while len(table) > self.max_graphs:
            table.popitem(last=False)

    # ------------------------------------------------------------------ synthesis
    @torch.no_grad()
    def __call__(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None, max_mel_len=None):
        """-> (wav [B, max(lens) * hop] (int16 when int16_scale), host mel lengths).  The wav is a fresh tensor,
        ordered on the caller's stream."""
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=texts.device)
        cur = torch.cuda.current_stream(texts.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            wav, lens = self._run(speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len)
        cur.wait_stream(self.stream)
        wav.record_stream(cur)
        return wav, lens

    def _run(self, speakers, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len):
        inp = (speakers, texts, src_lens, int(max_src_len), mels, mel_lens,
               None if max_mel_len is None else int(max_mel_len))
        if not self.supported(texts):
            self.stats["eager"] += 1
            front = self._front(inp)
            lens = [int(v) for v in front[2].cpu().tolist()]
            return self._back(front, lens), lens
        k1 = (tuple(texts.shape), None if mels is None else tuple(mels.shape), inp[3], inp[6], str(texts.device))
        e1 = self.g1.get(k1)
        if e1 is None:
            e1 = self.g1[k1] = {"seen": 0, "graph": None}
            self._evict(self.g1)
        else:
            self.g1.move_to_end(k1)
        if e1["graph"] is None:
            if e1["seen"] < self.warm:
                e1["seen"] += 1
                self.stats["eager"] += 1
                front = self._front(inp)
                lens = [int(v) for v in front[2].cpu().tolist()]
                return self._back(front, lens), lens
            static = tuple(t.clone() if isinstance(t, torch.Tensor) else t for t in inp)
            e1["static"] = static
            e1["graph"], e1["out"] = self._capture(lambda: self._front(static))
        pairs = [(dst, src) for dst, src in zip(e1["static"], inp) if isinstance(dst, torch.Tensor)]
        if not _multi_copy(pairs):  # one launch for all inputs when they are device tensors
            for dst, src in pairs:
                dst.copy_(src, non_blocking=True)
        e1["graph"].replay()
        self.stats["replays"] += 1
        lens = [int(v) for v in e1["out"][2].cpu().tolist()]  # the one host sync
        # graph 2 reads THIS graph-1 entry's static outputs: keyed by the entry object (held by the graph-2 entry,
        # so its id stays unique while the entry lives), not by the shape key
        k2 = (id(e1), tuple(lens))
        e2 = self.g2.get(k2)
        if e2 is None:
            e2 = self.g2[k2] = {"seen": 0, "graph": None, "front": e1}
            self._evict(self.g2)
        else:
            self.g2.move_to_end(k2)
        if e2["graph"] is None:
            if e2["seen"] < self.warm:
                e2["seen"] += 1
                self.stats["eager"] += 1
                return self._back(e1["out"], lens).clone(), lens
            e2["graph"], e2["out"] = self._capture(lambda: self._back(e1["out"], lens))
        e2["graph"].replay()
        self.stats["replays"] += 1
        return e2["out"].clone(), lens
