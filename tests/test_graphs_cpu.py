"""Shape bucketing of the HIP-graph training steps (train/graphs.py), on CPU tensors."""
import torch

from speakingstyle_amd.train.graphs import GraphedSteps


class _Tr:
    max_seq_len = 1000


def test_pad_batch_buckets_and_keeps_lengths():
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    b = SyntheticBatches(4, device="cpu", seed=3, phone_counts=[17, 33, 9, 21]).make_batch()
    gs = GraphedSteps(_Tr(), t_quant=16, m_quant=32)
    pb, key = gs.pad_batch(b)
    T, M = b[5], b[8]
    assert key == (4, (T + 15) // 16 * 16, (M + 31) // 32 * 32, False)
    assert pb[3].shape == (4, key[1]) and pb[11].shape == (4, key[1]) and pb[9].shape == (4, key[1])
    assert pb[6].shape == (4, key[2], 80) and pb[5] == key[1] and pb[8] == key[2]
    assert torch.equal(pb[3][:, :T], b[3]) and not pb[3][:, T:].any()
    assert torch.equal(pb[6][:, :M], b[6]) and not pb[6][:, M:].any()
    assert torch.equal(pb[4], b[4]) and torch.equal(pb[7], b[7])
    assert getattr(pb[7], "host_lengths", None) is None  # the padded (unpacked) layout
    pb2, key2 = gs.pad_batch(pb)  # idempotent on an already bucketed batch
    assert key2 == key and pb2[3].shape == pb[3].shape
