"""CPU proof of the whole-ResBlock kernel's tiling (csrc/k_vocoder.hip ``resblock_fused_kernel``).

The kernel cuts a sequence into tiles of R0 = 16 * NB rows whose middle BM = R0 - 2 * HT rows are
output rows, HT = (K-1)/2 * (d0 + d1 + d2 + 3) being the summed halo of the six convs.  Inside a tile
every conv is evaluated on ALL rows of one absolute row frame: rows whose window leaves the conv's
valid region are don't-care values, and the margin rows around the tile are never written.  This
emulation runs exactly that schedule in fp32 with the margins filled with NaN: if any output row
depended on a don't-care row, NaN would reach it.  It must equal the plain ResBlock1 (reference
``hifigan/models.py:20-44``) on every sample, including tiles cut at the sequence ends, sequences
shorter than one tile and the zeroing of rows outside [0, T) before every conv.  The tile constants
mirror ``struct RF`` (a change there must be mirrored here)."""
import pytest
import torch
import torch.nn.functional as F

from speakingstyle_amd.models.hifigan import LRELU_SLOPE, ResBlock1

# (C, K) -> NB of struct RF (16-row blocks per tile)
RF_NB = {(32, 3): 16, (32, 7): 40, (32, 11): 40, (64, 3): 24, (64, 7): 24, (128, 3): 12}
RF_NB_EXTRA = {(64, 11): 24, (128, 7): 12}  # behind ssamd_resblock_set_whole_extra (measured slower, off)
RF_NB_SHORT = {(32, 3): 8, (32, 7): 16, (32, 11): 16, (64, 3): 12, (64, 7): 12, (128, 3): 8}  # RF<C, K, 1>
MAXD = 5


def _lrelu(v):
    return F.leaky_relu(v, LRELU_SLOPE)


def _conv_all_rows(buf, w, b, d, mg):
    """conv over every row of a tile buffer laid out [margin | R0 rows | margin] (margins NaN);
    output row r reads rows r - h + tap*d, h = d*(K-1)/2 -- the kernel's absolute-frame evaluation."""
    K = w.shape[2]
    h = d * (K - 1) // 2
    assert h <= mg, "margin must cover the widest half window"
    R0 = buf.shape[0] - 2 * mg
    src = buf[mg - h: mg + R0 + h].t().unsqueeze(0)  # [1, C, R0 + 2h]
    return F.conv1d(src, w, b, dilation=d).squeeze(0).t()  # [R0, C]


def emulate_whole_block(x, blk, NB):
    """x [T, C] fp32 -> the kernel's output rows, tile by tile."""
    T, C = x.shape
    K = blk.kernel_size
    H2 = (K - 1) // 2
    d = blk.dilation
    R0 = 16 * NB
    HT = H2 * (sum(d) + 3)
    BM = R0 - 2 * HT
    assert BM >= 16
    mg = MAXD * H2
    out = torch.full((T, C), float("nan"))
    nan = float("nan")
    for t0 in range(0, T, BM):
        tb = t0 - HT
        t = torch.arange(R0) + tb
        inside = ((t >= 0) & (t < T)).unsqueeze(1)
        rows = x.new_zeros(R0, C)
        src_lo, src_hi = max(tb, 0), min(tb + R0, T)
        if src_hi > src_lo:
            rows[src_lo - tb: src_hi - tb] = x[src_lo:src_hi]
        X = rows.clone()                      # residual stream (registers in the kernel)
        A = torch.full((R0 + 2 * mg, C), nan)  # lrelu(x_p) tile with NaN margins
        Tt = torch.full((R0 + 2 * mg, C), nan)
        A[mg:mg + R0] = torch.where(inside, _lrelu(X), torch.zeros(()))
        for p, (c1, c2) in enumerate(zip(blk.convs1, blk.convs2)):
            v = _conv_all_rows(A, c1.weight, c1.bias, d[p], mg)
            Tt[mg:mg + R0] = torch.where(inside, _lrelu(v), torch.zeros(()))
            v = _conv_all_rows(Tt, c2.weight, c2.bias, 1, mg)
            X = X + v
            A[mg:mg + R0] = torch.where(inside, _lrelu(X), torch.zeros(()))
        n = min(BM, T - t0)
        out[t0:t0 + n] = X[HT:HT + n]
    return out


def _block(C, K, seed=0):
    torch.manual_seed(seed)
    blk = ResBlock1(C, K, (1, 3, 5))
    for m in blk.modules():
        if isinstance(m, torch.nn.Conv1d):
            if hasattr(m, "weight_g"):
                torch.nn.utils.remove_weight_norm(m)
            m.weight.data.normal_(0, 1.0 / (C * K) ** 0.5)
            m.bias.data.normal_(0, 0.1)
    return blk.eval()


@pytest.mark.parametrize("C,K,short", [(C, K, s) for (C, K) in sorted(RF_NB) for s in (False, True)])
def test_whole_block_tiling_matches_resblock(C, K, short):
    blk = _block(C, K)
    NB = (RF_NB_SHORT if short else RF_NB)[(C, K)]
    HT = (K - 1) // 2 * (1 + 3 + 5 + 3)
    BM = 16 * NB - 2 * HT
    for T in (3, BM - 1, BM, 2 * BM + 7):
        x = torch.randn(T, C)
        with torch.no_grad():
            ref = blk(x.t().unsqueeze(0)).squeeze(0).t()
            got = emulate_whole_block(x, blk, NB)
        assert torch.isfinite(got).all(), f"a don't-care row reached an output (C={C}, K={K}, T={T})"
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_whole_block_halo_is_necessary():
    """One row less of halo (HT - 1) makes the tile-edge outputs read don't-care (NaN) rows."""
    C, K = 32, 7
    blk = _block(C, K, seed=1)
    NB = RF_NB[(C, K)]
    d = blk.dilation
    H2 = (K - 1) // 2
    HT = H2 * (sum(d) + 3) - 1
    R0 = 16 * NB
    # one interior tile (no sequence end inside it) by hand, output rows [HT, R0 - HT) with the short halo
    mg = MAXD * H2
    X = torch.randn(R0, C)
    A = torch.full((R0 + 2 * mg, C), float("nan"))
    Tt = torch.full((R0 + 2 * mg, C), float("nan"))
    A[mg:mg + R0] = _lrelu(X)
    with torch.no_grad():
        for p, (c1, c2) in enumerate(zip(blk.convs1, blk.convs2)):
            Tt[mg:mg + R0] = _lrelu(_conv_all_rows(A, c1.weight, c1.bias, d[p], mg))
            X = X + _conv_all_rows(Tt, c2.weight, c2.bias, 1, mg)
            A[mg:mg + R0] = _lrelu(X)
    edge = X[HT:R0 - HT]
    assert not torch.isfinite(edge[0]).all() and not torch.isfinite(edge[-1]).all()
    assert torch.isfinite(edge[1:-1]).all()


def _balanced(e):
    depth = 0
    for ch in e:
        depth += ch == "("
        depth -= ch == ")"
        if depth < 0:
            return False
    return depth == 0


def test_tile_constants_mirror_the_kernel():
    """RF_NB above is the NB table of ``struct RF``; the fused geometries are those of
    ``ssamd_resblock_fusable``."""
    import os
    import re

    src = open(os.path.join(os.path.dirname(__file__), "..", "csrc", "k_vocoder.hip")).read()
    m = re.search(r"static constexpr int NB = (.+?);", src[src.index("struct RF {"):], re.S)
    expr = " ".join(m.group(1).split())

    def ev(e, C, K):  # right-associative C ternary chain -> value
        e = e.strip()
        while e.startswith("(") and e.endswith(")") and _balanced(e[1:-1]):
            e = e[1:-1].strip()
        depth, q = 0, -1
        for i, ch in enumerate(e):
            depth += ch == "("
            depth -= ch == ")"
            if ch == "?" and depth == 0:
                q = i
                break
        if q < 0:
            return eval(e.replace("&&", " and ").replace("||", " or "), {"C": C, "K": K, "S": S})
        depth, nest = 0, 0
        for i in range(q + 1, len(e)):
            ch = e[i]
            depth += ch == "("
            depth -= ch == ")"
            if depth == 0 and ch == "?":
                nest += 1
            elif depth == 0 and ch == ":":
                if nest == 0:
                    return ev(e[q + 1:i], C, K) if ev(e[:q], C, K) else ev(e[i + 1:], C, K)
                nest -= 1
        raise ValueError(e)

    S = 0  # the regular tile (RF_NB); the short tile (S = 1) only changes NB: the schedule proof above is per NB
    for (C, K), nb in list(RF_NB.items()) + list(RF_NB_EXTRA.items()):
        assert ev(expr, C, K) == nb, (C, K, expr)
    S = 1
    for (C, K), nb in RF_NB_SHORT.items():  # the short tiles (RF S = 1) simulated above
        assert ev(expr, C, K) == nb, (C, K, expr)
    fus = re.search(r"int ssamd_resblock_fusable\(int C, int K\) \{\s*return (.+?);", src, re.S).group(1)
    fus = " ".join(fus.replace("&&", " and ").replace("||", " or ").split())
    for extra in (0, 1):  # g_rf_extra: the whole-block instances of ssamd_resblock_set_whole_extra
        want = set(RF_NB) | (set(RF_NB_EXTRA) if extra else set())
        for C in (32, 64, 128, 256):
            for K in (3, 7, 11):
                assert bool(eval(fus, {"C": C, "K": K, "g_rf_extra": extra})) == ((C, K) in want), (C, K, extra)
