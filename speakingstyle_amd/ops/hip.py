"""HIP/CDNA4 kernel bindings (``csrc/*.hip`` -> ``_lib/libssamd_kernels.so``).

The library is a plain shared object loaded with ctypes (no torch C++ ABI
coupling, seconds to rebuild).  Every entry point takes raw device pointers plus
the current HIP stream, so the kernels order correctly with PyTorch's own work
and are capturable in HIP graphs.  Shapes, dtypes and contiguity are validated
on the host before every launch (a wrong shape must never reach a kernel).

Autograd wiring: one ``torch.autograd.Function`` per fused op; master weights
stay fp32 (flat arena), bf16 operand images in the kernels' layouts are produced
once per optimizer step and cached on the parameter's version counter.
"""
from __future__ import annotations

import collections
import ctypes
import sysconfig
import math
import os
import threading
import weakref
from typing import Optional

import torch

from . import gradslots
from . import reference as ref

_LIB_PATH = os.environ.get("SSAMD_KERNEL_LIB") or os.path.join(  # override: A/B runs of another build
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib", "libssamd_kernels.so")
_lib = None
_lock = threading.Lock()

P = ctypes.c_void_p
I = ctypes.c_int
L_ = ctypes.c_long
F = ctypes.c_float
U64 = ctypes.c_ulonglong

_SIGS = {
    "ssamd_conv_gemm": [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P],
    "ssamd_conv_wgrad": [P, P, P, L_, P, P, I, I, I, I, I, I, I, I, P, P, I, P],
    "ssamd_wgrad_set_variant": [I],
    "ssamd_attn_set_nf": [I, I],
    "ssamd_attn_set_nf32": [I, I],
    "ssamd_wgrad_set_imm": [I],
    "ssamd_gemm_set_splitk": [I],
    "ssamd_gemm_set_splitk_tiny": [I],
    "ssamd_gemm_set_ring_maxk": [I],
    "ssamd_gemm_set_skinny": [I],
    "ssamd_gemm_set_skinny_maxm": [I],
    "ssamd_gemm_set_skinny_w8": [I],
    "ssamd_gemm_set_skinny_any_cin": [I],
    "ssamd_addln_set_small_rows": [I],
    "ssamd_gemm_set_ring_maxn": [I],
    "ssamd_gemm_set_prio": [I],
    "ssamd_gemm_set_ngrp": [I],
    "ssamd_wgrad_set_buf": [I],
    "ssamd_gemm_set_buf": [I],
    "ssamd_gemm_set_stg": [I],
    "ssamd_gemm_set_mask_pre": [I],
    "ssamd_gemm_set_bnh_stg": [I],
    "ssamd_bn_set_dz_cfg": [I, I],
    "ssamd_wgrad_set_pp": [I],
    "ssamd_wgrad_set_prio": [I],
    "ssamd_film_grads": [P, P, P, P, P, P, I, I, P, P, P, P, P, P, I, P, L_, P],
    "ssamd_film_grads_ws": [I],
    "ssamd_attn_set_fwd": [I, I],
    "ssamd_attn_set_kv_dma": [I],
    "ssamd_attn_set_q_dma": [I, I],
    "ssamd_wgrad_set_blocks": [I],
    "ssamd_wgrad_set_cus": [P, I],
    "ssamd_head_fwd": [P, P, P, P, L_, I, I, P, P],
    "ssamd_head_bwd": [P, P, P, P, L_, I, I, P, P, P, P, L_, P],
    "ssamd_head_bwd_ws": [L_, I],
    "ssamd_conv_post": [P, P, P, I, I, I, F, F, P, P, P],
    "ssamd_colsum": [P, P, L_, I, P, L_, P],
    "ssamd_colsum_ws": [L_, I],
    "ssamd_addln_fwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, F, F, U64, F, I, P],
    "ssamd_addln_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, F, F, U64, I, I, P, L_, P],
    "ssamd_addln_bwd_ws": [I, I, I, I],
    "ssamd_addln_wb_reduce": [P, I, I, I, I, P, P, P, P],
    "ssamd_lr_fwd": [P, P, P, P, P, P, I, I, I, I, P],
    "ssamd_lr_bwd": [P, P, P, P, P, I, I, I, I, P],
    "ssamd_pack_info": [P, I, I, P, P, P, P],
    "ssamd_embed_fwd": [I, P, P, P, I, P, P, I, P, P, L_, I, P],
    "ssamd_embed_bwd": [P, P, P, L_, I, I, P],
    "ssamd_onehot": [P, L_, I, P, P],
    "ssamd_l1pair_fwd": [P, P, P, P, I, I, I, I, P, P, L_, P],
    "ssamd_l1pair_ws": [I, I, I],
    "ssamd_clip_adam_ws": [L_],
    "ssamd_l1pair_bwd": [P, P, P, P, I, I, I, I, P, P, P, P, P],
    "ssamd_clip_adam": [P, P, P, P, L_, P, F, F, F, F, F, F, I, P, P, P],
    "ssamd_clip_adam_img": [P, P, P, P, L_, P, F, F, F, F, F, F, I, P, P, P, P, I, P, P, I, L_, P],
    "ssamd_attn_fwd": [P, P, P, P, P, I, I, I, I, F, P],
    "ssamd_attn_bwd": [P, P, P, P, P, P, P, P, L_, I, I, I, I, F, P],
    "ssamd_relu_mask": [P, P, P, L_, P],
    "ssamd_gemm_set_epilogue": [I],
    "ssamd_gemm_set_variant": [I],
    "ssamd_weight_prep": [P, P, I, L_, P],
    "ssamd_weight_prep_tiled": [P, P, I, P],
    "ssamd_stream_wait": [P, P],
}


# HiFi-GAN training kernels (csrc/k_disc.hip; speakingstyle_amd/vocoder/hip_train.py)
_SIGS.update({
    "ssamd_sconv_fwd": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, F, I, P],
    "ssamd_sconv_tout": [I, I, I, I, I],
    "ssamd_sconv_dgrad": [P, P, P, I, I, I, I, I, I, I, I, I, I, I, P],
    "ssamd_sconv_wgrad_ws": [I, I, I, I, I, I, I, I, I],
    "ssamd_sconv_wgrad": [P, P, P, L_, P, P, I, I, I, I, I, I, I, I, I, P],
    "ssamd_sconv_images": [P, P, P, I, I, I, I, I, P],
    "ssamd_act_bwd": [P, P, P, F, P, L_, I, F, P],
    "ssamd_tanh_bwd_f32": [P, P, P, L_, P],
    "ssamd_ew": [I, P, P, P, P, L_, F, P],
    "ssamd_l1_sum": [P, P, L_, I, F, P, P, I, P],
    "ssamd_sum_parts": [P, I, F, P, I, P],
    "ssamd_lsgan": [P, I, F, F, P, F, P, P, P],
    "ssamd_avgpool4": [P, P, I, I, P],
    "ssamd_avgpool4_bwd": [P, P, I, I, I, P],
    "ssamd_mpd_fold": [P, P, I, I, I, P],
    "ssamd_mpd_unfold": [P, P, I, I, I, P],
    "ssamd_stft_prep": [P, P, I, I, I, P],
    "ssamd_stft_unpad": [P, P, I, I, I, I, P],
    "ssamd_mel_l1": [P, I, P, I, I, P, I, I, I, I, F, P, P, I, P],
})


_RESTYPES = {"ssamd_addln_bwd_ws": L_, "ssamd_head_bwd_ws": L_, "ssamd_colsum_ws": L_, "ssamd_embed_bwd_ws": L_,
             "ssamd_clip_adam_ws": L_, "ssamd_l1pair_ws": L_, "ssamd_film_grads_ws": L_,
             "ssamd_sconv_wgrad_ws": L_}


_FAST_PATH = os.path.join(os.path.dirname(_LIB_PATH),
                          "ssamd_fast" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
_USE_FAST = [True]  # bench.py --ctypes-bindings: A/B of the launch-binding host cost


class _KernelLib:
    """Kernel entry points: the generated METH_FASTCALL launch bindings (``csrc/gen_fastcall.py``,
    ~0.35 us per call instead of ctypes' ~3.3 us) where they exist, the ctypes handle otherwise
    (struct-by-value arguments).  Same library mapping, same ABI, same argument lists."""

    def __init__(self, handle, fast):
        self._handle = handle
        self._fast = fast

    def __getattr__(self, name):
        f = getattr(self._fast, name, None) if self._fast is not None and name.startswith("ssamd_") else None
        if f is None:
            f = getattr(self._handle, name)
        self.__dict__[name] = f
        return f


def _load_fast(handle):
    if not _USE_FAST[0] or os.environ.get("SSAMD_KERNEL_LIB") or not os.path.exists(_FAST_PATH):
        return None
    import importlib.util

    spec = importlib.util.spec_from_file_location("ssamd_fast", _FAST_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    # built from the current signature table? (an edited _SIGS entry without a rebuild would convert
    # arguments with the old types)
    import sys

    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "csrc")
    if csrc not in sys.path:
        sys.path.insert(0, csrc)
    import gen_fastcall

    if getattr(mod, "sig_hash", None) != gen_fastcall.sig_hash(_SIGS, _RESTYPES):
        import warnings

        warnings.warn(f"{_FAST_PATH} was generated from a different signature table (rebuild with "
                      "`python csrc/build.py`); using ctypes bindings")
        return None
    # one mapping of the kernel library (one set of its globals: workspaces, LDS opt-ins, variant state)
    mine = ctypes.cast(getattr(handle, mod.entry_name), ctypes.c_void_p).value
    if mod._entry_addr() != mine:
        import warnings

        warnings.warn(f"{_FAST_PATH} resolved a different copy of the kernel library; using ctypes bindings")
        return None
    return mod


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(_LIB_PATH):
                    raise RuntimeError(
                        f"HIP kernel library not built: {_LIB_PATH}. Run `python csrc/build.py` "
                        "(or __graft_entry__.build()). Refusing to fall back to eager PyTorch on a GPU.")
                handle = ctypes.CDLL(_LIB_PATH)
                for name, args in _SIGS.items():
                    fn = getattr(handle, name, None)
                    if fn is not None:
                        fn.argtypes = args
                        fn.restype = _RESTYPES.get(name, I)
                kl = _KernelLib(handle, _load_fast(handle))
                from .. import experimental

                experimental.apply_kernel_switches(kl)  # the validated switches reach every entry path
                _lib = kl
    return _lib


def fast_bindings() -> bool:
    """True when the kernel launches go through the generated native bindings."""
    return lib()._fast is not None


def available() -> bool:
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


def has(name: str) -> bool:
    return getattr(lib(), name, None) is not None


def _ptr(t: Optional[torch.Tensor]):
    """Device address as a plain int: every entry point has ``argtypes`` (_SIGS), so ctypes converts
    it to a pointer itself -- no c_void_p object per operand (~3k per training step)."""
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


_stream_override = [None]  # raw handle of the weight-gradient side stream while its kernels are issued


def _stream():
    """Current HIP stream handle.  The raw getter skips building a torch Stream object (and its
    device-guard calls) for every launch: ~10 us of host time per op on the hot path."""
    o = _stream_override[0]
    if o is not None:
        return o
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


_FALLBACK_OK = os.environ.get("SSAMD_ALLOW_TORCH_FALLBACK") == "1"
_fallback_seen = set()


def _torch_fallback(what: str):
    """A GPU op got a shape / dtype its HIP kernel does not cover.  That is an error (a silent
    torch path on the GPU would hide itself in every benchmark) unless explicitly opted into
    with ``SSAMD_ALLOW_TORCH_FALLBACK=1`` (then it warns once per site)."""
    if not _FALLBACK_OK:
        raise ValueError(f"{what}: not covered by the HIP kernels; set SSAMD_ALLOW_TORCH_FALLBACK=1 to run the "
                         "torch reference op on the GPU instead")
    if what not in _fallback_seen:
        _fallback_seen.add(what)
        import warnings

        warnings.warn(f"torch fallback on the GPU: {what}")


def _need(t, dtype, name):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name}: tensor must be on the GPU")


# ------------------------------------------------------------------------ weight images
# bf16 operand images of fp32 master weights, keyed by (parameter, layout).  An image is
# valid for one (param._version, weight generation) pair: the fused Adam kernel writes the
# arena through raw pointers (torch's version counters do not see it), so the optimizer
# calls ``bump_weight_generation()``; the first stale lookup afterwards refreshes EVERY
# registered image in one batched ``weight_prep`` launch instead of ~2 cast kernels per weight.
_wcache = {}          # key -> [version, generation, weakref(param), image, mode, src_ptr]
_wgen = 0
_wtable = {"n": -1}   # device descriptor table for the batched refresh
_wepoch = 0           # bumped whenever the set of cached images changes (fused Adam plan key)


def bump_weight_generation():
    """Mark every cached weight image stale (call after writing parameters through raw pointers)."""
    global _wgen
    _wgen += 1


def _eligible(w: torch.Tensor) -> bool:
    return w.is_cuda and w.dtype == torch.float32 and w.is_contiguous() and w.dim() in (2, 3)


def _refresh_all(device):
    live = []
    for k in list(_wcache):
        e = _wcache[k]
        owner, w = e[2](), e[7]
        if owner is None or w.data_ptr() != e[5]:
            del _wcache[k]
            _wtable["n"] = -1
            _bump_epoch()
        elif w.device == device and _eligible(w):
            live.append((e, w, owner))  # strong ref: the owner cannot die before its image is stamped
    if _wtable.get("n") != len(live) or _wtable.get("dev") != device:
        import numpy as np
        desc = np.zeros(len(live), dtype=[("src", "<u8"), ("dst", "<u8"), ("cout", "<i4"), ("cin", "<i4"),
                                          ("ks", "<i4"), ("mode", "<i4")])
        cum = np.zeros(len(live) + 1, dtype=np.int64)
        tiles = []
        for i, (e, w, _) in enumerate(live):
            ks = w.shape[2] if w.dim() == 3 else 1
            desc[i] = (w.data_ptr(), e[3].data_ptr(), w.shape[0], w.shape[1], ks, e[4])
            cum[i + 1] = cum[i] + w.numel()
            K = w.shape[1] * ks
            for co0 in range(0, w.shape[0], 64):
                for j0 in range(0, K, 64):
                    tiles.append((i, co0, j0, 0))
        tiles = np.asarray(tiles, dtype=np.int32).reshape(-1, 4)
        _wtable.update(n=len(live), dev=device, total=int(cum[-1]),
                       desc=torch.from_numpy(desc.view(np.uint8).copy()).to(device),
                       cum=torch.from_numpy(cum).to(device),
                       tiles=torch.from_numpy(tiles).to(device), ntiles=len(tiles))
    if _wtable["n"]:
        if has("ssamd_weight_prep_tiled"):  # 64x64 LDS tiles: coalesced reads and transposed writes
            rc = lib().ssamd_weight_prep_tiled(_ptr(_wtable["desc"]), _ptr(_wtable["tiles"]), _wtable["ntiles"],
                                               _stream())
        else:
            rc = lib().ssamd_weight_prep(_ptr(_wtable["desc"]), _ptr(_wtable["cum"]), _wtable["n"], _wtable["total"],
                                         _stream())
        _check(rc, "ssamd_weight_prep")
    for e, w, owner in live:
        e[0], e[1] = owner._version, _wgen


def refresh_stale_images(device):
    """Bring every cached weight image up to date now (one batched launch if any is stale).  A captured
    HIP-graph step reads the images by address and never performs the lookup that refreshes them lazily;
    the fused Adam launch rewrites the arena's images itself, this covers any other writer."""
    for e in _wcache.values():
        owner = e[2]()
        if owner is not None and (e[0] != owner._version or e[1] != _wgen):
            _refresh_all(device)
            return True
    return False


def _cached(param: torch.Tensor, kind: str, mode: int, make, src: Optional[torch.Tensor] = None):
    """Image of ``src`` (default: ``param`` itself), cached under the parameter ``param``."""
    src = param if src is None else src
    if not isinstance(param, torch.nn.Parameter):  # transient tensors: ids / addresses get reused
        return make(src.detach())
    key = (id(param), kind, tuple(src.shape))
    hit = _wcache.get(key)
    if hit is not None and hit[2]() is param and hit[5] == src.data_ptr() and hit[6] == tuple(src.shape):
        if hit[0] == param._version and hit[1] == _wgen:
            return hit[3]
        if _eligible(src) and has("ssamd_weight_prep"):
            _refresh_all(src.device)
            return hit[3]
    img = make(src.detach())
    _wcache[key] = [param._version, _wgen, weakref.ref(param), img, mode, src.data_ptr(), tuple(src.shape),
                    src.detach()]
    _wtable["n"] = -1  # entry set changed: rebuild the descriptor table on the next refresh
    _bump_epoch()
    return img


def _bump_epoch():
    global _wepoch
    _wepoch += 1


def weight_fwd(w: torch.Tensor, owner: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[Cout, Cin, ks] (or Linear [out, in]) fp32 -> bf16 [Cout][ks][Cin]."""
    o = w if owner is None else owner
    if w.dim() == 2:
        return _cached(o, "fwd", 0, lambda x: x.to(torch.bfloat16).contiguous(), w)
    return _cached(o, "fwd", 0, lambda x: x.permute(0, 2, 1).to(torch.bfloat16).contiguous(), w)


def weight_dgrad(w: torch.Tensor, owner: Optional[torch.Tensor] = None) -> torch.Tensor:
    """-> bf16 [Cin][ks][Cout] with taps flipped (data gradient = conv with W^T)."""
    o = w if owner is None else owner
    if w.dim() == 2:
        return _cached(o, "dgrad", 1, lambda x: x.t().to(torch.bfloat16).contiguous(), w)
    return _cached(o, "dgrad", 1, lambda x: x.flip(2).permute(1, 2, 0).to(torch.bfloat16).contiguous(), w)


_ACT = {None: 0, "relu": 1, "lrelu": 2, "tanh": 3, "relu_ln": 1}  # relu_ln: ReLU, mask left to the consumer LN

_ws = {}
# HIP graphs (infer/graphs.py) bake the workspace address into their kernels: once one has been captured, a
# workspace that grows is retired here instead of freed, so a later replay of an older graph never writes
# into memory the caching allocator has handed to another tensor
_GRAPHS_LIVE = [False]
_ws_retired = []


def graphs_live():
    """Called before the first HIP-graph capture: from now on no workspace a graph may hold is ever freed (the
    Python scratch buffers here, the split-K workspaces of the GEMM library)."""
    if not _GRAPHS_LIVE[0]:
        _GRAPHS_LIVE[0] = True
        lib().ssamd_gemm_retain_workspaces(1)


def _workspace(device, nfloats: int) -> torch.Tensor:
    """Scratch buffer of the current stream (the weight-gradient side stream has its own, allocated
    under that stream so the caching allocator orders its reuse after the side-stream kernels)."""
    key = (device, _stream())
    cur = _ws.get(key)
    if cur is None or cur.numel() < nfloats:
        if cur is not None and (_GRAPHS_LIVE[0] or torch.cuda.is_current_stream_capturing()):
            _ws_retired.append(cur)
        side = _side_by_handle.get(key[1])
        if side is not None:
            with torch.cuda.stream(side):
                cur = torch.empty(max(nfloats, 1 << 20), dtype=torch.float32, device=device)
        else:
            cur = torch.empty(max(nfloats, 1 << 20), dtype=torch.float32, device=device)
        _ws[key] = cur
    return cur


# ------------------------------------------------------------------------ weight-gradient side stream
# The weight gradients of a layer feed only the optimizer (and the DDP buckets), never the rest of the
# backward chain.  They run on a second HIP stream, so their GEMMs fill the CUs the data-gradient chain
# leaves idle (partial last rounds of 256x256 tiles, the small encoder-sized kernels).  Only kernels
# that write straight into claimed arena slots go there (nothing the main stream touches before the
# join); their inputs are record_stream()-ed so the caching allocator cannot recycle them early.
# join_side_streams() orders the current stream after everything queued (before the optimizer reads the
# arena and before a gradient bucket is all-reduced).
_side = {}
_side_used = {}
_side_by_handle = {}  # raw handle -> torch Stream (workspace allocation under the side stream)
_side_keep = {}       # device -> inputs of queued side-stream kernels, released at the join
# issue a layer's weight gradient (side stream) BEFORE its data gradient (main stream): the side stream
# then waits only for the operands, not for the data-gradient GEMM too.  It pays when the data-gradient
# GEMMs leave CUs idle: fewer 256-row tiles than ~1.25 waves of the device's CUs (e.g. 320 tiles = 82k
# rows on 256 CUs).  Measured (profiles/r3_v10_wgrad_first_ab.txt, as a row threshold of 80k): +0.6 %
# LJSpeech (~113k rows: not first), +0.7 % BC2013, +1.2 % GST (40-50k rows: first), vs never; always-first
# -0.7 % on LJSpeech.  Experiment switches ``wgrad_first`` (0 / 1 / auto) and ``wgrad_first_waves``.
_CUS = {}


def _device_cus(dev_index=None) -> int:
    i = torch.cuda.current_device() if dev_index is None else dev_index
    n = _CUS.get(i)
    if n is None:
        n = _CUS[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return n


def _wgrad_first(rows: int) -> bool:
    from .. import experimental

    m = experimental.get("wgrad_first")
    if m != "auto":
        return m == "1"
    return (rows + 255) // 256 < experimental.get("wgrad_first_waves") * _device_cus()


_SIDE_WGRAD = [True]
_SIDE_LN = [True]  # LayerNorm weight-gradient reductions on the side stream too (A/B: bench --ln-reduce-main)


def set_wgrad_stream(enabled: bool):
    _SIDE_WGRAD[0] = bool(enabled)


def side_stream_handle(device):
    """Raw handle of the weight-gradient side stream of ``device`` (created on first use)."""
    return _side_stream(device).cuda_stream


def _side_stream(device):
    s = _side.get(device.index)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _side[device.index] = s
        _side_by_handle[s.cuda_stream] = s
    return s


def wgrad_async(launch, inputs, slots_ok: bool, params=()):
    """``launch()`` (weight-gradient kernels writing the arena slots of ``params``) on the side stream
    when every slot was claimed and every parameter is known to receive that single gradient
    (``gradslots.single_contribution``: autograd adopts the slot view without touching its data).

    Host-lean: one native event record + stream wait (``ssamd_stream_wait``), the launch issued with
    the side stream's raw handle (``_stream_override``; ``launch`` allocates nothing but the side
    stream's own workspace), and the inputs kept alive until ``join_side_streams`` instead of a
    ``record_stream`` per tensor (after the join the current stream is ordered behind every
    side-stream read, so the caching allocator may recycle them).  ``inputs`` must list EVERY device
    tensor the launch reads, the packed-row tables included: one freed early could be handed out by
    the main stream's allocator while the side-stream kernel is still pending.  (Measured and lost:
    issuing each launch one weight-gradient call later, so the main stream's next kernels are queued
    first -- neutral, profiles/r3_v8_wgrad_defer_ab.txt.)"""
    if not (_SIDE_WGRAD[0] and slots_ok and all(gradslots.single_contribution(p) for p in params)):
        return launch()
    dev = inputs[0].device
    gradslots.mark_side(params)
    sh = _side_stream(dev).cuda_stream
    _check(lib().ssamd_stream_wait(sh, _stream()), "ssamd_stream_wait")
    _stream_override[0] = sh
    try:
        out = launch()
    finally:
        _stream_override[0] = None
    keep = _side_keep.get(dev.index)
    if keep is None:
        keep = _side_keep[dev.index] = []
    keep.extend(t for t in inputs if t is not None)
    _side_used[dev.index] = True
    if len(keep) > 4096:  # a caller that never joins (no optimizer step): bound the held references
        join_side_streams()
    return out


def side_stream_for_collective(device):
    """The side stream, made to wait for the current (compute) stream, when weight-gradient kernels are
    queued on it since the last join -- else None.  A collective issued with this stream current is
    ordered after both streams' gradient writes while the compute stream itself does not wait
    (``parallel/ddp.py::GradBuckets._launch``).  The side stream only gains an order it already had:
    every later side-stream launch waits for the compute stream anyway (``wgrad_async``)."""
    idx = device.index
    if not _side_used.get(idx):
        return None
    s = _side[idx]
    _check(lib().ssamd_stream_wait(s.cuda_stream, _stream()), "ssamd_stream_wait")
    return s


def join_side_streams(defer_release=False):
    """Make the current stream wait for the side-stream weight-gradient kernels.  The inputs those
    kernels held are released here, or -- ``defer_release`` -- handed back to the caller: dropping a
    few hundred tensors costs the host ~0.5 ms, which at the end of a backward is GPU idle time, so
    the trainer drops them while the next step's forward keeps the GPU busy (their memory stays
    reserved until then; safe either way, the join orders every later reuse after those kernels)."""
    held = []
    for idx, used in _side_used.items():
        if used:
            with torch.cuda.device(idx):
                _check(lib().ssamd_stream_wait(_stream(), _side[idx].cuda_stream), "ssamd_stream_wait")
            _side_used[idx] = False
            keep = _side_keep.get(idx)
            if keep:
                if defer_release:
                    held.append(keep)
                    _side_keep[idx] = []
                else:
                    keep.clear()
    return held


# ------------------------------------------------------------------------ raw launchers
def _rinfo_ptr(rinfo, rows):
    """Packed-sequence row table: int32 [rows, 2] = (position in sequence, sequence length)."""
    if rinfo is None:
        return None
    _need(rinfo, torch.int32, "rinfo")
    assert rinfo.numel() == 2 * rows, "rinfo must hold (t, len) for every row"
    return _ptr(rinfo)

def conv_gemm_raw(x, wimg, bias, B, L, Cin, ks, dil, pad, N, act=0, aux=None, resid=None, lens=None, out_f32=False,
                  rinfo=None):
    _need(x, torch.bfloat16, "conv_gemm.x")
    _need(wimg, torch.bfloat16, "conv_gemm.w")
    assert x.numel() == B * L * Cin, "conv_gemm: x shape mismatch"
    assert wimg.numel() == N * ks * Cin, "conv_gemm: w shape mismatch"
    if Cin % 8:
        raise ValueError("conv_gemm: Cin must be a multiple of 8")
    y = torch.empty(B, L, N, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    if bias is not None:
        _need(bias, torch.float32, "conv_gemm.bias")
        assert bias.numel() == N
    for t, nm in ((aux, "aux"), (resid, "resid")):
        if t is not None:
            _need(t, torch.bfloat16, "conv_gemm." + nm)
            assert t.numel() == B * L * N
    if lens is not None:
        _need(lens, torch.int64, "conv_gemm.lens")
        assert lens.numel() == B
    rc = lib().ssamd_conv_gemm(_ptr(x), _ptr(wimg), _ptr(bias), _ptr(aux), _ptr(resid), _ptr(lens), _ptr(y),
                               int(out_f32), B, L, Cin, ks, dil, pad, N, act, N, _rinfo_ptr(rinfo, B * L), _stream())
    _check(rc, "ssamd_conv_gemm")
    return y


_SIGS["ssamd_conv_gemm_mask"] = [P, P, P, P, I, I, I, I, I, I, I, I, P, P, P, P]


def conv_gemm_mask_raw(x, wimg, bias, B, L, Cin, ks, pad, N, act, rinfo=None, mask_out=None, mask_in=None):
    """conv_gemm with the ReLU bitmask epilogue (``ssamd_conv_gemm_mask``): ``mask_out`` (uint8
    [B*L, N/8], act = ReLU) receives bit (y > 0) per element; ``mask_in`` zeroes the elements whose
    bit is clear (the data gradient through that ReLU)."""
    _need(x, torch.bfloat16, "conv_mask.x")
    _need(wimg, torch.bfloat16, "conv_mask.w")
    assert x.numel() == B * L * Cin and wimg.numel() == N * ks * Cin, "conv_mask: shape"
    for m in (mask_out, mask_in):
        if m is not None:
            _need(m, torch.uint8, "conv_mask.mask")
            assert m.numel() == B * L * N // 8, "conv_mask: mask shape"
    if bias is not None:
        _need(bias, torch.float32, "conv_mask.bias")
    y = torch.empty(B, L, N, device=x.device, dtype=torch.bfloat16)
    rc = lib().ssamd_conv_gemm_mask(_ptr(x), _ptr(wimg), _ptr(bias), _ptr(y), B, L, Cin, ks, 1, pad, N, act,
                                    _rinfo_ptr(rinfo, B * L), _ptr(mask_out), _ptr(mask_in), _stream())
    _check(rc, "ssamd_conv_gemm_mask")
    return y


def conv_wgrad_raw(x, dy, B, L, Cin, ks, dil, pad, N, with_bias=False, dW=None, db=None, rinfo=None, cu=None):
    """-> dW [N, Cin, ks] fp32 (and db [N] when ``with_bias``: fused column sums of dY).

    ``dW`` / ``db``: optional destinations (arena gradient slots), fully overwritten."""
    _need(x, torch.bfloat16, "wgrad.x")
    _need(dy, torch.bfloat16, "wgrad.dy")
    assert x.numel() == B * L * Cin and dy.numel() == B * L * N
    if N % 8:
        raise ValueError("wgrad: N must be a multiple of 8")
    K = ks * Cin
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    max_splits = max(1, min(64, (1536 + tiles - 1) // tiles))  # 128x128 kernels
    if N >= 256 and K >= 256:  # 256x256 kernel: up to one split per CU per output tile (C++ cost model)
        max_splits = max(max_splits, min(256, 256 // max(1, ((N + 255) // 256) * ((K + 255) // 256)) * 2))
    ws = _workspace(x.device, max_splits * (N * K + N))
    if dW is None:
        dW = torch.empty(N, Cin, ks, device=x.device, dtype=torch.float32)
    else:
        assert dW.dtype == torch.float32 and dW.is_contiguous() and dW.numel() == N * Cin * ks
    if not with_bias:
        db = None
    elif db is None:
        db = torch.empty(N, device=x.device, dtype=torch.float32)
    else:
        assert db.dtype == torch.float32 and db.is_contiguous() and db.numel() == N
    rc = lib().ssamd_conv_wgrad(_ptr(x), _ptr(dy), _ptr(ws), ws.numel(), _ptr(dW), _ptr(db), B, L, Cin, ks, dil, pad,
                                N, max_splits, _rinfo_ptr(rinfo, B * L), _ptr(cu),
                                0 if cu is None else cu.numel() - 1, _stream())
    _check(rc, "ssamd_conv_wgrad")
    return (dW, db) if with_bias else dW


def colsum_raw(dy, N, db=None):
    _need(dy, torch.bfloat16, "colsum.dy")
    if db is None:
        db = torch.empty(N, device=dy.device, dtype=torch.float32)
    M = dy.numel() // N
    ws = _workspace(dy.device, int(lib().ssamd_colsum_ws(M, N)))
    rc = lib().ssamd_colsum(_ptr(dy), _ptr(db), M, N, _ptr(ws), ws.numel(), _stream())
    _check(rc, "ssamd_colsum")
    return db


def relu_mask_(dy, y, out=None):
    """out = dy * (y > 0) (bf16); in place into dy when ``out`` is None."""
    _need(dy, torch.bfloat16, "relu_mask.dy")
    _need(y, torch.bfloat16, "relu_mask.y")
    assert dy.is_contiguous() and y.is_contiguous() and y.numel() == dy.numel()
    out = dy if out is None else out
    rc = lib().ssamd_relu_mask(_ptr(dy), _ptr(y), _ptr(out), dy.numel(), _stream())
    _check(rc, "ssamd_relu_mask")
    return out


# ------------------------------------------------------------------------ conv / linear
class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad, dil, act, out_f32, pack=None):
        """``pack``: x is packed [1, R, Cin]; the conv zero-pads at every sequence end (rinfo)."""
        B, L, Cin = x.shape
        ks = 1 if w.dim() == 2 else w.shape[2]
        N = w.shape[0]
        xc = x.contiguous()
        bf = None if b is None else b.detach().float().contiguous()
        rinfo = pack.rinfo if (pack is not None and ks > 1) else None
        if rinfo is not None:
            assert B == 1 and L == pack.R, "packed conv: x must be [1, R, C]"
        y = conv_gemm_raw(xc, weight_fwd(w), bf, B, L, Cin, ks, dil, pad, N, _ACT[act], out_f32=out_f32,
                          rinfo=rinfo)
        ctx.pack = pack if rinfo is not None else None
        ctx.geom = (B, L, Cin, ks, dil, pad, N)
        ctx.act = act
        ctx.has_b = b is not None
        ctx.b = b if isinstance(b, torch.nn.Parameter) else None  # gradient-slot owner only
        ctx.save_for_backward(xc, w, y if act == "relu" else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w, y = ctx.saved_tensors
        B, L, Cin, ks, dil, pad, N = ctx.geom
        dy = dy.to(torch.bfloat16).contiguous()
        if ctx.act == "relu":
            dy = relu_mask_(dy, y, out=torch.empty_like(dy))  # out of place: dy may be shared
        elif ctx.act == "relu_ln":
            pass  # the consuming add_layernorm(relu_input=True) applied the ReLU mask in its backward
        elif ctx.act is not None:
            raise NotImplementedError("backward for activation " + str(ctx.act))
        dx = dw = db = None
        pk = ctx.pack
        rinfo = None if pk is None else pk.rinfo
        first = _wgrad_first(B * L)
        if ctx.needs_input_grad[0] and not first:
            dx = conv_gemm_raw(dy, weight_dgrad(w), None, B, L, N, ks, dil, (ks - 1) * dil - pad, Cin, rinfo=rinfo)
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        sb = gradslots.claim(ctx.b) if want_b else None
        if ctx.needs_input_grad[1]:
            sw = gradslots.claim(w)
            res = wgrad_async(lambda: conv_wgrad_raw(xc, dy, B, L, Cin, ks, dil, pad, N, with_bias=want_b, dW=sw,
                                                     db=sb, rinfo=rinfo, cu=None if pk is None else pk.cu),
                              (xc, dy, rinfo, None if pk is None else pk.cu),
                              sw is not None and (sb is not None or not want_b),
                              (w, ctx.b) if want_b else (w,))
            dw, db = res if want_b else (res, None)
            if w.dim() == 2:
                dw = dw.view(N, Cin)
        elif want_b:
            db = colsum_raw(dy, N, sb)
        if ctx.needs_input_grad[0] and first:
            dx = conv_gemm_raw(dy, weight_dgrad(w), None, B, L, N, ks, dil, (ks - 1) * dil - pad, Cin, rinfo=rinfo)
        return dx, dw, db, None, None, None, None, None


def conv1d(x, w, b=None, pad=0, dil=1, act=None, out_f32=False, pack=None):
    return _ConvFn.apply(x, w, b, pad, dil, act, out_f32, pack)


def linear(x, w, b=None, act=None, out_f32=False):
    shp = x.shape
    x3 = x.reshape(1, -1, shp[-1]) if x.dim() != 3 else x
    if x3.shape[-1] % 8 or w.shape[0] % 8:
        # not MFMA-shaped (the N = 1 variance-predictor head has its own kernel: predictor_head)
        _torch_fallback(f"linear {x3.shape[-1]}->{w.shape[0]} (dims must be multiples of 8)")
        return ref.linear(x, w, b, act)
    y = _ConvFn.apply(x3, w, b, 0, 1, act, out_f32)
    return y.reshape(*shp[:-1], w.shape[0])


class GradMailbox:
    """Hands the residual-branch gradient of a sub-layer input to the GEMM that consumes the same
    input: ``add_layernorm(..., residual=x, mailbox=mb)`` puts d(residual) here instead of
    returning it, and the first GEMM of the sub-layer (``linear_group`` / ``ffn`` on x, whose
    backward runs later) adds it in its data-gradient epilogue (``resid``).  Autograd then sees
    one gradient for x: no separate bf16 accumulation kernel per sub-layer."""

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None

    def put(self, g):
        self.grad = g if self.grad is None else self.grad + g

    def take(self):
        g, self.grad = self.grad, None
        return g


def _resid_for(mailbox, like):
    if mailbox is None:
        return None
    g = mailbox.take()
    if g is None:
        return None
    g = g.to(torch.bfloat16).contiguous()
    assert g.shape == like.shape, "mailbox gradient shape mismatch"
    return g


class _GroupLinearFn(torch.autograd.Function):
    """One GEMM for several Linear layers whose weights / biases are contiguous in the
    arena: ``wf`` / ``bf`` are the fused data views; the member parameters are inputs
    only so autograd routes each one its slice of the (in-place written) gradient."""

    @staticmethod
    def forward(ctx, x, wf, bf, n, mailbox, *params):
        ws, bs = params[:n], params[n:]
        B, L, Cin = x.shape
        N = wf.shape[0]
        xc = x.contiguous()
        y = conv_gemm_raw(xc, weight_fwd(wf, owner=ws[0]), bf, B, L, Cin, 1, 1, 0, N, 0)
        ctx.mailbox = mailbox
        ctx.save_for_backward(xc, wf)
        ctx.members = (ws, bs)
        ctx.dims = (B, L, Cin, N)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wf = ctx.saved_tensors
        ws, bs = ctx.members
        B, L, Cin, N = ctx.dims
        dy = dy.to(torch.bfloat16).contiguous()
        first = _wgrad_first(B * L)
        if not first:
            dx = conv_gemm_raw(dy, weight_dgrad(wf, owner=ws[0]), None, B, L, N, 1, 1, 0, Cin,
                               resid=_resid_for(ctx.mailbox, xc))
        sw, sb = gradslots.claim_fused(ws), gradslots.claim_fused(bs)
        dw, db = wgrad_async(lambda: conv_wgrad_raw(xc, dy, B, L, Cin, 1, 1, 0, N, with_bias=True,
                                                    dW=None if sw is None else sw.view(N, Cin, 1), db=sb),
                             (xc, dy), sw is not None and sb is not None, tuple(ws) + tuple(bs))
        if first:
            dx = conv_gemm_raw(dy, weight_dgrad(wf, owner=ws[0]), None, B, L, N, 1, 1, 0, Cin,
                               resid=_resid_for(ctx.mailbox, xc))
        dw = dw.view(N, Cin)
        return (dx, None, None, None, None, *gradslots.split_rows(dw, ws), *gradslots.split_rows(db, bs))


_GROUP_CAT = None  # IdCache: first weight of a projection group -> (versions, fused weight, bias)


def linear_group(x, weights, biases, mailbox=None):
    weights, biases = list(weights), list(biases)
    wf, bf = gradslots.fused_data(weights), gradslots.fused_data(biases)
    if wf is None or bf is None:
        if mailbox is not None:
            raise ValueError("residual mailbox needs the fused (arena) projection path")
        if torch.is_grad_enabled():
            w, b = torch.cat(weights, 0), torch.cat(biases, 0)
        else:  # inference outside an arena: the concatenation cached per weight version, held as a Parameter so
            #     that its bf16 operand image is cached too (_cached); nothing is attached to the model's tensors
            key = tuple((t.data_ptr(), t._version) for t in weights + biases)
            global _GROUP_CAT
            if _GROUP_CAT is None:
                from . import IdCache

                _GROUP_CAT = IdCache()
            hit = _GROUP_CAT.get(weights[0])
            if hit is None or hit[0] != key:
                wc = torch.nn.Parameter(torch.cat([t.detach() for t in weights], 0), requires_grad=False)
                hit = (key, wc, torch.cat([t.detach().float() for t in biases], 0).contiguous())
                _GROUP_CAT.put(weights[0], hit)
            w, b = hit[1], hit[2]
        return linear(x, w, b)
    shp = x.shape
    x3 = x.reshape(1, -1, shp[-1]) if x.dim() != 3 else x
    y = _GroupLinearFn.apply(x3, wf, bf, len(weights), mailbox, *weights, *biases)
    return y.reshape(*shp[:-1], wf.shape[0])


class _FFNFn(torch.autograd.Function):
    """conv(k0) -> ReLU -> conv(k1): the ReLU derivative is fused into the
    data-gradient epilogue of the second conv (aux = h), so no extra pass."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, rinfo, mailbox, need_mask=True):
        B, L, C = x.shape
        ctx.mailbox = mailbox
        k1, k2 = w1.shape[2], w2.shape[2]
        H = w1.shape[0]
        xc = x.contiguous()
        rinfo, cu = (None, None) if rinfo is None else rinfo
        r1 = rinfo if k1 > 1 else None
        r2 = rinfo if k2 > 1 else None
        ctx.cu = (cu if k1 > 1 else None, cu if k2 > 1 else None)
        mask = None
        if H >= 256 and H % 8 == 0 and need_mask and has("ssamd_conv_gemm_mask"):
            # ReLU bitmask of h for the second conv's data gradient (M x H/8 bytes instead of h itself); not
            # in inference, where the plain epilogue keeps the split-K path open for tile-poor row counts
            mask = torch.empty(B * L, H // 8, device=x.device, dtype=torch.uint8)
            h = conv_gemm_mask_raw(xc, weight_fwd(w1), b1.detach().float(), B, L, C, k1, (k1 - 1) // 2, H, 1,
                                   rinfo=r1, mask_out=mask)
        else:
            h = conv_gemm_raw(xc, weight_fwd(w1), b1.detach().float(), B, L, C, k1, 1, (k1 - 1) // 2, H, 1,
                              rinfo=r1)
        z = conv_gemm_raw(h, weight_fwd(w2), b2.detach().float(), B, L, H, k2, 1, (k2 - 1) // 2, C, 0, rinfo=r2)
        ctx.rinfo = (r1, r2)
        ctx.save_for_backward(xc, h, w1, w2, mask)
        ctx.biases = (b1, b2)
        ctx.dims = (B, L, C, H, k1, k2)
        return z

    @staticmethod
    def backward(ctx, dz):
        xc, h, w1, w2, mask = ctx.saved_tensors
        B, L, C, H, k1, k2 = ctx.dims
        dz = dz.to(torch.bfloat16).contiguous()
        p1, p2 = (k1 - 1) // 2, (k2 - 1) // 2
        b1, b2 = ctx.biases
        r1, r2 = ctx.rinfo
        first = _wgrad_first(B * L)

        def _wgrad2():
            s2w, s2b = gradslots.claim(w2), gradslots.claim(b2)
            return wgrad_async(lambda: conv_wgrad_raw(h, dz, B, L, H, k2, 1, p2, C, with_bias=True, dW=s2w,
                                                      db=s2b, rinfo=r2, cu=ctx.cu[1]),
                               (h, dz, r2, ctx.cu[1]), s2w is not None and s2b is not None, (w2, b2))

        if first:
            dw2, db2 = _wgrad2()
        if mask is not None:
            dh = conv_gemm_mask_raw(dz, weight_dgrad(w2), None, B, L, C, k2, (k2 - 1) - p2, H, 0, rinfo=r2,
                                    mask_in=mask)
        else:
            dh = conv_gemm_raw(dz, weight_dgrad(w2), None, B, L, C, k2, 1, (k2 - 1) - p2, H, 0, aux=h, rinfo=r2)
        if not first:
            dw2, db2 = _wgrad2()

        def _wgrad1():
            s1w, s1b = gradslots.claim(w1), gradslots.claim(b1)
            return wgrad_async(lambda: conv_wgrad_raw(xc, dh, B, L, C, k1, 1, p1, H, with_bias=True, dW=s1w,
                                                      db=s1b, rinfo=r1, cu=ctx.cu[0]),
                               (xc, dh, r1, ctx.cu[0]), s1w is not None and s1b is not None, (w1, b1))

        if first:
            dw1, db1 = _wgrad1()
        dx = conv_gemm_raw(dh, weight_dgrad(w1), None, B, L, H, k1, 1, (k1 - 1) - p1, C, 0, rinfo=r1,
                           resid=_resid_for(ctx.mailbox, xc))
        if not first:
            dw1, db1 = _wgrad1()
        return dx, dw1, db1, dw2, db2, None, None, None


def ffn(x, w1, b1, w2, b2, pack=None, mailbox=None):
    if pack is not None:
        assert x.shape[0] == 1 and x.shape[1] == pack.R, "packed FFN expects [1, R, C]"
    grad = torch.is_grad_enabled() and any(t.requires_grad for t in (x, w1, b1, w2, b2))
    return _FFNFn.apply(x, w1, b1, w2, b2, None if pack is None else (pack.rinfo, pack.cu), mailbox, grad)


# ------------------------------------------------------------------------ add + LayerNorm
_seed_counter = [0x1234]


def _next_seed():
    _seed_counter[0] = (_seed_counter[0] * 6364136223846793005 + 1442695040888963407) & ((1 << 64) - 1)
    return _seed_counter[0]


def set_seed(s: int):
    _seed_counter[0] = int(s) & ((1 << 64) - 1)


def get_seed() -> int:
    return _seed_counter[0]


# Per-step dropout salt (csrc/common.h g_drop_salt, one copy per kernel file): the step-dependent part of
# every dropout mask.  ``set_dropout_salt`` writes the value into a device word (an ordinary stream-ordered
# copy, outside any captured graph); ``load_dropout_salt`` launches the three loaders that copy it into the
# kernel files' globals -- captured at the start of a HIP-graph step, so each replay draws its own masks.
_SIGS.update({"ssamd_norm_salt_load": [P, P], "ssamd_bn_salt_load": [P, P], "ssamd_gemm_salt_load": [P, P]})
_salt = {}


def _salt_word(device):
    w = _salt.get(device)
    if w is None:
        w = _salt[device] = torch.zeros(1, device=device, dtype=torch.int64)
    return w


def set_dropout_salt(value: int, device=None):
    device = device or torch.device("cuda", torch.cuda.current_device())
    v = int(value) & ((1 << 63) - 1)
    _salt_word(device).fill_(v)


def load_dropout_salt(device=None):
    device = device or torch.device("cuda", torch.cuda.current_device())
    w = _salt_word(device)
    for fn in ("ssamd_norm_salt_load", "ssamd_bn_salt_load", "ssamd_gemm_salt_load"):
        _check(getattr(lib(), fn)(_ptr(w), _stream()), fn)


_F32_MEMO = {}


def _f32_view(t):
    """fp32 contiguous copy of a (small) FiLM vector, shared by every LayerNorm site that uses
    the same tensor in this step (the 11 FiLM sites of a styled model read ONE gamma / beta)."""
    if t.dtype == torch.float32 and t.is_contiguous():
        return t.detach()
    key = (t.data_ptr(), t._version, tuple(t.shape), t.dtype)
    hit = _F32_MEMO.get(key)
    if hit is not None and hit[0]() is t:
        return hit[1]
    if len(_F32_MEMO) > 64:
        _F32_MEMO.clear()
    v = t.detach().float().contiguous()
    _F32_MEMO[key] = (weakref.ref(t), v)
    return v


class _FilmAcc:
    """Running d gamma / d beta of the LayerNorm sites sharing one FiLM (gamma, beta) pair -- used
    for the model's style tensors (fresh per forward, marked ``_ssamd_film_acc``), never for a
    tensor reused across graphs (a leaf fed to several forwards gets per-site gradients).  The
    first site to run backward returns the buffer (a view in gamma's shape/dtype: autograd keeps it
    as-is in the producer's input buffer), the later sites add into it in place and return None.
    The producer of gamma / beta runs only after every site reachable in this backward, so it reads
    the complete sum -- one gradient instead of one per site plus an autograd add per extra site.
    Contract: a marked tensor is consumed ONLY by FiLM LayerNorm sites (true for the model's style
    gamma / beta); another consumer's gradient could be added out of place before the later sites
    add theirs into the buffer."""

    __slots__ = ("ref", "buf")

    def __init__(self, g):
        self.ref = weakref.ref(g)
        self.buf = None


_FILM_ACC = {}


def _film_acc(g):
    key = (g.data_ptr(), g._version, tuple(g.shape), g.dtype)
    acc = _FILM_ACC.get(key)
    if acc is None or acc.ref() is not g:
        if len(_FILM_ACC) > 64:
            _FILM_ACC.clear()
        acc = _FilmAcc(g)
        _FILM_ACC[key] = acc
    return acc


class _FilmCatFn(torch.autograd.Function):
    """torch.cat of the FiLM scalars whose backward parks the L2 term's gradient in the
    gradslots.FilmL2Holder (folded in by the sites' film_grads kernels) instead of returning it."""

    @staticmethod
    def forward(ctx, holder, *ps):
        holder.reset()
        ctx.holder = holder
        ctx.ids = [id(p) for p in ps]
        return torch.cat([p.detach().reshape(-1) for p in ps])

    @staticmethod
    def backward(ctx, g):
        h = ctx.holder
        pend, h.pending = h.pending, set()
        if h.sites_started or not pend:  # a site already ran / none will: plain per-scalar gradients
            return (None, *[g[i:i + 1] for i in range(g.numel())])
        h.grad = g.float().contiguous()  # the sites in ``pend`` fold their entries in
        return (None, *[None if k in pend else g[i:i + 1] for i, k in enumerate(ctx.ids)])


def film_scalars_cat(ps):
    """Concat of the FiLM scalar parameters (``[1]`` each) for the ``lambda_f`` L2 loss term."""
    if not ps:
        return None
    if not (torch.is_grad_enabled() and ps[0].is_cuda and all(p.numel() == 1 for p in ps)
            and any(p.requires_grad for p in ps)):
        return torch.cat(ps)
    return _FilmCatFn.apply(gradslots.film_holder_for(ps), *ps)


class _AddLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, res, w, b, g, bt, sg, sb, lens, pre_p, post_p, seed, eps, cu, geom, mailbox, relu_in=False):
        B, L, C = a.shape if geom is None else geom  # packed: (sequences, longest, C) over [1, R, C] rows
        # relu_in: a = ReLU(conv) whose backward left the ReLU mask to this one (conv1d act "relu_ln")
        ctx.relu_in = bool(relu_in)
        ac = a.contiguous()
        rc_ = None if res is None else res.contiguous()
        gf = None if g is None else _f32_view(g)
        bf = None if bt is None else _f32_view(bt)
        out = torch.empty_like(ac)
        mean = torch.empty(a.numel() // C, device=a.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        rc = lib().ssamd_addln_fwd(_ptr(ac), _ptr(rc_), _ptr(w), _ptr(b), _ptr(gf), _ptr(bf), _ptr(sg), _ptr(sb),
                                   _ptr(lens), _ptr(cu), _ptr(out), _ptr(mean), _ptr(rstd), B, L, C, pre_p,
                                   post_p, seed, eps, 0, _stream())
        _check(rc, "ssamd_addln_fwd")
        ctx.cu = cu
        ctx.mailbox = mailbox
        ctx.film_scales = (sg, sb)  # the Parameters themselves: gradient-slot owners
        for k, p in ((6, sg), (7, sb)):
            hold = gradslots.film_holder(p) if ctx.needs_input_grad[k] else None
            if hold is not None:
                hold.register_site(p)
        ctx.acc = None
        if (g is not None and bt is not None and getattr(g, "_ssamd_film_acc", False)
                and g.dtype == bt.dtype and g.dtype in (torch.float32, torch.bfloat16)
                and g.shape == bt.shape and g.numel() == B * C):
            ctx.acc = _film_acc(g)
            ctx.gshape = g.shape
        ctx.save_for_backward(ac, rc_, w, b, gf, bf, sg, sb, lens, mean, rstd)
        ctx.cfg = (B, L, C, pre_p, post_p, seed, res is not None, g is not None)
        ctx.gdtype = None if g is None else (g.dtype, bt.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        ac, rc_, w, b, gf, bf, sg, sb, lens, mean, rstd = ctx.saved_tensors
        B, L, C, pre_p, post_p, seed, has_res, has_film = ctx.cfg
        dout = dout.to(torch.bfloat16).contiguous()
        dh = torch.empty_like(ac)
        da = torch.empty_like(ac) if pre_p > 0 else None
        dw, db = gradslots.claim(w), gradslots.claim(b)  # written (not accumulated) by the fixed-order reduce
        in_slots = dw is not None and db is not None
        if dw is None:
            dw = torch.empty(C, device=ac.device, dtype=torch.float32)
        if db is None:
            db = torch.empty(C, device=ac.device, dtype=torch.float32)
        S1 = torch.empty(B, C, device=ac.device, dtype=torch.float32) if has_film else None
        S2 = torch.empty_like(S1) if has_film else None
        nws = int(lib().ssamd_addln_bwd_ws(B, L, C, int(has_film)))
        # the dw / db column sums are weight gradients: reduced on the side stream from a partials buffer
        # of their own (the shared workspace is reused by the next main-stream op) when both slots are
        # in place and single-contribution, like wgrad_async's weight-gradient GEMMs
        side = (_SIDE_WGRAD[0] and _SIDE_LN[0] and in_slots and ctx.needs_input_grad[2]
                and gradslots.single_contribution(w) and gradslots.single_contribution(b))
        ws = torch.empty(nws, device=ac.device, dtype=torch.float32) if side else _workspace(ac.device, nws)
        rc = lib().ssamd_addln_bwd(_ptr(dout), _ptr(ac), _ptr(rc_), _ptr(w), _ptr(b), _ptr(gf), _ptr(sg), _ptr(lens),
                                   _ptr(ctx.cu), _ptr(mean), _ptr(rstd), _ptr(dh), _ptr(da),
                                   None if side else _ptr(dw), _ptr(db), _ptr(S1), _ptr(S2),
                                   B, L, C, pre_p, post_p, seed, int(ctx.relu_in), 0, _ptr(ws), ws.numel(), _stream())
        _check(rc, "ssamd_addln_bwd")
        if side:
            scratch = ws[nws - 16 * 2 * C:]  # the tail of the buffer is the column-sum scratch
            p_dw, p_db = dw.data_ptr(), db.data_ptr()  # raw addresses: the closure holds no slot tensor

            def _reduce():
                _check(lib().ssamd_addln_wb_reduce(_ptr(ws), B, L, C, int(has_film), p_dw, p_db, _ptr(scratch),
                                                   _stream()), "ssamd_addln_wb_reduce")
            wgrad_async(_reduce, (ws,), True, (w, b))
        d_a = da if da is not None else dh
        d_res = dh if has_res else None
        if d_res is not None and ctx.mailbox is not None:  # the consumer GEMM adds it (GradMailbox)
            ctx.mailbox.put(d_res)
            d_res = None
        dg = dbt = dsg = dsb = None
        if has_film:  # one kernel: d gamma, d beta and the two scale gradients (into their slots)
            f32 = ctx.gdtype[0] == torch.float32
            acc = ctx.acc if (ctx.needs_input_grad[4] and ctx.needs_input_grad[5]) else None
            first = False
            if acc is not None:  # sites sharing gamma / beta: one running sum (see _FilmAcc)
                first = acc.buf is None
                if first:
                    acc.buf = torch.empty((2,) + tuple(S1.shape), device=S1.device, dtype=ctx.gdtype[0])
                dg, dbt = acc.buf[0], acc.buf[1]
                f32 = ctx.gdtype[0] == torch.float32
            else:
                dg = torch.empty(S1.shape, device=S1.device, dtype=torch.float32 if f32 else torch.bfloat16)
                dbt = torch.empty_like(dg)
            ps_g, ps_b = ctx.film_scales
            hold = gradslots.film_holder(ps_g) or gradslots.film_holder(ps_b)
            l2g = l2b = None
            if hold is not None:
                l2g, l2b = hold.entry(ps_g), hold.entry(ps_b)
            dsg = gradslots.claim(ps_g)
            dsb = gradslots.claim(ps_b)
            if dsg is None:
                dsg = torch.empty(1, device=S1.device, dtype=torch.float32)
            if dsb is None:
                dsb = torch.empty(1, device=S1.device, dtype=torch.float32)
            # per-block partials: a stream-ordered allocation of this launch (no library-global buffer two
            # streams or threads could share)
            part = torch.empty(max(1, int(lib().ssamd_film_grads_ws(S1.numel()))), device=S1.device,
                               dtype=torch.float32)
            rc = lib().ssamd_film_grads(_ptr(S1), _ptr(S2), _ptr(gf), _ptr(bf), _ptr(sg), _ptr(sb), S1.numel(),
                                        int(f32), _ptr(dg), _ptr(dbt), _ptr(dsg), _ptr(dsb),
                                        _ptr(l2g), _ptr(l2b), int(acc is not None and not first), _ptr(part),
                                        part.numel(), _stream())
            _check(rc, "ssamd_film_grads")
            if acc is not None:
                dg, dbt = (dg.view(ctx.gshape), dbt.view(ctx.gshape)) if first else (None, None)
            else:
                dg, dbt = dg.to(ctx.gdtype[0]), dbt.to(ctx.gdtype[1])
        return d_a, d_res, dw, db, dg, dbt, dsg, dsb, None, None, None, None, None, None, None, None, None


def add_layernorm(a, residual, ln_w, ln_b, *, pre_drop=0.0, post_drop=0.0, training=False, film_params=None,
                  lengths=None, eps=1e-5, pack=None, mailbox=None, relu_input=False):
    """``relu_input``: ``a`` came from ``conv1d(..., act="relu_ln")``, whose backward skips the ReLU mask: this
    LayerNorm's backward applies it (it reads ``a`` anyway).  Needs no residual and no pre-dropout."""
    C = a.shape[-1]
    if C not in (256, 512, 1024) or a.dtype != torch.bfloat16:
        if pack is not None:
            raise ValueError("packed add_layernorm needs C in (256, 512, 1024) and bf16")
        if relu_input:
            raise ValueError("add_layernorm(relu_input=True) needs the HIP kernel (C in 256/512/1024, bf16)")
        _torch_fallback(f"add_layernorm C={C} dtype={a.dtype} (kernel: C in 256/512/1024, bf16)")
        return ref.add_layernorm(a, residual, ln_w, ln_b, pre_drop=pre_drop, post_drop=post_drop, training=training,
                                 film_params=film_params, lengths=lengths, eps=eps)
    if not training:
        pre_drop = post_drop = 0.0
    g = bt = sg = sb = None
    if film_params is not None:
        g, bt, sg, sb = film_params
    cu = geom = None
    if pack is not None:
        assert a.shape[0] == 1 and a.shape[1] == pack.R, "packed add_layernorm expects [1, R, C]"
        lens, cu, geom = pack.lens, pack.cu, (pack.B, pack.M, C)
    else:
        lens = None if lengths is None else lengths.to(torch.int64).contiguous()
    if residual is not None:
        residual = residual.to(a.dtype)
    if relu_input and (residual is not None or pre_drop > 0):
        raise ValueError("add_layernorm(relu_input=True) needs no residual and no pre-dropout")
    out = _AddLNFn.apply(a, residual, ln_w, ln_b, g, bt, sg, sb, lens, float(pre_drop), float(post_drop),
                         _next_seed(), float(eps), cu, geom, mailbox, bool(relu_input))
    return out


_SIGS["ssamd_gemm_addln"] = [P, P, P, P, P, P, P, P, P, P, P, P, I, I, L_, I, P, F, P]
# Off (0): measured slower at batch 1 -- 1.82 / 1.83 ms vs 1.74 / 1.74 ms with skinny GEMM + add_layernorm
# (profiles/r6_b1_latency.txt): one block owns whole rows, so a 14-row encoder step streams the whole weight through
# ONE CU, where the skinny GEMM spreads it over 16-64.  Kept for A/B (bench_synth --gemm-addln-rows) and tested.
GEMM_ADDLN_MAX_ROWS = 0


def gemm_addln(x, w, b, residual, ln_w, ln_b, *, film_params=None, lengths=None, pack=None, eps=1e-5):
    """Inference LN(x W^T + b + residual) (+ FiLM, pad mask) in ONE kernel (``ssamd_gemm_addln``) for C = 256 and
    <= GEMM_ADDLN_MAX_ROWS rows; returns None when the shapes do not qualify (the caller runs linear +
    add_layernorm).  ``w``: Linear [256, K] or Conv1d [256, K, 1]."""
    C = w.shape[0]
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    if (C != 256 or K % 32 or rows > GEMM_ADDLN_MAX_ROWS or (w.dim() == 3 and w.shape[2] != 1)
            or residual is None or tuple(residual.shape) != tuple(x.shape[:-1]) + (C,) or x.dim() != 3
            or not has("ssamd_gemm_addln")):
        return None
    B, L = x.shape[0], x.shape[1]
    xc = x.to(torch.bfloat16).contiguous()
    res = residual.to(torch.bfloat16).contiguous()
    wi = weight_fwd(w)
    bf = None if b is None else b.detach().float().contiguous()
    g = bt = sg = sb = None
    if film_params is not None:
        g, bt, sg, sb = film_params
        g, bt = _f32_view(g), _f32_view(bt)  # the style's gamma / beta may be bf16 or column views
    cu = None
    if pack is not None:
        assert B == 1 and L == pack.R, "packed gemm_addln expects [1, R, K]"
        lens, cu, nb = pack.lens, pack.cu, pack.B
    else:
        lens = None if lengths is None else lengths.to(torch.int64).contiguous()
        nb = B
    out = torch.empty(B, L, C, device=x.device, dtype=torch.bfloat16)
    rc = lib().ssamd_gemm_addln(_ptr(xc), _ptr(wi), _ptr(bf), _ptr(res), _ptr(ln_w), _ptr(ln_b), _ptr(g), _ptr(bt),
                                _ptr(sg), _ptr(sb), _ptr(lens), _ptr(cu), nb, L, rows, K, _ptr(out), float(eps),
                                _stream())
    _check(rc, "ssamd_gemm_addln")
    return out


def _ln_bwd_strided(dout, a, a_off, lda, w, b, mean, rstd, dh, dh_off, B, L, C, post_p, seed, relu_in):
    """One LayerNorm backward over a column slice (row stride ``lda``) of ``a`` / ``dh``: the dense dout,
    no residual / pre-dropout / FiLM / mask.  -> (dw, db), written into the parameters' arena slots when
    claimable (reduced on the side stream when both are single-contribution, as in _AddLNFn)."""
    dw, db = gradslots.claim(w), gradslots.claim(b)
    in_slots = dw is not None and db is not None
    if dw is None:
        dw = torch.empty(C, device=dout.device, dtype=torch.float32)
    if db is None:
        db = torch.empty(C, device=dout.device, dtype=torch.float32)
    nws = int(lib().ssamd_addln_bwd_ws(B, L, C, 0))
    side = (_SIDE_WGRAD[0] and _SIDE_LN[0] and in_slots and gradslots.single_contribution(w)
            and gradslots.single_contribution(b))
    ws = torch.empty(nws, device=dout.device, dtype=torch.float32) if side else _workspace(dout.device, nws)
    rc = lib().ssamd_addln_bwd(_ptr(dout), _ptr(a) + 2 * a_off, None, _ptr(w), _ptr(b), None, None, None, None,
                               _ptr(mean), _ptr(rstd), _ptr(dh) + 2 * dh_off, None, None if side else _ptr(dw),
                               _ptr(db), None, None, B, L, C, 0.0, post_p, seed, int(relu_in), lda, _ptr(ws),
                               ws.numel(), _stream())
    _check(rc, "ssamd_addln_bwd")
    if side:
        scratch = ws[nws - 16 * 2 * C:]
        p_dw, p_db = dw.data_ptr(), db.data_ptr()

        def _reduce():
            _check(lib().ssamd_addln_wb_reduce(_ptr(ws), B, L, C, 0, p_dw, p_db, _ptr(scratch), _stream()),
                   "ssamd_addln_wb_reduce")
        wgrad_async(_reduce, (ws,), True, (w, b))
    return dw, db


class _DualConvReluLNFn(torch.autograd.Function):
    """Two variance predictors' first blocks on the SAME input (duration and pitch, reference
    ``model/modules.py:121-125``): [conv k -> ReLU -> LayerNorm -> dropout] x 2 as ONE
    N = 2C implicit-GEMM conv (the two weights are adjacent in the flat arena, so the fused [2C, Cin, k]
    weight and its gradient are views), two LayerNorms over the column halves of its output (row stride
    2C), and in the backward the two LayerNorm backwards write the halves of one [M, 2C] gradient, which
    feeds ONE data-gradient GEMM (K = k * 2C: the two predictors' contributions to dx summed inside it)
    and ONE weight-gradient GEMM (N = 2C, fused bias gradient) into the fused slots.  The ReLU mask of the
    conv is applied by the LayerNorm backwards (they read its output anyway)."""

    @staticmethod
    def forward(ctx, x, wf, bf, pad, dil, post_p, w_d, w_p, b_d, b_p, lw_d, lb_d, lw_p, lb_p):
        B, L, Cin = x.shape
        N2, _, ks = wf.shape
        C = N2 // 2
        xc = x.contiguous()
        h = conv_gemm_raw(xc, weight_fwd(wf, owner=w_d), bf, B, L, Cin, ks, dil, pad, N2, _ACT["relu_ln"])
        outs, stats, seeds = [], [], []
        for half, (lw, lb) in enumerate(((lw_d, lb_d), (lw_p, lb_p))):
            out = torch.empty(B, L, C, device=x.device, dtype=torch.bfloat16)
            mean = torch.empty(B * L, device=x.device, dtype=torch.float32)
            rstd = torch.empty_like(mean)
            seed = _next_seed()
            rc = lib().ssamd_addln_fwd(_ptr(h) + 2 * half * C, None, _ptr(lw), _ptr(lb), None, None, None, None,
                                       None, None, _ptr(out), _ptr(mean), _ptr(rstd), B, L, C, 0.0, post_p, seed,
                                       1e-5, N2, _stream())
            _check(rc, "ssamd_addln_fwd")
            outs.append(out)
            stats += [mean, rstd]
            seeds.append(seed)
        ctx.save_for_backward(xc, h, wf, *stats)
        ctx.members = (w_d, w_p, b_d, b_p, lw_d, lb_d, lw_p, lb_p)
        ctx.cfg = (B, L, Cin, C, ks, pad, dil, post_p, tuple(seeds))
        return tuple(outs)

    @staticmethod
    def backward(ctx, g_d, g_p):
        xc, h, wf, m_d, r_d, m_p, r_p = ctx.saved_tensors
        w_d, w_p, b_d, b_p, lw_d, lb_d, lw_p, lb_p = ctx.members
        B, L, Cin, C, ks, pad, dil, post_p, seeds = ctx.cfg
        N2 = 2 * C
        dh = torch.empty(B, L, N2, device=xc.device, dtype=torch.bfloat16)
        lngrads = []
        for half, (g, lw, lb, mean, rstd) in enumerate(((g_d, lw_d, lb_d, m_d, r_d), (g_p, lw_p, lb_p, m_p, r_p))):
            if g is None:
                g = torch.zeros(B, L, C, device=xc.device, dtype=torch.bfloat16)
            gc = g.to(torch.bfloat16).contiguous()
            lngrads += _ln_bwd_strided(gc, h, half * C, N2, lw, lb, mean, rstd, dh, half * C, B, L, C, post_p,
                                       seeds[half], True)
        first = _wgrad_first(B * L)
        if not first:
            dx = conv_gemm_raw(dh, weight_dgrad(wf, owner=w_d), None, B, L, N2, ks, dil, (ks - 1) * dil - pad, Cin)
        ws_, bs_ = (w_d, w_p), (b_d, b_p)
        sw, sb = gradslots.claim_fused(ws_), gradslots.claim_fused(bs_)
        dw, db = wgrad_async(lambda: conv_wgrad_raw(xc, dh, B, L, Cin, ks, dil, pad, N2, with_bias=True,
                                                    dW=sw, db=sb),
                             (xc, dh), sw is not None and sb is not None, ws_ + bs_)
        if first:
            dx = conv_gemm_raw(dh, weight_dgrad(wf, owner=w_d), None, B, L, N2, ks, dil, (ks - 1) * dil - pad, Cin)
        return (dx, None, None, None, None, None, *gradslots.split_rows(dw, ws_), *gradslots.split_rows(db, bs_),
                *lngrads)


def dual_conv_relu_layernorm(x, ws, bs, pad, dil, lns, post_p):
    """(LN_d(ReLU(conv_d(x))), LN_p(ReLU(conv_p(x)))) with post-dropout ``post_p`` (0 in eval): one N = 2C
    GEMM each way when the two conv weights / biases are adjacent in the arena (``_DualConvReluLNFn``);
    otherwise None (the caller runs the two blocks separately)."""
    wf, bf = gradslots.fused_data(list(ws)), gradslots.fused_data(list(bs))
    C = ws[0].shape[0]
    if (wf is None or bf is None or x.dtype != torch.bfloat16 or C not in (256, 512, 1024) or ws[1].shape[0] != C
            or x.shape[-1] % 8):
        return None
    (lw_d, lb_d), (lw_p, lb_p) = lns
    return _DualConvReluLNFn.apply(x, wf, bf, pad, dil, float(post_p), ws[0], ws[1], bs[0], bs[1], lw_d, lb_d,
                                   lw_p, lb_p)


# ------------------------------------------------------------------------ length regulator
class _LRFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dur, M, pe):
        B, T, C = x.shape
        xc = x.contiguous()
        out = torch.empty(B, M, C, device=x.device, dtype=x.dtype)
        pe_c = None if pe is None else pe.to(x.dtype).contiguous()
        if pe_c is not None:
            assert pe_c.shape[0] >= M and pe_c.shape[1] == C
        rc = lib().ssamd_lr_fwd(_ptr(xc), _ptr(dur), _ptr(pe_c), _ptr(out), None, None, B, T, M, C, _stream())
        _check(rc, "ssamd_lr_fwd")
        ctx.save_for_backward(dur)
        ctx.dims = (B, T, M, C)
        return out

    @staticmethod
    def backward(ctx, dout):
        (dur,) = ctx.saved_tensors
        B, T, M, C = ctx.dims
        dout = dout.to(torch.bfloat16).contiguous()
        dx = torch.empty(B, T, C, device=dout.device, dtype=torch.bfloat16)
        rc = lib().ssamd_lr_bwd(_ptr(dout), _ptr(dur), _ptr(dx), None, None, B, T, M, C, _stream())
        _check(rc, "ssamd_lr_bwd")
        return dx, None, None, None


def length_regulate(x, durations, max_len, pe=None, mel_len=None):
    """``mel_len``: the row sums of ``durations`` when the caller already has them (duration_round)."""
    if x.dtype != torch.bfloat16 or x.shape[-1] % 8:
        _torch_fallback(f"length_regulate C={x.shape[-1]} dtype={x.dtype} (kernel: bf16, C % 8 == 0)")
        out, ml = ref.length_regulate(x, durations, max_len)
        return (out + pe[: out.shape[1]].to(out.dtype) if pe is not None else out), ml
    dur = durations.to(torch.int64).contiguous()
    if mel_len is None:
        mel_len = dur.clamp(min=0).sum(1)
    if max_len is None:
        max_len = int(mel_len.max().item()) if dur.shape[0] else 0  # inference: one D2H for allocation
    return _LRFn.apply(x, dur, int(max_len), pe), mel_len


class _LRPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dur, pe, cu, plen, R, M):
        B, T, C = x.shape
        xc = x.contiguous()
        out = torch.empty(1, R, C, device=x.device, dtype=x.dtype)
        pe_c = pe.to(x.dtype).contiguous()
        assert pe_c.shape[0] >= M and pe_c.shape[1] == C
        rc = lib().ssamd_lr_fwd(_ptr(xc), _ptr(dur), _ptr(pe_c), _ptr(out), _ptr(cu), _ptr(plen), B, T, M, C,
                                _stream())
        _check(rc, "ssamd_lr_fwd(packed)")
        ctx.save_for_backward(dur, cu, plen)
        ctx.dims = (B, T, M, C)
        return out

    @staticmethod
    def backward(ctx, dout):
        dur, cu, plen = ctx.saved_tensors
        B, T, M, C = ctx.dims
        dout = dout.to(torch.bfloat16).contiguous()
        dx = torch.empty(B, T, C, device=dout.device, dtype=torch.bfloat16)
        rc = lib().ssamd_lr_bwd(_ptr(dout), _ptr(dur), _ptr(dx), _ptr(cu), _ptr(plen), B, T, M, C, _stream())
        _check(rc, "ssamd_lr_bwd(packed)")
        return dx, None, None, None, None, None, None


def length_regulate_packed(x, durations, pack, pe):
    if x.dtype != torch.bfloat16 or x.shape[-1] % 8:
        raise ValueError("packed length regulator needs bf16 and C % 8 == 0")
    dur = durations.to(torch.int64).contiguous()
    return _LRPackedFn.apply(x, dur, pe, pack.cu, pack.lens, pack.R, pack.M)


def pack_info(lens, M, cu, rinfo, dst):
    _need(lens, torch.int64, "pack.lens")
    rc = lib().ssamd_pack_info(_ptr(lens), lens.numel(), int(M), _ptr(cu), _ptr(rinfo), _ptr(dst), _stream())
    _check(rc, "ssamd_pack_info")


# ------------------------------------------------------------------------ embeddings
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mode, ids, vals, bins, table, addend, L):
        C = table.shape[1]
        rows = (ids if mode == 0 else vals).numel()
        out_shape = (*((ids if mode == 0 else vals).shape), C)
        out = torch.empty(out_shape, device=table.device, dtype=torch.bfloat16)
        idx = torch.empty(rows, device=table.device, dtype=torch.int32)
        # fp32 parameter: its cached bf16 image (refreshed with every other weight image after the
        # optimizer step), and the gradient goes straight into the parameter's arena slot
        tb = weight_fwd(table) if (isinstance(table, torch.nn.Parameter) and _eligible(table)) \
            else table.to(torch.bfloat16).contiguous()
        ad = addend.to(torch.bfloat16).contiguous()
        rc = lib().ssamd_embed_fwd(mode, _ptr(ids), _ptr(vals), _ptr(bins), 0 if bins is None else bins.numel(),
                                   _ptr(tb), _ptr(ad), L, _ptr(out), _ptr(idx), rows, C, _stream())
        _check(rc, "ssamd_embed_fwd")
        ctx.save_for_backward(idx)
        ctx.table = table if isinstance(table, torch.nn.Parameter) else None
        ctx.tshape = (table.shape, table.dtype)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        shape, dtype = ctx.tshape
        dout = dout.to(torch.bfloat16).contiguous()
        dt = gradslots.claim(ctx.table) if ctx.needs_input_grad[4] else None
        if dt is None:
            dt = torch.empty(shape, device=dout.device, dtype=torch.float32)
        V, C = shape[0], shape[1]
        rows = idx.numel()
        if C % 8 == 0 and rows > 0:
            # dtable = onehot(idx)^T @ dout on the MFMA weight-gradient GEMM (deterministic split-M reduce)
            Vp = (V + 7) // 8 * 8
            oh = torch.empty(rows, Vp, device=dout.device, dtype=torch.bfloat16)
            rc = lib().ssamd_onehot(_ptr(idx), rows, Vp, _ptr(oh), _stream())
            _check(rc, "ssamd_onehot")
            if Vp == V:
                conv_wgrad_raw(dout.view(1, rows, C), oh.view(1, rows, Vp), 1, rows, C, 1, 1, 0, Vp,
                               dW=dt.view(V, C, 1))
            else:
                dt.copy_(conv_wgrad_raw(dout.view(1, rows, C), oh.view(1, rows, Vp), 1, rows, C, 1, 1, 0, Vp)
                         .view(Vp, C)[:V])
        else:  # one block per table row, fixed summation order (deterministic; every row is written)
            rc = lib().ssamd_embed_bwd(_ptr(idx), _ptr(dout), _ptr(dt), rows, C, V, _stream())
            _check(rc, "ssamd_embed_bwd")
        d_add = dout if ctx.mode == 1 else None
        return None, None, None, None, dt if dtype == torch.float32 else dt.to(dtype), d_add, None


def embed_add_pe(ids, table, pe, extra=None):
    B, L = ids.shape
    out = _EmbedFn.apply(0, ids.contiguous(), None, None, table, pe[:L].contiguous(), L)
    if extra is not None:
        out = out + extra.unsqueeze(1).to(out.dtype)
    return out


def bucketize_embed_add(x, values, bins, table):
    return _EmbedFn.apply(1, None, values.float().contiguous(), bins.float().contiguous(), table, x, 0)


# ------------------------------------------------------------------------ attention
def attention(qkv, lengths, n_head, pack=None):
    if pack is not None:
        assert qkv.shape[0] == 1 and qkv.shape[1] == pack.R, "packed attention expects [1, R, 3C]"
        return _AttnFn.apply(qkv, pack.lens, n_head, pack.cu, (pack.B, pack.M))
    return _AttnFn.apply(qkv, lengths.to(torch.int64).contiguous(), n_head, None, None)


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, lens, n_head, cu, geom):
        rows = qkv.shape[0] * qkv.shape[1]
        C3 = qkv.shape[2]
        B, L = (qkv.shape[0], qkv.shape[1]) if geom is None else geom
        D = C3 // (3 * n_head)
        if D not in (32, 64, 128):
            raise ValueError("attention head dim must be 32/64/128")
        q = qkv.contiguous()
        o = torch.empty(*qkv.shape[:2], n_head * D, device=q.device, dtype=torch.bfloat16)
        lse = torch.empty(B, n_head, L, device=q.device, dtype=torch.float32)
        rc = lib().ssamd_attn_fwd(_ptr(q), _ptr(lens), _ptr(cu), _ptr(o), _ptr(lse), B, L, n_head, D,
                                  1.0 / math.sqrt(D), _stream())
        _check(rc, "ssamd_attn_fwd")
        ctx.save_for_backward(q, lens, o, lse)
        ctx.cu = cu
        ctx.dims = (B, L, n_head, D, rows)
        return o

    @staticmethod
    def backward(ctx, do):
        q, lens, o, lse = ctx.saved_tensors
        B, L, H, D, rows = ctx.dims
        do = do.to(torch.bfloat16).contiguous()
        dqkv = torch.empty_like(q)
        delta = torch.empty(rows * H, device=q.device, dtype=torch.float32)
        rc = lib().ssamd_attn_bwd(_ptr(q), _ptr(lens), _ptr(ctx.cu), _ptr(o), _ptr(lse), _ptr(do), _ptr(dqkv),
                                  _ptr(delta), rows, B, L, H, D, 1.0 / math.sqrt(D), _stream())
        _check(rc, "ssamd_attn_bwd")
        return dqkv, None, None, None, None


# ------------------------------------------------------------------------ loss / optimizer
class _L1PairFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p1, p2, tgt, lens, count):
        B, M, C = p1.shape
        Mt = tgt.shape[1]
        p1c, p2c, tc = p1.float().contiguous(), p2.float().contiguous(), tgt.float().contiguous()
        sums = torch.empty(2, device=p1.device, dtype=torch.float32)
        ws = _workspace(p1.device, int(lib().ssamd_l1pair_ws(B, M, C)))
        rc = lib().ssamd_l1pair_fwd(_ptr(p1c), _ptr(p2c), _ptr(tc), _ptr(lens), B, M, Mt, C, _ptr(sums), _ptr(ws),
                                    ws.numel(), _stream())
        _check(rc, "ssamd_l1pair_fwd")
        cnt = count.float().reshape(1).contiguous()
        ctx.save_for_backward(p1c, p2c, tc, lens, cnt)
        res = sums / cnt.clamp(min=1)
        return res[0], res[1]

    @staticmethod
    def backward(ctx, g1, g2):
        p1c, p2c, tc, lens, cnt = ctx.saved_tensors
        B, M, C = p1c.shape
        gs = torch.stack([g1.reshape(()), g2.reshape(())]).float().contiguous()
        d1 = torch.empty_like(p1c)
        d2 = torch.empty_like(p2c)
        rc = lib().ssamd_l1pair_bwd(_ptr(p1c), _ptr(p2c), _ptr(tc), _ptr(lens), B, M, tc.shape[1], C, _ptr(gs),
                                    _ptr(cnt), _ptr(d1), _ptr(d2), _stream())
        _check(rc, "ssamd_l1pair_bwd")
        return d1, d2, None, None, None


class VTerm(ctypes.Structure):
    _fields_ = [("pred", P), ("tgt", P), ("mask", P), ("grad", P), ("L", I), ("ldp", I), ("ldt", I), ("dur", I)]


_SIGS.update({"ssamd_var_loss_fwd": [VTerm, VTerm, VTerm, I, P, P, P, P, P],
              "ssamd_var_loss_bwd": [VTerm, VTerm, VTerm, I, P, P, P],
              "ssamd_var_loss_ws": []})
_RESTYPES["ssamd_var_loss_ws"] = L_


def _vterm(pred, tgt, mask, grad=None):
    B, L = mask.shape
    _need(pred, torch.float32, "var_loss.pred")
    _need(mask, torch.bool, "var_loss.mask")
    dur = tgt.dtype == torch.int64
    if not dur:
        _need(tgt, torch.float32, "var_loss.target")
    assert pred.dim() == 2 and tgt.dim() == 2 and pred.shape[0] == tgt.shape[0] == B
    assert pred.shape[1] >= L and tgt.shape[1] >= L and tgt.stride(1) == 1, "var_loss: operand shapes"
    return VTerm(pred.data_ptr(), tgt.data_ptr(), mask.data_ptr(), 0 if grad is None else grad.data_ptr(), L,
                 pred.stride(0), tgt.stride(0), int(dur))


class _VarLossFn(torch.autograd.Function):
    """pitch / energy / log-duration masked MSE (reference ``model/loss.py:76-89``) in one fused,
    deterministic kernel pair; ``counts`` (3 fp32, optional): the all-reduced global divisors."""

    @staticmethod
    def forward(ctx, pp, pt, pm, ep, et, em, ld, dt, dm, counts):
        tensors = [t.contiguous() for t in (pp, pt, ep, et, ld, dt)]
        pp, pt, ep, et, ld, dt = tensors
        pm, em, dm = pm.contiguous(), em.contiguous(), dm.contiguous()
        B = pm.shape[0]
        loss = torch.empty(3, device=pp.device, dtype=torch.float32)
        cnt = torch.empty(3, device=pp.device, dtype=torch.float32)
        ws = _workspace(pp.device, int(lib().ssamd_var_loss_ws()))
        ext = None if counts is None else counts.float().contiguous()
        rc = lib().ssamd_var_loss_fwd(_vterm(pp, pt, pm), _vterm(ep, et, em), _vterm(ld, dt, dm), B, _ptr(ext),
                                      _ptr(loss), _ptr(cnt), _ptr(ws), _stream())
        _check(rc, "ssamd_var_loss_fwd")
        ctx.save_for_backward(pp, pt, pm, ep, et, em, ld, dt, dm, cnt)
        return loss[0], loss[1], loss[2]

    @staticmethod
    def backward(ctx, g0, g1, g2):
        pp, pt, pm, ep, et, em, ld, dt, dm, cnt = ctx.saved_tensors
        gs = torch.stack([g.reshape(()) for g in (g0, g1, g2)]).float().contiguous()
        # columns past the mask width (frame-level preds longer than the truncated mel) get no gradient
        gp, ge, gd = [torch.empty_like(x) if x.shape[1] == m.shape[1] else torch.zeros_like(x)
                      for x, m in ((pp, pm), (ep, em), (ld, dm))]
        rc = lib().ssamd_var_loss_bwd(_vterm(pp, pt, pm, gp), _vterm(ep, et, em, ge), _vterm(ld, dt, dm, gd),
                                      pm.shape[0], _ptr(gs), _ptr(cnt), _stream())
        _check(rc, "ssamd_var_loss_bwd")
        return gp, None, None, ge, None, None, gd, None, None, None


def variance_losses(p_pred, p_t, p_mask, e_pred, e_t, e_mask, logd, d_t, src_mask, counts=None):
    """-> (pitch, energy, duration) losses; masks are the reference's pad masks (True = padded)."""
    return _VarLossFn.apply(p_pred.float(), p_t.float(), p_mask, e_pred.float(), e_t.float(), e_mask,
                            logd.float(), d_t.to(torch.int64), src_mask, counts)


_SIGS["ssamd_fs2_loss_final"] = [P, P, P, I, I, I, P, P, P, P]


class _FS2LossFn(torch.autograd.Function):
    """All five FastSpeech2 loss terms and their total in ONE autograd node: masked L1 of mel and
    postnet (``l1pair``), masked MSE of pitch / energy / log-duration (``var_loss``), and a one-block
    finalize kernel (mel count from the lengths, divisions, total in the reference's order) --
    instead of ~15 small torch ops (masks, counts, casts, divisions, adds) on the host-paced loss
    path.  Backward: per-term scale = g_term + g_total, then the two fused gradient kernels."""

    @staticmethod
    def forward(ctx, mel_p, post_p, mel_t, lens, mel_count, pp, pt, pm, ep, et, em, ld, dt, dm, var_counts):
        B, M, C = mel_p.shape
        Mt = mel_t.shape[1]
        p1c, p2c, tc = mel_p.float().contiguous(), post_p.float().contiguous(), mel_t.float().contiguous()
        lens = lens.contiguous()
        dev = mel_p.device
        sums = torch.empty(2, device=dev, dtype=torch.float32)
        ws = _workspace(dev, int(lib().ssamd_l1pair_ws(B, M, C)))
        rc = lib().ssamd_l1pair_fwd(_ptr(p1c), _ptr(p2c), _ptr(tc), _ptr(lens), B, M, Mt, C, _ptr(sums), _ptr(ws),
                                    ws.numel(), _stream())
        _check(rc, "ssamd_l1pair_fwd")
        pp, pt, ep, et, ld, dt = [t.contiguous() for t in (pp, pt, ep, et, ld, dt)]
        pm, em, dm = pm.contiguous(), em.contiguous(), dm.contiguous()
        var3 = torch.empty(3, device=dev, dtype=torch.float32)
        vcnt = torch.empty(3, device=dev, dtype=torch.float32)
        vws = _workspace(dev, int(lib().ssamd_var_loss_ws()))  # stream-ordered after l1pair: reuse is safe
        ext = None if var_counts is None else var_counts.float().contiguous()
        rc = lib().ssamd_var_loss_fwd(_vterm(pp, pt, pm), _vterm(ep, et, em), _vterm(ld, dt, dm), B, _ptr(ext),
                                      _ptr(var3), _ptr(vcnt), _ptr(vws), _stream())
        _check(rc, "ssamd_var_loss_fwd")
        out = torch.empty(6, device=dev, dtype=torch.float32)
        mcnt = torch.empty(1, device=dev, dtype=torch.float32)
        mext = None if mel_count is None else mel_count.float().reshape(1).contiguous()
        rc = lib().ssamd_fs2_loss_final(_ptr(sums), _ptr(var3), _ptr(lens), B, M, C, _ptr(mext), _ptr(out),
                                        _ptr(mcnt), _stream())
        _check(rc, "ssamd_fs2_loss_final")
        ctx.save_for_backward(p1c, p2c, tc, lens, mcnt, pp, pt, pm, ep, et, em, ld, dt, dm, vcnt)
        return out[0], out[1], out[2], out[3], out[4], out[5]

    @staticmethod
    def backward(ctx, g_tot, g_mel, g_post, g_pitch, g_energy, g_dur):
        p1c, p2c, tc, lens, mcnt, pp, pt, pm, ep, et, em, ld, dt, dm, vcnt = ctx.saved_tensors
        B, M, C = p1c.shape
        gs = (torch.stack([g_mel, g_post, g_pitch, g_energy, g_dur]).float() + g_tot.float()).contiguous()
        d1 = torch.empty_like(p1c)
        d2 = torch.empty_like(p2c)
        rc = lib().ssamd_l1pair_bwd(_ptr(p1c), _ptr(p2c), _ptr(tc), _ptr(lens), B, M, tc.shape[1], C, _ptr(gs),
                                    _ptr(mcnt), _ptr(d1), _ptr(d2), _stream())
        _check(rc, "ssamd_l1pair_bwd")
        gp, ge, gd = [torch.empty_like(x) if x.shape[1] == m.shape[1] else torch.zeros_like(x)
                      for x, m in ((pp, pm), (ep, em), (ld, dm))]
        rc = lib().ssamd_var_loss_bwd(_vterm(pp, pt, pm, gp), _vterm(ep, et, em, ge), _vterm(ld, dt, dm, gd),
                                      pm.shape[0], ctypes.c_void_p(gs.data_ptr() + 2 * 4), _ptr(vcnt), _stream())
        _check(rc, "ssamd_var_loss_bwd")
        return d1, d2, None, None, None, gp, None, None, ge, None, None, gd, None, None, None


def fs2_losses(mel_p, post_p, mel_t, mel_lens, p_pred, p_t, p_mask, e_pred, e_t, e_mask, logd, d_t, src_mask,
               mel_count=None, var_counts=None):
    """-> (total, mel, postnet, pitch, energy, duration) losses; ``mel_lens`` (int64 [B], may exceed
    the truncated length M) replaces the mel pad mask; masks are the reference's (True = padded);
    ``mel_count`` / ``var_counts``: optional all-reduced global divisors (data parallelism)."""
    return _FS2LossFn.apply(mel_p, post_p, mel_t, mel_lens.to(torch.int64), mel_count, p_pred.float(), p_t.float(),
                            p_mask, e_pred.float(), e_t.float(), e_mask, logd.float(), d_t.to(torch.int64),
                            src_mask, var_counts)


def masked_l1_pair(mel_p, post_p, mel_t, mel_valid, count):
    lens = mel_valid.sum(1).to(torch.int64).contiguous()
    return _L1PairFn.apply(mel_p, post_p, mel_t, lens, count)


_adam_ws = {}


_adam_plan = {}
_adam_plan_builds = [0]  # diagnostics: plan (re)builds


def _adam_image_plan(p: torch.Tensor):
    """Fused clip+Adam+image plan for the arena ``p``: the cached weight images whose source lies
    in the arena (grouped per weight: forward and/or dgrad image), their 64x64 tiles, and the
    arena ranges NOT covered by an image-bearing weight (updated element-wise).  Rebuilt when
    the image set changes (``_wepoch``)."""
    key = (p.data_ptr(), p.numel())
    plan = _adam_plan.get(key)
    if plan is not None and plan["epoch"] == _wepoch:
        return plan
    import numpy as np

    base, n = p.data_ptr(), p.numel()
    weights = {}  # src ptr -> [off, cout, cin, ks, fwd_dst, dgrad_dst, entries]
    for k, e in list(_wcache.items()):
        owner, w = e[2](), e[7]
        if owner is None or w.data_ptr() != e[5] or w.device != p.device or not _eligible(w):
            continue
        sp = w.data_ptr()
        if not (base <= sp and sp + w.numel() * 4 <= base + n * 4):
            continue
        ks = w.shape[2] if w.dim() == 3 else 1
        rec = weights.setdefault(sp, [(sp - base) // 4, w.shape[0], w.shape[1], ks, 0, 0, []])
        rec[4 + e[4]] = e[3].data_ptr()
        rec[6].append(k)
    recs = sorted(weights.values(), key=lambda r: r[0])
    # an element must be updated exactly once: weights whose ranges overlap another image source
    # (e.g. a fused view and one of its members) stay on the element-wise path + lazy refresh
    span = [(r[0], r[0] + r[1] * r[2] * r[3]) for r in recs]
    clash = [any(j != i and span[j][0] < b and a < span[j][1] for j in range(len(span))) for i, (a, b) in
             enumerate(span)]
    recs = [r for r, c in zip(recs, clash) if not c]
    desc = np.zeros(len(recs), dtype=[("off", "<i8"), ("fwd", "<u8"), ("dgrad", "<u8"), ("cout", "<i4"),
                                      ("cin", "<i4"), ("ks", "<i4"), ("pad", "<i4")])
    tiles, covered = [], []
    for i, (off, cout, cin, ks, fwd, dgr, _) in enumerate(recs):
        desc[i] = (off, fwd, dgr, cout, cin, ks, 0)
        K = cin * ks
        covered.append((off, off + cout * K))
        for co0 in range(0, cout, 64):
            for j0 in range(0, K, 64):
                tiles.append((i, co0, j0, 0))
    rest, cur = [], 0
    for a, b in covered:  # sorted, disjoint (distinct parameters)
        if a > cur:
            rest.append((cur, a))
        cur = max(cur, b)
    if cur < n:
        rest.append((cur, n))
    rstart = np.array([a for a, _ in rest] or [0], dtype=np.int64)
    rcum = np.zeros(len(rest) + 1, dtype=np.int64)
    rcum[1:] = np.cumsum([b - a for a, b in rest]) if rest else 0
    dev = p.device
    tiles = np.asarray(tiles, dtype=np.int32).reshape(-1, 4)
    plan = {
        "epoch": _wepoch,
        "desc": torch.from_numpy(desc.view(np.uint8).copy()).to(dev) if len(recs) else None,
        "tiles": torch.from_numpy(tiles).to(dev) if len(tiles) else None, "ntiles": len(tiles),
        "rcum": torch.from_numpy(rcum).to(dev), "rstart": torch.from_numpy(rstart).to(dev),
        "nr": len(rest), "rtotal": int(rcum[-1]),
        "keys": [k for r in recs for k in r[6]],
        # the cache entry lists themselves (an entry replaced in _wcache bumps _wepoch -> new plan)
        "entries": [_wcache[k] for r in recs for k in r[6]],
    }
    _adam_plan[key] = plan
    _adam_plan_builds[0] += 1
    return plan


def clip_adam_step(p, g, m, v, lr, betas, eps, wd, step, clip, norm_out, skipped, images=True):
    """Global-norm clip + Adam over the flat arena (no host sync).  ``images``: the same launch
    rewrites the bf16 operand images of every cached weight inside the arena (no separate
    ``weight_prep`` refresh before the next forward); the caller still bumps the generation."""
    for t, nm in ((p, "p"), (g, "g"), (m, "m"), (v, "v")):
        _need(t, torch.float32, "adam." + nm)
    assert p.numel() == g.numel() == m.numel() == v.numel()
    n_ws = int(lib().ssamd_clip_adam_ws(p.numel()))
    ws = _adam_ws.get(p.device)
    if ws is None or ws.numel() < n_ws:  # [global sum of squares, per-block partials]
        ws = _adam_ws[p.device] = torch.zeros(n_ws, device=p.device, dtype=torch.float32)
    if images and has("ssamd_clip_adam_img"):
        plan = _adam_image_plan(p)
        rc = lib().ssamd_clip_adam_img(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(ws), float(clip),
                                       float(lr), float(betas[0]), float(betas[1]), float(eps), float(wd), int(step),
                                       _ptr(norm_out), _ptr(skipped), _ptr(plan["desc"]), _ptr(plan["tiles"]),
                                       plan["ntiles"], _ptr(plan["rcum"]), _ptr(plan["rstart"]), plan["nr"],
                                       plan["rtotal"], _stream())
        _check(rc, "ssamd_clip_adam_img")
        return plan["entries"]
    rc = lib().ssamd_clip_adam(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(ws), float(clip), float(lr),
                               float(betas[0]), float(betas[1]), float(eps), float(wd), int(step), _ptr(norm_out),
                               _ptr(skipped), _stream())
    _check(rc, "ssamd_clip_adam")
    return []


def stamp_images(entries):
    """Mark the given cached image entries current (their fused-Adam rewrite is already queued)."""
    g = _wgen
    for e in entries:
        owner = e[2]()
        if owner is not None:
            e[0], e[1] = owner._version, g


# ------------------------------------------------------------------------ multi-tensor copy
_SIGS["ssamd_multi_copy"] = [I] + [P, P, L_] * 6 + [P]


def multi_copy(pairs) -> bool:
    """dst.copy_(src) for up to 6 (dst, src) pairs of contiguous same-size device tensors in ONE launch (the HIP-graph
    replays' static-input refresh, ``infer/graphs.py``).  Returns False (nothing done) when the pairs do not qualify:
    the caller copies them one by one."""
    if not pairs or len(pairs) > 6 or not has("ssamd_multi_copy"):
        return False
    args = []
    for d, s in pairs:
        if not (d.is_cuda and s.is_cuda and d.device == s.device and d.is_contiguous() and s.is_contiguous()
                and d.dtype == s.dtype and d.numel() == s.numel()):
            return False
        args += [_ptr(s), _ptr(d), d.numel() * d.element_size()]
    args += [None, None, 0] * (6 - len(pairs))
    _check(lib().ssamd_multi_copy(len(pairs), *args, _stream()), "ssamd_multi_copy")
    return True


# ------------------------------------------------------------------------ BatchNorm (+tanh, dropout)
_SIGS.update({
    "ssamd_bn_fwd": [P, P, P, P, P, P, P, P, P, P, I, L_, I, I, F, F, I, F, U64, P, P],
    "ssamd_bn_bwd": [P, I, P, P, P, P, P, P, P, P, P, L_, I, I, I, F, U64, P, P],
})


def _bn_ws(device, R, C):
    return _workspace(device, 2 * 1024 * C + 16)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, gamma, beta, rmean, rvar, training, momentum, eps, act_tanh, p, out_f32, seed):
        B, L, C = h.shape
        R = B * L
        hc = h.contiguous()
        _need(hc, torch.bfloat16, "bn.h")
        dev = h.device
        stats = torch.empty(4, C, device=dev, dtype=torch.float32)  # mean, rstd, scale, shift
        out = torch.empty(B, L, C, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        ws = _bn_ws(dev, R, C)
        rc = lib().ssamd_bn_fwd(_ptr(hc), _ptr(gamma), _ptr(beta), _ptr(rmean), _ptr(rvar), _ptr(stats[0]),
                                _ptr(stats[1]), _ptr(stats[2]), _ptr(stats[3]), _ptr(out), int(out_f32), R, C,
                                int(training), float(momentum), float(eps), int(act_tanh), float(p), seed, _ptr(ws),
                                _stream())
        _check(rc, "ssamd_bn_fwd")
        ctx.save_for_backward(hc, gamma, stats)
        ctx.beta = beta
        ctx.cfg = (R, C, int(training), int(act_tanh), float(p), seed)
        return out

    @staticmethod
    def backward(ctx, dy):
        hc, gamma, stats = ctx.saved_tensors
        R, C, training, act_tanh, p, seed = ctx.cfg
        dyf32 = dy.dtype == torch.float32
        dy = dy.contiguous() if dyf32 else dy.to(torch.bfloat16).contiguous()
        dh = torch.empty_like(hc)
        dg, db = gradslots.claim(gamma), gradslots.claim(ctx.beta)
        if dg is None:
            dg = torch.empty(C, device=hc.device, dtype=torch.float32)
        if db is None:
            db = torch.empty(C, device=hc.device, dtype=torch.float32)
        ws = _bn_ws(hc.device, R, C)
        rc = lib().ssamd_bn_bwd(_ptr(dy), int(dyf32), _ptr(hc), _ptr(gamma), _ptr(stats[2]), _ptr(stats[3]),
                                _ptr(stats[0]), _ptr(stats[1]), _ptr(dh), _ptr(dg), _ptr(db), R, C, training, act_tanh,
                                p, seed, _ptr(ws), _stream())
        _check(rc, "ssamd_bn_bwd")
        return dh, dg, db, None, None, None, None, None, None, None, None, None


_SIGS.update({
    "ssamd_conv_gemm_bnbwd": [P, P, P, I, I, I, I, I, I, I, P, P, P, I, F, U64, P],
    "ssamd_bn_bwd_dz": [P, P, P, P, P, I, P, P, P, L_, I, I, P],
})


class _BNActConvFn(torch.autograd.Function):
    """h_out = conv(drop(act(BN(h))))  -- one PostNet link (``transformer/Layers.py:140-148``).

    Forward = ``ssamd_bn_fwd`` + the conv GEMM.  Backward: the conv's data-gradient GEMM starts the
    BatchNorm backward in its epilogue (``ssamd_conv_gemm_bnbwd``: dz = dy * keep * act' and the per-tile
    column partials of dz and dz * (h - mean)), so the separate BatchNorm reduction pass over dy and h is gone;
    ``ssamd_bn_bwd_dz`` combines the partials (fixed order) and streams dh = k1 dz + k2 h + k3.  The
    weight gradient reads the saved BN output y, as a plain conv's would."""

    @staticmethod
    def forward(ctx, h, gamma, beta, rmean, rvar, w, b, training, momentum, eps, act, p, seed, pad):
        B, L, C = h.shape
        R = B * L
        hc = h.contiguous()
        _need(hc, torch.bfloat16, "bn_conv.h")
        dev = h.device
        stats = torch.empty(4, C, device=dev, dtype=torch.float32)  # mean, rstd, scale, shift
        y = torch.empty(B, L, C, device=dev, dtype=torch.bfloat16)
        ws = _bn_ws(dev, R, C)
        rc = lib().ssamd_bn_fwd(_ptr(hc), _ptr(gamma), _ptr(beta), _ptr(rmean), _ptr(rvar), _ptr(stats[0]),
                                _ptr(stats[1]), _ptr(stats[2]), _ptr(stats[3]), _ptr(y), 0, R, C, int(training),
                                float(momentum), float(eps), int(act), float(p), seed, _ptr(ws), _stream())
        _check(rc, "ssamd_bn_fwd")
        ks = w.shape[2]
        N = w.shape[0]
        bf = None if b is None else b.detach().float().contiguous()
        out = conv_gemm_raw(y, weight_fwd(w), bf, B, L, C, ks, 1, pad, N)
        ctx.save_for_backward(hc, y, gamma, stats, w)
        ctx.beta, ctx.b = beta, b
        ctx.cfg = (B, L, C, ks, pad, N, int(training), int(act), float(p), seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        hc, y, gamma, stats, w = ctx.saved_tensors
        B, L, C, ks, pad, N, training, act, p, seed = ctx.cfg
        R = B * L
        dev = hc.device
        dout = dout.to(torch.bfloat16).contiguous()
        first = _wgrad_first(R)

        def dgrad():
            nparts = (R + 255) // 256
            part = torch.empty(2 * nparts * C, device=dev, dtype=torch.float32)
            dz = torch.empty(B, L, C, device=dev, dtype=torch.bfloat16)
            rc = lib().ssamd_conv_gemm_bnbwd(_ptr(dout), _ptr(weight_dgrad(w)), _ptr(dz), B, L, N, ks, 1,
                                             (ks - 1) - pad, C, _ptr(hc), _ptr(stats), _ptr(part), act, p, seed,
                                             _stream())
            _check(rc, "ssamd_conv_gemm_bnbwd")
            dh = torch.empty_like(hc)
            dg, db = gradslots.claim(gamma), gradslots.claim(ctx.beta)
            if dg is None:
                dg = torch.empty(C, device=dev, dtype=torch.float32)
            if db is None:
                db = torch.empty(C, device=dev, dtype=torch.float32)
            rc = lib().ssamd_bn_bwd_dz(_ptr(dz), _ptr(hc), _ptr(gamma), _ptr(stats), _ptr(part), nparts, _ptr(dh),
                                       _ptr(dg), _ptr(db), R, C, training, _stream())
            _check(rc, "ssamd_bn_bwd_dz")
            return dh, dg, db

        if not first:
            dh, dg, dbeta = dgrad()
        want_b = ctx.b is not None and ctx.needs_input_grad[6]
        sb = gradslots.claim(ctx.b) if want_b else None
        dw = dbias = None
        if ctx.needs_input_grad[5]:
            sw = gradslots.claim(w)
            res = wgrad_async(lambda: conv_wgrad_raw(y, dout, B, L, C, ks, 1, pad, N, with_bias=want_b, dW=sw, db=sb),
                              (y, dout), sw is not None and (sb is not None or not want_b),
                              (w, ctx.b) if want_b else (w,))
            dw, dbias = res if want_b else (res, None)
        elif want_b:
            dbias = colsum_raw(dout, N, sb)
        if first:
            dh, dg, dbeta = dgrad()
        return dh, dg, dbeta, None, None, dw, dbias, None, None, None, None, None, None, None


def bn_act_conv(h, bn, training, act_tanh, p, w, b, pad):
    """conv(drop(act(BN(h)))) -- see _BNActConvFn.  The BN channel count C must satisfy C % 8 == 0 and
    C >= 256 (the data-gradient GEMM's 256x256-tile epilogue); ``bn_act_conv_ok`` tells callers."""
    momentum = bn.momentum if bn.momentum is not None else 0.1
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    act = 2 if act_tanh == "relu" else int(bool(act_tanh))
    return _BNActConvFn.apply(h.to(torch.bfloat16), bn.weight, bn.bias, bn.running_mean, bn.running_var, w, b,
                              bool(training), momentum, bn.eps, act, float(p if training else 0.0), _next_seed(), pad)


def bn_act_conv_ok(C: int, w) -> bool:
    return C >= 256 and C % 8 == 0 and w.dim() == 3 and w.shape[0] % 8 == 0


def bn_act(h, bn, training, act_tanh, p, out_f32=False):
    """BatchNorm over all rows of channel-last h (+tanh, or ReLU with ``act_tanh="relu"``) + dropout,
    one fused op."""
    momentum = bn.momentum if bn.momentum is not None else 0.1
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    act = 2 if act_tanh == "relu" else int(bool(act_tanh))
    return _BNActFn.apply(h.to(torch.bfloat16), bn.weight, bn.bias, bn.running_mean, bn.running_var, bool(training),
                          momentum, bn.eps, act, float(p if training else 0.0), bool(out_f32), _next_seed())


# ------------------------------------------------------------------------ GST reference encoder
_SIGS.update({
    "ssamd_im2col_s2": [P, P, I, I, I, I, I, P],
    "ssamd_col2im_s2": [P, P, I, I, I, I, I, P],
    "ssamd_gru_fwd": [P, P, P, P, I, I, I, P, P, P, P],
    "ssamd_gru_bwd": [P, P, P, P, I, I, I, P, P, P],
    "ssamd_token_attn_fwd": [P, P, P, I, I, I, I, F, P, P, P],
    "ssamd_token_attn_bwd": [P, P, P, P, P, P, I, I, I, I, F, P, P, P, P],
})


def _s2(n):
    return (n - 1) // 2 + 1  # Conv2d k3 / s2 / p1 output size


def im2col_s2(x, Kp):
    """NHWC x [B, H, W, C] bf16 -> patch rows [B*Ho*Wo, Kp] (k = (ky*3 + kx)*C + c, zero padded)."""
    _need(x, torch.bfloat16, "im2col.x")
    B, H, W, C = x.shape
    col = torch.empty(B * _s2(H) * _s2(W), Kp, device=x.device, dtype=torch.bfloat16)
    _check(lib().ssamd_im2col_s2(_ptr(x), _ptr(col), B, H, W, C, Kp, _stream()), "ssamd_im2col_s2")
    return col


def _conv2d_wimg(w, Kp):
    """[Cout, Cin, 3, 3] fp32 -> bf16 [Cout, Kp] in the im2col k order (tiny: rebuilt per call)."""
    m = w.detach().permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    img = torch.zeros(w.shape[0], Kp, device=w.device, dtype=torch.bfloat16)
    img[:, : m.shape[1]] = m
    return img


class _Conv2dS2Fn(torch.autograd.Function):
    """Conv2d(k3, s2, p1) on NHWC bf16: im2col + MFMA GEMM; backward = GEMM + col2im gather and the
    split-M weight-gradient kernel on the (recomputed) patch rows with the fused bias gradient."""

    @staticmethod
    def forward(ctx, x, w, b):
        B, H, W, C = x.shape
        Cout = w.shape[0]
        assert w.shape[1:] == (C, 3, 3), "conv2d_s2 expects a [Cout, Cin, 3, 3] weight"
        Kp = (9 * C + 7) // 8 * 8
        Ho, Wo = _s2(H), _s2(W)
        xc = x.to(torch.bfloat16).contiguous()
        col = im2col_s2(xc, Kp)
        wimg = _conv2d_wimg(w, Kp)
        bf = None if b is None else b.detach().float().contiguous()
        y = conv_gemm_raw(col, wimg, bf, 1, B * Ho * Wo, Kp, 1, 1, 0, Cout)
        ctx.save_for_backward(xc, w, wimg)
        ctx.b = b
        ctx.dims = (B, H, W, C, Ho, Wo, Cout, Kp)
        return y.view(B, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        xc, w, wimg = ctx.saved_tensors
        B, H, W, C, Ho, Wo, Cout, Kp = ctx.dims
        rows = B * Ho * Wo
        dy = dy.to(torch.bfloat16).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dcol = conv_gemm_raw(dy, wimg.t().contiguous(), None, 1, rows, Cout, 1, 1, 0, Kp)
            dx = torch.empty_like(xc)
            _check(lib().ssamd_col2im_s2(_ptr(dcol), _ptr(dx), B, H, W, C, Kp, _stream()), "ssamd_col2im_s2")
        col = im2col_s2(xc, Kp)  # recomputed: cheaper than keeping [rows, 9C] alive over the step
        want_b = ctx.b is not None and ctx.needs_input_grad[2]
        res = conv_wgrad_raw(col, dy, 1, rows, Kp, 1, 1, 0, Cout, with_bias=want_b,
                             db=gradslots.claim(ctx.b) if want_b else None)
        dWp, db = res if want_b else (res, None)
        dw = dWp.view(Cout, Kp)[:, : 9 * C].reshape(Cout, 3, 3, C).permute(0, 3, 1, 2).contiguous()
        return dx, dw, db


def conv2d_s2(x, w, b=None):
    """NHWC [B, H, W, Cin] -> [B, ceil(H/2), ceil(W/2), Cout] bf16 (Conv2d 3x3, stride 2, pad 1)."""
    return _Conv2dS2Fn.apply(x, w, b)


def conv2d_s2_image(w):
    """Inference operand of ``conv2d_s2_infer``: the bf16 [Cout, Kp] im2col-order weight image."""
    return _conv2d_wimg(w, (9 * w.shape[1] + 7) // 8 * 8)


def conv2d_s2_infer(x, wimg, bias, act=None):
    """Forward-only conv2d_s2 on a prebuilt weight image (``conv2d_s2_image``) with the GEMM epilogue's
    activation: im2col + one GEMM, nothing rebuilt per call."""
    B, H, W, C = x.shape
    Cout, Kp = wimg.shape
    assert Kp == (9 * C + 7) // 8 * 8, "conv2d_s2_infer: weight image / input channel mismatch"
    Ho, Wo = _s2(H), _s2(W)
    col = im2col_s2(x.to(torch.bfloat16).contiguous(), Kp)
    y = conv_gemm_raw(col, wimg, bias, 1, B * Ho * Wo, Kp, 1, 1, 0, Cout, _ACT[act])
    return y.view(B, Ho, Wo, Cout)


class _GRUFn(torch.autograd.Function):
    """Single-layer batch-first GRU returning the hidden state at step ``last[b]`` of every row.

    Input projection and all weight / input gradients are MFMA GEMMs; the recurrence is the
    persistent ``gru_fwd`` / ``gru_bwd`` kernel pair (csrc/k_gst.hip)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, last):
        B, T, I = x.shape
        G, Hd = w_hh.shape
        assert G == 3 * Hd and tuple(w_ih.shape) == (G, I), "GRU weight shapes"
        _need(last, torch.int64, "gru.last")
        xc = x.to(torch.bfloat16).contiguous()
        gi = conv_gemm_raw(xc, weight_fwd(w_ih), b_ih.detach().float().contiguous(), 1, B * T, I, 1, 1, 0, G,
                           out_f32=True)
        hlast = torch.empty(B, Hd, device=x.device, dtype=torch.float32)
        sv = torch.empty(B, T, 5, Hd, device=x.device, dtype=torch.float32)
        hprev = torch.empty(B, T, Hd, device=x.device, dtype=torch.bfloat16)
        rc = lib().ssamd_gru_fwd(_ptr(gi), _ptr(weight_fwd(w_hh)), _ptr(b_hh.detach().float().contiguous()), _ptr(last),
                                 B, T, Hd, _ptr(hlast), _ptr(sv), _ptr(hprev), _stream())
        _check(rc, "ssamd_gru_fwd")
        ctx.save_for_backward(xc, w_ih, w_hh, last, sv, hprev)
        ctx.biases = (b_ih, b_hh)
        return hlast

    @staticmethod
    def backward(ctx, dh):
        xc, w_ih, w_hh, last, sv, hprev = ctx.saved_tensors
        b_ih, b_hh = ctx.biases
        B, T, I = xc.shape
        G, Hd = w_hh.shape
        dgi = torch.empty(B, T, G, device=xc.device, dtype=torch.bfloat16)
        dgh = torch.empty_like(dgi)
        rc = lib().ssamd_gru_bwd(_ptr(dh.float().contiguous()), _ptr(sv), _ptr(weight_dgrad(w_hh)), _ptr(last), B, T,
                                 Hd, _ptr(dgi), _ptr(dgh), _stream())
        _check(rc, "ssamd_gru_bwd")

        def wgrad(inp, dY, w, b, cin):
            sw = gradslots.claim(w)
            dw, db = conv_wgrad_raw(inp, dY, 1, B * T, cin, 1, 1, 0, G, with_bias=True,
                                    dW=None if sw is None else sw.view(G, cin, 1), db=gradslots.claim(b))
            return dw.view(G, cin), db

        dw_hh, db_hh = wgrad(hprev, dgh, w_hh, b_hh, Hd)
        dw_ih, db_ih = wgrad(xc, dgi, w_ih, b_ih, I)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = conv_gemm_raw(dgi, weight_dgrad(w_ih), None, 1, B * T, G, 1, 1, 0, I).view(B, T, I)
        return dx, dw_ih, dw_hh, db_ih, db_hh, None


def gru_last(x, gru, last):
    """``nn.GRU`` (1 layer, batch_first) parameters; x [B, T, I] -> h at step last[b] [B, H] fp32."""
    if gru.num_layers != 1 or gru.bidirectional or not gru.batch_first or not gru.bias:
        raise ValueError("gru_last supports a single-layer, unidirectional, batch-first GRU with biases")
    return _GRUFn.apply(x, gru.weight_ih_l0, gru.weight_hh_l0, gru.bias_ih_l0, gru.bias_hh_l0,
                        last.to(torch.int64).contiguous())


class _TokenAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, K, V):
        B = q.shape[0]
        NH, N, D = K.shape
        qc, Kc, Vc = q.float().contiguous(), K.float().contiguous(), V.float().contiguous()
        assert qc.shape[1] == NH * D and Vc.shape == Kc.shape
        o = torch.empty(B, NH * D, device=q.device, dtype=torch.float32)
        w = torch.empty(B, NH, N, device=q.device, dtype=torch.float32)
        scale = 1.0 / math.sqrt(D)
        _check(lib().ssamd_token_attn_fwd(_ptr(qc), _ptr(Kc), _ptr(Vc), B, NH, N, D, scale, _ptr(o), _ptr(w),
                                          _stream()), "ssamd_token_attn_fwd")
        ctx.save_for_backward(qc, Kc, Vc, w)
        return o, w

    @staticmethod
    def backward(ctx, do, dw):
        qc, Kc, Vc, w = ctx.saved_tensors
        B = qc.shape[0]
        NH, N, D = Kc.shape
        dq = torch.empty_like(qc)
        part = _workspace(qc.device, B * 2 * NH * N * D)
        dkv = torch.empty(2, NH, N, D, device=qc.device, dtype=torch.float32)
        do = torch.zeros_like(qc) if do is None else do.float().contiguous()
        dw = None if dw is None else dw.float().contiguous()
        rc = lib().ssamd_token_attn_bwd(_ptr(do), _ptr(qc), _ptr(Kc), _ptr(Vc), _ptr(w), _ptr(dw), B, NH, N,
                                        D, 1.0 / math.sqrt(D), _ptr(dq), _ptr(part), _ptr(dkv), _stream())
        _check(rc, "ssamd_token_attn_bwd")
        return dq, dkv[0], dkv[1]


def token_attention(q, K, V):
    """q [B, NH*D], K/V [NH, N, D] -> (style [B, NH*D] fp32, weights [B, NH, N])."""
    return _TokenAttnFn.apply(q, K, V)


_SIGS.update({"ssamd_token_bank_fwd": [P, P, P, I, I, I, I, P, P, P, P],
              "ssamd_token_bank_bwd": [P, P, P, P, P, I, I, I, I, P, P, P, P]})


class _TokenBankFn(torch.autograd.Function):
    """keys = tanh(E); K / V = keys @ Wk^T / Wv^T split into heads [NH, N, D] (reference GST token bank)."""

    @staticmethod
    def forward(ctx, E, Wk, Wv, n_head):
        N, dt = E.shape
        T = Wk.shape[0]
        Ec, Wkc, Wvc = (t.detach().float().contiguous() for t in (E, Wk, Wv))
        D = T // n_head
        K = torch.empty(n_head, N, D, device=E.device, dtype=torch.float32)
        V = torch.empty_like(K)
        tE = torch.empty(N, dt, device=E.device, dtype=torch.float32)
        _check(lib().ssamd_token_bank_fwd(_ptr(Ec), _ptr(Wkc), _ptr(Wvc), N, dt, T, n_head, _ptr(K), _ptr(V), _ptr(tE),
                                          _stream()), "ssamd_token_bank_fwd")
        ctx.save_for_backward(tE, Wkc, Wvc)
        ctx.n_head = n_head
        ctx.owners = (E, Wk, Wv)
        return K, V

    @staticmethod
    def backward(ctx, dK, dV):
        tE, Wkc, Wvc = ctx.saved_tensors
        N, dt = tE.shape
        T = Wkc.shape[0]
        dK = torch.zeros(ctx.n_head, N, T // ctx.n_head, device=tE.device) if dK is None else dK.float().contiguous()
        dV = torch.zeros_like(dK) if dV is None else dV.float().contiguous()
        outs = []
        for p, shape in zip(ctx.owners, ((N, dt), (T, dt), (T, dt))):
            slot = gradslots.claim(p)
            outs.append(slot if slot is not None else torch.empty(shape, device=tE.device, dtype=torch.float32))
        dE, dWk, dWv = outs
        _check(lib().ssamd_token_bank_bwd(_ptr(dK), _ptr(dV), _ptr(tE), _ptr(Wkc), _ptr(Wvc), N, dt, T, ctx.n_head,
                                          _ptr(dE), _ptr(dWk), _ptr(dWv), _stream()), "ssamd_token_bank_bwd")
        return dE, dWk, dWv, None


def token_bank(E, Wk, Wv, n_head):
    """GST style-token bank keys / values [NH, N, D] (fp32) from the token table E [N, dt]."""
    return _TokenBankFn.apply(E, Wk, Wv, n_head)


# ------------------------------------------------------------------------ vocoder (inference)
_SIGS.update({"ssamd_conv3_sq": [P, P, P, P, I, I, I, P]})
_SIGS.update({"ssamd_resblock_layer_prof": [P, P, P, P, P, P, P, I, I, I, I, I, F, F, I, P, L_, I, P],
              "ssamd_resblock_layer_tile": [I, I]})
_SIGS.update({"ssamd_resblock_layer": [P, P, P, P, P, P, P, I, I, I, I, I, F, F, I, P],
              "ssamd_conv_gemm_ex": [P, P, P, P, P, I, I, I, I, I, I, I, I, P, P, F, I, P],
              "ssamd_conv_gemm_ex2": [P, P, P, P, P, I, I, I, I, I, I, I, I, P, P, F, I, I, P]})


def resblock_layer(x, c1, c2, d, slope, acc=None, out_scale=1.0, post_lrelu=False):
    """One fused HiFi-GAN ResBlock1 layer (csrc/k_vocoder.hip), channel-last bf16, no autograd:
    ``(acc +) x + conv2(lrelu(conv1_d(lrelu(x)) + b1)) + b2``, times ``out_scale`` [then lrelu when
    ``post_lrelu``: the next upsampling conv's input].  With ``acc`` the result is written into
    ``acc`` in place (the MRF branch sum)."""
    _need(x, torch.bfloat16, "resblock.x")
    B, T, C = x.shape
    K = c1.weight.shape[2]
    assert tuple(c1.weight.shape) == (C, C, K) and tuple(c2.weight.shape) == (C, C, K)
    w1, w2 = weight_fwd(c1.weight), weight_fwd(c2.weight)
    b1 = c1.bias.detach().float().contiguous()
    b2 = c2.bias.detach().float().contiguous()
    for t, nm in ((w1, "resblock.w1"), (w2, "resblock.w2"), (b1, "resblock.b1"), (b2, "resblock.b2")):
        _need(t, t.dtype, nm)  # a host tensor here (e.g. a weight-norm .weight left on the CPU) would fault the GPU
    if acc is not None:
        _need(acc, torch.bfloat16, "resblock.acc")
        assert acc.shape == x.shape and acc.data_ptr() != x.data_ptr(), "acc must be a separate [B, T, C] buffer"
        out = acc
    else:
        out = torch.empty_like(x)
    rc = lib().ssamd_resblock_layer(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), _ptr(acc), _ptr(out), B, T, C,
                                    K, int(d), float(slope), float(out_scale), int(bool(post_lrelu)), _stream())
    _check(rc, "ssamd_resblock_layer")
    return out


_SIGS.update({"ssamd_resblock_fused": [P] * 15 + [I, I, I, I, I, I, I, F, F, I, P],
              "ssamd_resblock_fusable": [I, I]})


def resblock_fusable(C: int, K: int) -> bool:
    """Geometry with a whole-ResBlock kernel instance (``ssamd_resblock_fused``)."""
    return bool(lib().ssamd_resblock_fusable(int(C), int(K)))


def conv3_sq(x, wimg, bias):
    """Square 3-tap conv (pad 1), channel-last bf16, no autograd: ``y = conv(x) + bias`` with ``wimg`` the bf16
    [C][3][C] implicit-GEMM image (csrc/k_vocoder.hip ``conv3_sq_kernel``: the upsamplers whose
    ``convT_as_conv3`` form has N = stride * Cout = Cin).  C in {64, 128}."""
    _need(x, torch.bfloat16, "conv3_sq.x")
    _need(wimg, torch.bfloat16, "conv3_sq.w")
    _need(bias, torch.float32, "conv3_sq.bias")
    B, T, C = x.shape
    assert tuple(wimg.shape) == (C, 3, C) and bias.numel() == C, "conv3_sq: weight / bias shape"
    out = torch.empty_like(x)
    _check(lib().ssamd_conv3_sq(_ptr(x), _ptr(wimg), _ptr(bias), _ptr(out), B, T, C, _stream()), "ssamd_conv3_sq")
    return out


def resblock_fused(x, convs1, convs2, dilations, slope, acc=None, out_scale=1.0, post_lrelu=False):
    """A whole HiFi-GAN ResBlock1 (three lrelu -> dilated conv -> lrelu -> conv -> + x layers) in ONE
    kernel (csrc/k_vocoder.hip ``resblock_fused_kernel``): the residual stream stays in fp32 registers
    across the three layers, the activations in LDS.  Channel-last bf16, no autograd; same output
    contract as three ``resblock_layer`` calls."""
    _need(x, torch.bfloat16, "resblock.x")
    B, T, C = x.shape
    K = convs1[0].weight.shape[2]
    ws, bs = [], []
    for c1, c2 in zip(convs1, convs2):
        for c in (c1, c2):
            assert tuple(c.weight.shape) == (C, C, K)
            ws.append(weight_fwd(c.weight))
            bs.append(c.bias.detach().float().contiguous())
            _need(ws[-1], torch.bfloat16, "resblock.w")  # host weights (weight-norm .weight on the CPU) would fault
            _need(bs[-1], torch.float32, "resblock.b")
    if acc is not None:
        _need(acc, torch.bfloat16, "resblock.acc")
        assert acc.shape == x.shape and acc.data_ptr() != x.data_ptr(), "acc must be a separate [B, T, C] buffer"
        out = acc
    else:
        out = torch.empty_like(x)
    d0, d1, d2 = (int(v) for v in dilations)
    rc = lib().ssamd_resblock_fused(_ptr(x), *[_ptr(w) for w in ws], *[_ptr(b) for b in bs], _ptr(acc), _ptr(out),
                                    B, T, C, K, d0, d1, d2, float(slope), float(out_scale),
                                    int(bool(post_lrelu)), _stream())
    _check(rc, "ssamd_resblock_fused")
    return out


# ------------------------------------------------------------------------ packed (length-exact) vocoder
_SIGS.update({"ssamd_gemm_retain_workspaces": [I],
              "ssamd_resblock_set_tall": [I],
              "ssamd_resblock_set_whole_extra": [I],
              "ssamd_voc_tile_rows": [I, I, I, I, I, I],
              "ssamd_voc_rinfo": [P, I, I, I, P, P],
              "ssamd_voc_pack": [P, I, P, I, I, I, P, P],
              "ssamd_resblock_layer_pk": [P, P, P, P, P, P, P, P, I, I, I, I, F, F, I, P],
              "ssamd_resblock_layer_pk2": [P, P, P, P, P, P, P, P, I, I, I, I, F, F, I, I, P],
              "ssamd_resblock_fused_pk": [P] * 16 + [I, I, I, I, I, I, F, F, I, I, P],
              "ssamd_conv3_sq_pk": [P, P, P, P, P, I, I, P],
              "ssamd_conv_post_pk": [P, P, P, P, I, I, F, F, P, P, L_, P],
              "ssamd_conv_post_tile_rows": [],
              "ssamd_conv_gemm_ex3": [P, P, P, P, P, I, I, I, I, I, I, I, P, P, F, I, I, P, P]})


class VocPack:
    """Row layout of a packed vocoder batch: sequence b's frames at rows ``cu[b] .. cu[b+1]-1`` of every stage
    (times the stage's rate), no padding.  ``tiles(kind, rate, BM)`` returns (device int32 [n, 4] table, n) of the
    tiled kernels' work items -- {first row of the sequence, its rows, t0, sequence} per tile of BM rows at that
    rate, tiles never straddling two sequences -- and ``rinfo(rate)`` the per-row {position, length} table of the
    GEMM stages; both are built once per batch and cached per key.  The host knows the lengths (they sized the
    batch), so the tables cost no device sync: all of them go up in ONE pinned host-to-device copy."""

    def __init__(self, lens, device, rate_tiles):
        import numpy as np

        self.lens = np.asarray([int(v) for v in lens], dtype=np.int64)
        self.B = len(self.lens)
        self.R = int(self.lens.sum())
        self.device = device
        cu = np.zeros(self.B + 1, dtype=np.int64)
        cu[1:] = np.cumsum(self.lens)
        self.cu_host = cu
        # every (rate, BM) tile table the caller will ask for, laid out back to back in one int32 buffer
        parts, self._off = [cu.astype(np.int32)], {}
        o = self.B + 1
        for rate, bm in rate_tiles:
            key = (int(rate), int(bm))
            if key in self._off or bm <= 0:
                continue
            L = self.lens * rate
            cnt = (L + bm - 1) // bm
            n = int(cnt.sum())
            u = np.repeat(np.arange(self.B), cnt)
            first = np.zeros(self.B, dtype=np.int64)
            first[1:] = np.cumsum(cnt)[:-1]
            t0 = (np.arange(n) - first[u]) * bm
            tab = np.stack([cu[u] * rate, L[u], t0, u], axis=1).astype(np.int32)
            assert (cu[-1] * rate) < 2 ** 31, "packed vocoder: row offsets exceed int32"
            parts.append(tab.reshape(-1))
            self._off[key] = (o, n)
            o += 4 * n
        host = torch.from_numpy(np.concatenate(parts)).pin_memory() if device.type == "cuda" else \
            torch.from_numpy(np.concatenate(parts))
        self.buf = host.to(device, non_blocking=True)
        self.cu = self.buf[: self.B + 1]
        self._rinfo = {}

    def tiles(self, rate, bm):
        o, n = self._off[(int(rate), int(bm))]
        return self.buf[o: o + 4 * n], n

    def rinfo(self, rate):
        r = self._rinfo.get(rate)
        if r is None:
            rows = int(self.lens.max()) * rate if self.B else 0
            r = torch.empty(self.R * rate, 2, device=self.device, dtype=torch.int32)
            _check(lib().ssamd_voc_rinfo(_ptr(self.cu), self.B, int(rate), rows, _ptr(r), _stream()), "ssamd_voc_rinfo")
            self._rinfo[rate] = r
        return r


_VOC_PACKS = collections.OrderedDict()  # (device, lengths, geometries) -> VocPack: tables of a repeated length set


def voc_pack_for(lens, device, rate_tiles, cache: int = 32) -> "VocPack":
    """A VocPack for these lengths, reused when the same length set comes back (batch-1 serving repeats lengths;
    the tables depend on the lengths only, never on the data, and are never written after they are built)."""
    key = (str(device), tuple(int(v) for v in lens), tuple(rate_tiles))
    vp = _VOC_PACKS.get(key)
    if vp is not None:
        _VOC_PACKS.move_to_end(key)
        return vp
    vp = VocPack(lens, device, rate_tiles)
    _VOC_PACKS[key] = vp
    while len(_VOC_PACKS) > cache:
        _VOC_PACKS.popitem(last=False)
    return vp


_TILE_ROWS = {}


def voc_tile_rows(kind, C: int, K: int = 0, dil=(0, 0, 0)) -> int:
    """Tile height of a tiled vocoder kernel (0 resblock_layer (the global variant), 1 resblock_fused, 2 conv3_sq,
    3 / 4 the tall / 128-row per-layer tile, "post" conv_post)."""
    key = (kind, C, K, tuple(dil))
    v = _TILE_ROWS.get(key)
    if v is None:
        if kind == "post":
            v = int(lib().ssamd_conv_post_tile_rows())
        else:
            d0, d1, d2 = (int(x) for x in dil)
            v = int(lib().ssamd_voc_tile_rows(int(kind), int(C), int(K), d0, d1, d2))
        _TILE_ROWS[key] = v
    return v


def voc_pack(mel, vp: "VocPack"):
    """[B, M, C] (fp32 / bf16) -> [R, C] bf16 valid rows in the VocPack order."""
    B, M, C = mel.shape
    src = mel.contiguous()
    f32 = src.dtype == torch.float32
    if not f32:
        _need(src, torch.bfloat16, "voc_pack.src")
    out = torch.empty(vp.R, C, device=mel.device, dtype=torch.bfloat16)
    _check(lib().ssamd_voc_pack(_ptr(src), int(f32), _ptr(vp.cu), B, M, C, _ptr(out), _stream()), "ssamd_voc_pack")
    return out


def conv1d_infer_packed(x, vp, rate, w, b, pad, dil, act=None, resid=None, acc=None, scale=1.0, post_act=None,
                        dual_lrelu=False, wimg=None, ksplit=0):
    """``conv1d_infer`` on packed rows x [R*rate, Cin]: every conv zero-pads at its own sequence's ends."""
    Rr, Cin = x.shape
    ks = 1 if w.dim() == 2 else w.shape[2]
    N = w.shape[0]
    bf = None if b is None else b.detach().float().contiguous()
    wi = weight_fwd(w) if wimg is None else wimg
    xc = x.contiguous()
    _need(xc, torch.bfloat16, "conv_pk.x")
    _need(wi, torch.bfloat16, "conv_pk.w")
    assert Rr == vp.R * rate and wi.numel() == N * ks * Cin and N % 8 == 0 and Cin % 8 == 0, "conv_pk: shape"
    for t in (resid, acc):
        if t is not None:
            _need(t, torch.bfloat16, "conv_pk.operand")
            assert t.numel() == Rr * N, "conv_pk: operand shape"
    y = acc if acc is not None else torch.empty(Rr, N, device=x.device, dtype=torch.bfloat16)
    y2 = torch.empty_like(y) if dual_lrelu else None
    ri = vp.rinfo(rate)
    rc = lib().ssamd_conv_gemm_ex3(_ptr(xc), _ptr(wi), _ptr(bf), _ptr(resid), _ptr(y), Rr, Cin, ks, dil, pad, N,
                                   _ACT[act], _ptr(acc), _ptr(y2), float(scale), _ACT[post_act], int(ksplit), _ptr(ri),
                                   _stream())
    _check(rc, "ssamd_conv_gemm_ex3")
    return (y, y2) if dual_lrelu else y


_TALL_MIN_TILES = [512]
_SMALL_MAX_TILES = [192]  # the 64-row tile below this many 128-row tiles (3/4 of the CUs; 0: never)  # packed per-layer ResBlock: the tall tile only when it still yields >= this many tiles


def rb_layer_tile(C: int, K: int, lens, rate: int):
    """(tile mode, tile rows) of the per-layer ResBlock kernel for a packed batch: 1 = the tall tile (fewer LDS
    reads per MFMA, ``csrc/k_vocoder.hip`` RBT) when the batch gives it at least ``_TALL_MIN_TILES`` tiles (two per
    CU), 0 = the 128-row tile, -1 = the 64-row tile (RBS) when even the 128-row tile gives fewer than
    ``_SMALL_MAX_TILES`` workgroups (batch-1 latency).  Deterministic in (C, K, lengths, rate), so the tile tables
    and the launch agree."""
    bt, br = voc_tile_rows(3, C, K), voc_tile_rows(4, C, K)
    if not br:
        return 1, bt
    if bt and _TALL[0] and sum(-(-int(L) * rate // bt) for L in lens) >= _TALL_MIN_TILES[0]:
        return 1, bt
    bs = voc_tile_rows(5, C, K)
    if bs and sum(-(-int(L) * rate // br) for L in lens) < _SMALL_MAX_TILES[0]:
        return -1, bs
    return 0, br


_TALL = [True]


def resblock_layer_packed(x, vp, rate, c1, c2, d, slope, acc=None, out_scale=1.0, post_lrelu=False):
    """``resblock_layer`` on packed rows x [R*rate, C] (tile variant: ``rb_layer_tile``)."""
    _need(x, torch.bfloat16, "resblock.x")
    Rr, C = x.shape
    K = c1.weight.shape[2]
    w1, w2 = weight_fwd(c1.weight), weight_fwd(c2.weight)
    b1 = c1.bias.detach().float().contiguous()
    b2 = c2.bias.detach().float().contiguous()
    out = acc if acc is not None else torch.empty_like(x)
    tall, bm = rb_layer_tile(C, K, vp.lens, rate)
    tt, n = vp.tiles(rate, bm)
    rc = lib().ssamd_resblock_layer_pk2(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), _ptr(acc), _ptr(out),
                                        _ptr(tt), n, C, K, int(d), float(slope), float(out_scale),
                                        int(bool(post_lrelu)), int(tall), _stream())
    _check(rc, "ssamd_resblock_layer_pk2")
    return out


_RF_SHORT_MAX_TILES = [128]  # whole-ResBlock kernel: the short tile below this many regular tiles (0: never)


def rf_tile(C: int, K: int, dilations, lens, rate: int):
    """(short, tile rows) of the whole-ResBlock kernel for a packed batch: its short tile (RF S = 1: 2-4x the
    workgroups, more halo recompute) when the regular tile gives fewer than ``_RF_SHORT_MAX_TILES`` tiles (a batch-1
    stage runs 40-125 regular tiles on 256 CUs).  Deterministic in its arguments: table and launch agree."""
    bm = voc_tile_rows(1, C, K, tuple(dilations))
    bs = voc_tile_rows(6, C, K, tuple(dilations))
    if bs and sum(-(-int(L) * rate // bm) for L in lens) < _RF_SHORT_MAX_TILES[0]:
        return True, bs
    return False, bm


def resblock_fused_packed(x, vp, rate, convs1, convs2, dilations, slope, acc=None, out_scale=1.0, post_lrelu=False):
    """``resblock_fused`` on packed rows x [R*rate, C]."""
    _need(x, torch.bfloat16, "resblock.x")
    Rr, C = x.shape
    K = convs1[0].weight.shape[2]
    ws, bs = [], []
    for c1, c2 in zip(convs1, convs2):
        for c in (c1, c2):
            ws.append(weight_fwd(c.weight))
            bs.append(c.bias.detach().float().contiguous())
    out = acc if acc is not None else torch.empty_like(x)
    d0, d1, d2 = (int(v) for v in dilations)
    short, bm = rf_tile(C, K, (d0, d1, d2), vp.lens, rate)
    tt, n = vp.tiles(rate, bm)
    rc = lib().ssamd_resblock_fused_pk(_ptr(x), *[_ptr(w) for w in ws], *[_ptr(b) for b in bs], _ptr(acc), _ptr(out),
                                       _ptr(tt), n, C, K, d0, d1, d2, float(slope), float(out_scale),
                                       int(bool(post_lrelu)), int(short), _stream())
    _check(rc, "ssamd_resblock_fused_pk")
    return out


def conv3_sq_packed(x, vp, rate, wimg, bias):
    Rr, C = x.shape
    out = torch.empty_like(x)
    tt, n = vp.tiles(rate, voc_tile_rows(2, C))
    _check(lib().ssamd_conv3_sq_pk(_ptr(x), _ptr(wimg), _ptr(bias), _ptr(out), _ptr(tt), n, C, _stream()),
           "ssamd_conv3_sq_pk")
    return out


def conv_post_packed(x, vp, rate, w, b, out, slope=0.01, int16_scale=None):
    """conv_post on packed rows x [R*rate, C] into out [B, W] (sample t of sequence u at out[u, t]; the caller
    zero-fills out)."""
    Rr, C = x.shape
    wf = w.detach().reshape(-1).float().contiguous()
    bf = None if b is None else b.detach().reshape(-1).float().contiguous()
    tt, n = vp.tiles(rate, voc_tile_rows("post", C))
    assert out.shape[0] == vp.B and out.shape[1] >= int(vp.lens.max()) * rate, "conv_post_packed: output shape"
    if int16_scale is None:
        assert out.dtype == torch.float32
        rc = lib().ssamd_conv_post_pk(_ptr(x), _ptr(wf), _ptr(bf), _ptr(tt), n, C, float(slope), 1.0, _ptr(out), None,
                                      out.stride(0), _stream())
    else:
        assert out.dtype == torch.int16
        rc = lib().ssamd_conv_post_pk(_ptr(x), _ptr(wf), _ptr(bf), _ptr(tt), n, C, float(slope), float(int16_scale),
                                      None, _ptr(out), out.stride(0), _stream())
    _check(rc, "ssamd_conv_post_pk")
    return out


def conv1d_infer(x, w, b, pad, dil, act=None, resid=None, acc=None, scale=1.0, post_act=None, dual_lrelu=False,
                 wimg=None, ksplit=0):
    """Inference conv (no autograd), channel-last bf16, everything in the GEMM epilogue:
    ``v = act(conv(x) + b) [+ resid]``; ``v = (v [+ acc]) * scale``; returns ``post_act(v)``
    (and ``lrelu(v)`` as a second output when ``dual_lrelu``).  ``acc`` may be the output
    buffer itself (in-place accumulation; it is then returned).  ``wimg``: a prepared bf16
    [N][ks][Cin] operand image (with ``w`` the fp32 [N, Cin, ks] it came from, for shapes).  ``ksplit``: the
    weights are the 3-tap ConvTranspose form (hifigan ``convT_as_conv3``) and output columns >= ksplit read
    taps {1, 2} only, the others taps {0, 1} -- each 256-column tile skips its all-zero tap."""
    B, L, Cin = x.shape
    ks = 1 if w.dim() == 2 else w.shape[2]
    N = w.shape[0]
    bf = None if b is None else b.detach().float().contiguous()
    wi = weight_fwd(w) if wimg is None else wimg
    if acc is None and scale == 1.0 and post_act is None and not dual_lrelu and not ksplit:
        return conv_gemm_raw(x.contiguous(), wi, bf, B, L, Cin, ks, dil, pad, N, _ACT[act],
                             resid=None if resid is None else resid.contiguous())
    xc = x.contiguous()
    _need(xc, torch.bfloat16, "conv_ex.x")
    _need(wi, torch.bfloat16, "conv_ex.w")
    assert wi.numel() == N * ks * Cin and N % 8 == 0 and Cin % 8 == 0, "conv_ex: shape"
    if bf is not None:
        assert bf.numel() == N
    for t in (resid, acc):
        if t is not None:
            _need(t, torch.bfloat16, "conv_ex.operand")
            assert t.numel() == B * L * N, "conv_ex: operand shape"
    y = acc if acc is not None else torch.empty(B, L, N, device=x.device, dtype=torch.bfloat16)
    y2 = torch.empty_like(y) if dual_lrelu else None
    if ksplit:
        rc = lib().ssamd_conv_gemm_ex2(_ptr(xc), _ptr(wi), _ptr(bf), _ptr(resid), _ptr(y), B, L, Cin, ks, dil, pad,
                                       N, _ACT[act], _ptr(acc), _ptr(y2), float(scale), _ACT[post_act], int(ksplit),
                                       _stream())
    else:
        rc = lib().ssamd_conv_gemm_ex(_ptr(xc), _ptr(wi), _ptr(bf), _ptr(resid), _ptr(y), B, L, Cin, ks, dil, pad,
                                      N, _ACT[act], _ptr(acc), _ptr(y2), float(scale), _ACT[post_act], _stream())
    _check(rc, "ssamd_conv_gemm_ex")
    return (y, y2) if dual_lrelu else y


# ------------------------------------------------------------------------ audio front-end
_SIGS.update({"ssamd_logmel": [P, I, L_, I, I, P, P, I, F, P, P, P]})


def logmel(y, n_fft, hop, window, basis, clip=1e-5):
    """y [B, N] fp32 -> (log-mel [B, n_mel, N // hop + 1], energy [B, frames]): TacotronSTFT semantics
    (centre reflect padding, |FFT|, mel basis, log(clamp)), one fused kernel (csrc/k_audio.hip)."""
    _need(y, torch.float32, "logmel.y")
    _need(window, torch.float32, "logmel.window")
    _need(basis, torch.float32, "logmel.basis")
    y2 = y.reshape(-1, y.shape[-1])
    B, N = y2.shape
    n_mel = basis.shape[0]
    assert window.numel() == n_fft and basis.shape[1] == n_fft // 2 + 1
    frames = N // hop + 1
    mel = torch.empty(B, n_mel, frames, device=y.device, dtype=torch.float32)
    energy = torch.empty(B, frames, device=y.device, dtype=torch.float32)
    rc = lib().ssamd_logmel(_ptr(y2), B, N, n_fft, hop, _ptr(window), _ptr(basis), n_mel, float(clip), _ptr(mel),
                            _ptr(energy), _stream())
    _check(rc, "ssamd_logmel")
    return mel, energy


# ------------------------------------------------------------------------ N = 1 heads
class _HeadFn(torch.autograd.Function):
    """Variance-predictor head Linear(C -> 1) + pad mask (one wave per row)."""

    @staticmethod
    def forward(ctx, h, w, b, lens):
        B, L, C = h.shape
        hc = h.to(torch.bfloat16).contiguous()
        wf = w.detach().reshape(-1).float().contiguous()
        bf = None if b is None else b.detach().reshape(-1).float().contiguous()
        out = torch.empty(B, L, device=h.device, dtype=torch.float32)
        rc = lib().ssamd_head_fwd(_ptr(hc), _ptr(wf), _ptr(bf), _ptr(lens), B * L, L, C, _ptr(out), _stream())
        _check(rc, "ssamd_head_fwd")
        ctx.save_for_backward(hc, wf, lens)
        ctx.params = (w, b)
        ctx.hdtype = h.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        hc, wf, lens = ctx.saved_tensors
        w, b = ctx.params
        B, L, C = hc.shape
        g = g.float().contiguous()
        dh = torch.empty_like(hc)
        dw = gradslots.claim(w)  # arena slot (overwritten by the fixed-order reduce) or a fresh buffer
        if dw is None:
            dw = torch.empty_like(w, dtype=torch.float32)
        db = None
        if b is not None:
            db = gradslots.claim(b)
            if db is None:
                db = torch.empty_like(b, dtype=torch.float32)
        ws = _workspace(hc.device, int(lib().ssamd_head_bwd_ws(B * L, C)))
        rc = lib().ssamd_head_bwd(_ptr(g), _ptr(hc), _ptr(wf), _ptr(lens), B * L, L, C, _ptr(dh), _ptr(dw), _ptr(db),
                                  _ptr(ws), ws.numel(), _stream())
        _check(rc, "ssamd_head_bwd")
        return dh.to(ctx.hdtype), dw, db, None


def predictor_head(h, w, b, lengths):
    """[B, L, C] -> [B, L] fp32 = h @ w^T + b, 0 at padded rows (lengths may be None)."""
    C = h.shape[-1]
    if C not in (64, 128, 256, 512) or w.shape[0] != 1:
        _torch_fallback(f"predictor_head(C={C}, out={w.shape[0]})")  # raises unless explicitly allowed
        out = ref.linear(h, w, b).float().squeeze(-1)
        return out if lengths is None else out.masked_fill(ref.lengths_to_mask(lengths, out.shape[1]), 0.0)
    lens = None if lengths is None else lengths.to(torch.int64).contiguous()
    return _HeadFn.apply(h, w, b, lens)


def conv_post(x, w, b, slope=0.01, int16_scale=None):
    """HiFi-GAN conv_post (inference): lrelu(slope) -> Conv1d(C->1, k7, pad 3) -> tanh, channel-last
    x [B, T, C] bf16 -> [B, T] fp32, or int16 (x int16_scale, clamped) when ``int16_scale`` is given."""
    B, T, C = x.shape
    xc = x.to(torch.bfloat16).contiguous()
    wf = w.detach().reshape(-1).float().contiguous()
    assert wf.numel() == C * 7, "conv_post expects a [1, C, 7] weight"
    bf = None if b is None else b.detach().reshape(-1).float().contiguous()
    if int16_scale is None:
        out = torch.empty(B, T, device=x.device, dtype=torch.float32)
        rc = lib().ssamd_conv_post(_ptr(xc), _ptr(wf), _ptr(bf), B, T, C, float(slope), 1.0, _ptr(out), None, _stream())
    else:
        out = torch.empty(B, T, device=x.device, dtype=torch.int16)
        rc = lib().ssamd_conv_post(_ptr(xc), _ptr(wf), _ptr(bf), B, T, C, float(slope), float(int16_scale), None,
                                   _ptr(out), _stream())
    _check(rc, "ssamd_conv_post")
    return out


# ------------------------------------------------------------------------ small glue kernels
_SIGS.update({"ssamd_duration_round": [P, P, I, P, I, I, P, P, P],
              "ssamd_seq_mean": [P, P, I, I, I, F, P, P],
              "ssamd_seq_mean_bwd": [P, P, I, I, I, F, P, L_, P],
              "ssamd_add_rowvec": [P, P, P, I, I, I, P, P]})


def duration_round(log_d, lengths, control=1.0):
    """Inference durations (reference ``model/modules.py:132-137``): max(round(exp(log_d) - 1), 0),
    times the control (scalar or per-phoneme [B, T]), rounded, 0 at padded phonemes; plus the mel
    lengths.  -> (d int64 [B, T], mel_len int64 [B]); one kernel, no host sync."""
    ld = log_d.float().contiguous()
    B, T = ld.shape
    ctl, per = None, 0
    if isinstance(control, torch.Tensor):
        c = control.to(ld.device, torch.float32)
        if c.dim() == 2:
            if c.shape[1] != T:
                c = torch.nn.functional.pad(c, (0, max(0, T - c.shape[1])), value=1.0)[:, :T]
            ctl, per = c.expand(B, T).contiguous(), 1
        else:
            ctl = c.reshape(-1)[:1].contiguous()
    elif float(control) != 1.0:
        ctl = torch.full((1,), float(control), device=ld.device, dtype=torch.float32)
    lens = None if lengths is None else lengths.to(torch.int64).contiguous()
    d = torch.empty(B, T, device=ld.device, dtype=torch.int64)
    ml = torch.empty(B, device=ld.device, dtype=torch.int64)
    rc = lib().ssamd_duration_round(_ptr(ld), _ptr(ctl), per, _ptr(lens), B, T, _ptr(d), _ptr(ml), _stream())
    _check(rc, "ssamd_duration_round")
    return d, ml


class _SeqMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cu, B, L, div):
        xc = x.to(torch.bfloat16).contiguous()
        C = xc.shape[-1]
        out = torch.empty(B, C, device=x.device, dtype=torch.float32)
        rc = lib().ssamd_seq_mean(_ptr(xc), _ptr(cu), B, L, C, float(div), _ptr(out), _stream())
        _check(rc, "ssamd_seq_mean")
        ctx.save_for_backward(cu)
        ctx.geom = (B, L, C, float(div), xc.shape, x.dtype, cu is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        B, L, C, div, shape, dtype, has_cu = ctx.geom
        (cu,) = ctx.saved_tensors
        dx = torch.empty(shape, device=g.device, dtype=torch.bfloat16)
        rows = dx.numel() // C
        rc = lib().ssamd_seq_mean_bwd(_ptr(g.float().contiguous()), _ptr(cu if has_cu else None), B, L, C, div,
                                      _ptr(dx), rows, _stream())
        _check(rc, "ssamd_seq_mean_bwd")
        return dx.to(dtype), None, None, None, None


def seq_mean(x, divisor=None, pack=None):
    """[B, L, C] -> [B, C] fp32 mean over L (the reference's mean over the padded length; ``divisor``
    overrides L), or per packed sequence ([1, R, C] rows, ``pack``) divided by ``divisor``."""
    if pack is not None:
        return _SeqMeanFn.apply(x, pack.cu, pack.B, pack.M, float(divisor or pack.M))
    B, L, C = x.shape
    if C % 8:
        _torch_fallback(f"seq_mean C={C}")
        return x.float().sum(1) / float(divisor or L)
    return _SeqMeanFn.apply(x, None, B, L, float(divisor or L))


class _AddRowVecFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, v):
        xc = x.to(torch.bfloat16).contiguous()
        B, L, C = xc.shape
        vf = v.detach().float().contiguous()
        assert vf.shape == (B, C), "add_rowvec: one vector per sequence"
        out = torch.empty_like(xc)
        rc = lib().ssamd_add_rowvec(_ptr(xc), _ptr(vf), None, B, L, C, _ptr(out), _stream())
        _check(rc, "ssamd_add_rowvec")
        ctx.geom = (B, L, C, v.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        B, L, C, vdtype = ctx.geom
        gc = g.to(torch.bfloat16).contiguous()
        dv = None
        if ctx.needs_input_grad[1]:
            dv = torch.empty(B, C, device=g.device, dtype=torch.float32)
            rc = lib().ssamd_seq_mean(_ptr(gc), None, B, L, C, 1.0, _ptr(dv), _stream())  # fixed-order row sums
            _check(rc, "ssamd_seq_mean")
            dv = dv.to(vdtype)
        return g, dv


def add_rowvec(x, v):
    """x [B, L, C] + v[b] broadcast over L (bf16 out): the speaker-embedding add (reference
    ``model/fastspeech2.py:74-77``), backward = per-utterance fixed-order row sums."""
    if x.shape[-1] % 8:
        _torch_fallback(f"add_rowvec C={x.shape[-1]}")
        return x + v.to(x.dtype).unsqueeze(1)
    return _AddRowVecFn.apply(x, v)


_SIGS.update({"ssamd_rowvec_grad": [P, P, I, I, I, I, P, P, L_, P]})


class _AddTableRowsFn(torch.autograd.Function):
    """x [B, L, C] + table[ids[b]] broadcast over L: the speaker-embedding lookup fused into the add (one
    kernel, no [B, C] gathered intermediate).  Backward: per-utterance fixed-order row sums of dout, then
    dtable[v] = sum of the sums of utterances with ids == v, in utterance order (deterministic, no
    atomics), written straight into the table's arena gradient slot -- every row (0 where unused)."""

    @staticmethod
    def forward(ctx, x, table, ids):
        xc = x.to(torch.bfloat16).contiguous()
        B, L, C = xc.shape
        idc = ids.to(torch.int64).contiguous()
        assert idc.numel() == B and table.dim() == 2 and table.shape[1] == C, "add_table_rows: shapes"
        tf = table.detach()
        if tf.dtype != torch.float32 or not tf.is_contiguous():
            tf = tf.float().contiguous()
        out = torch.empty_like(xc)
        rc = lib().ssamd_add_rowvec(_ptr(xc), _ptr(tf), _ptr(idc), B, L, C, _ptr(out), _stream())
        _check(rc, "ssamd_add_rowvec")
        ctx.save_for_backward(idc)
        ctx.table = table if isinstance(table, torch.nn.Parameter) else None  # gradient-slot owner
        ctx.geom = (B, L, C, table.shape[0], table.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        (idc,) = ctx.saved_tensors
        B, L, C, V, tdtype = ctx.geom
        dt = None
        if ctx.needs_input_grad[1]:
            gc = g.to(torch.bfloat16).contiguous()
            dt = gradslots.claim(ctx.table)
            if dt is None:
                dt = torch.empty(V, C, device=g.device, dtype=torch.float32)
            ws = _workspace(g.device, B * C)
            rc = lib().ssamd_rowvec_grad(_ptr(gc), _ptr(idc), B, L, C, V, _ptr(dt), _ptr(ws), ws.numel(), _stream())
            _check(rc, "ssamd_rowvec_grad")
            if tdtype != torch.float32:
                dt = dt.to(tdtype)
        return g, dt, None


def add_table_rows(x, table, ids):
    """x [B, L, C] + table[ids[b]] broadcast over L (bf16 out): the speaker embedding (reference
    ``model/fastspeech2.py:39-42,74-77``) gathered inside the add kernel; its backward writes the table
    gradient in place."""
    if x.shape[-1] % 8:
        _torch_fallback(f"add_table_rows C={x.shape[-1]}")
        return x + table[ids].to(x.dtype).unsqueeze(1)
    return _AddTableRowsFn.apply(x, table, ids)


# ------------------------------------------------------------------------ packed <-> padded rows
_SIGS.update({"ssamd_pack_rows": [P, P, P, I, L_, I, I, P, P],
              "ssamd_unpack_rows": [P, P, P, P, I, I, I, I, P, P],
              "ssamd_pad_colsum_ws": [I, I, I],
              "ssamd_pad_colsum": [P, I, P, I, I, I, P, P, L_, P]})
_RESTYPES["ssamd_pad_colsum_ws"] = L_


def _pack_raw(x, pk, pe=None):
    f32 = x.dtype == torch.float32
    xc = x.contiguous() if f32 else x.to(torch.bfloat16).contiguous()
    C = xc.shape[-1]
    assert xc.numel() == pk.B * pk.M * C, "pack_rows: x must be [B, M, C]"
    pec = None if pe is None else pe.to(torch.bfloat16).contiguous()
    if pec is not None:
        assert pec.shape[0] >= pk.M and pec.shape[-1] == C
    out = torch.empty(1, pk.R, C, device=xc.device, dtype=xc.dtype)
    rc = lib().ssamd_pack_rows(_ptr(xc), _ptr(pk.dst), _ptr(pec), pk.M, pk.R, C, int(f32), _ptr(out), _stream())
    _check(rc, "ssamd_pack_rows")
    return out


def _unpack_raw(x, pk, fill=None):
    f32 = x.dtype == torch.float32
    xc = x.contiguous() if f32 else x.to(torch.bfloat16).contiguous()
    C = xc.shape[-1]
    assert xc.numel() == pk.R * C, "unpack_rows: x must be [1, R, C]"
    fc = None if fill is None else fill.detach().float().reshape(C).contiguous()
    out = torch.empty(pk.B, pk.M, C, device=xc.device, dtype=xc.dtype)
    rc = lib().ssamd_unpack_rows(_ptr(xc), _ptr(pk.cu), _ptr(pk.lens), _ptr(fc), pk.B, pk.M, C, int(f32), _ptr(out),
                                 _stream())
    _check(rc, "ssamd_unpack_rows")
    return out


_SIGS.update({"ssamd_repack_rows": [P, P, P, P, I, L_, I, P, I, P, P]})


def _repack_raw(x, src_pk, out_pk, pe=None):
    """Rows of packed layout ``src_pk`` -> packed layout ``out_pk`` (same sequences; an output row
    whose position is past the source length gets 0), + ``pe[t]``."""
    f32 = x.dtype == torch.float32
    xc = x.contiguous() if f32 else x.to(torch.bfloat16).contiguous()
    C = xc.shape[-1]
    assert xc.numel() == src_pk.R * C and src_pk.B == out_pk.B, "repack_rows: x must be [1, R_src, C]"
    pec = None if pe is None else pe.to(torch.bfloat16).contiguous()
    if pec is not None:
        assert pec.shape[0] >= out_pk.M and pec.shape[-1] == C
    out = torch.empty(1, out_pk.R, C, device=xc.device, dtype=xc.dtype)
    rc = lib().ssamd_repack_rows(_ptr(xc), _ptr(src_pk.cu), _ptr(src_pk.lens), _ptr(out_pk.dst), out_pk.M, out_pk.R, C,
                                 _ptr(pec), int(f32), _ptr(out), _stream())
    _check(rc, "ssamd_repack_rows")
    return out


class _RepackRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, src_pk, out_pk, pe):
        ctx.pks, ctx.dtype = (src_pk, out_pk), x.dtype
        return _repack_raw(x, src_pk, out_pk, pe)

    @staticmethod
    def backward(ctx, g):
        src_pk, out_pk = ctx.pks
        gc = g.contiguous() if g.dtype == torch.float32 else g.to(torch.bfloat16).contiguous()
        return _repack_raw(gc, out_pk, src_pk).to(ctx.dtype), None, None, None  # rows not gathered: 0


def repack_rows(x, src_pk, out_pk, pe=None):
    """[1, R_src, C] packed as ``src_pk`` -> [1, R_out, C] packed as ``out_pk`` (+ ``pe[t]``)."""
    if x.shape[-1] % 8 or x.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError(f"repack_rows: C={x.shape[-1]} dtype={x.dtype} not covered by the HIP kernel")
    return _RepackRowsFn.apply(x, src_pk, out_pk, pe)


class _PackRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pk, pe):
        ctx.pk, ctx.dtype = pk, x.dtype
        return _pack_raw(x, pk, pe)

    @staticmethod
    def backward(ctx, g):
        return _unpack_raw(g, ctx.pk).to(ctx.dtype), None, None  # padded rows get zero gradient


class _UnpackRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pk, fill):
        ctx.pk, ctx.dtype = pk, x.dtype
        ctx.fill_dtype = None if fill is None else fill.dtype
        return _unpack_raw(x, pk, fill)

    @staticmethod
    def backward(ctx, g):
        pk = ctx.pk
        gc = g.contiguous() if g.dtype == torch.float32 else g.to(torch.bfloat16).contiguous()
        dx = _pack_raw(gc, pk).to(ctx.dtype)
        dfill = None
        if ctx.fill_dtype is not None and ctx.needs_input_grad[2]:
            C = gc.shape[-1]
            dfill = torch.empty(C, device=g.device, dtype=torch.float32)
            ws = _workspace(g.device, int(lib().ssamd_pad_colsum_ws(pk.B, pk.M, C)))
            rc = lib().ssamd_pad_colsum(_ptr(gc), int(gc.dtype == torch.float32), _ptr(pk.lens), pk.B, pk.M, C,
                                        _ptr(dfill), _ptr(ws), ws.numel(), _stream())
            _check(rc, "ssamd_pad_colsum")
            dfill = dfill.to(ctx.fill_dtype)
        return dx, None, dfill


def pack_rows(x, pk, pe=None):
    """[B, M, C] -> [1, R, C] valid rows (+ ``pe[t]`` at position t); backward scatters, pads get 0."""
    if x.shape[-1] % 8 or x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        _torch_fallback(f"pack_rows C={x.shape[-1]}")
        from .packing import pack

        return pack(x if pe is None else x + pe[: pk.M].to(x.dtype).unsqueeze(0), pk)
    return _PackRowsFn.apply(x, pk, pe)


def unpack_rows(x, pk, fill=None):
    """[1, R, C] -> [B, M, C], padded rows = ``fill`` ([C], default 0; its gradient = column sums of
    the padded rows' gradient, fixed order)."""
    return _UnpackRowsFn.apply(x, pk, fill)
