"""ctypes binding of libprodiff_hip.so (the C-ABI declared in include/prodiff_hip.h).

The product path has no CPU fallback: if the library is missing or fails to
load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PRODIFF_HIP_LIB", os.path.join(_HERE, "libprodiff_hip.so"))

PD_DTYPE_F32 = 0
PD_DTYPE_BF16 = 1
PD_REFLOW = {"euler": 0, "rk2": 1, "rk4": 2, "rk5": 3}
# fd_set_option / nsf_set_option ids (include/prodiff_hip.h)
FD_OPTIONS = {"lvc_ts": 0, "lvc_ts_sub": 1, "lvc_fuse": 2, "lvc_pf": 3, "lvc_sub": 4, "kp_side": 5, "kp_chunk": 7,
               "lvc_tpw": 10, "lvc_prio": 11, "lvc_ps": 14}
NSF_OPTIONS = {"small_max": 0, "wconv": 1, "pair": 2, "pair16": 3, "ups_nc": 4, "rb16": 5, "rb32": 6, "rb64": 7, "c256": 8, "nc_mfma": 9}
WN_OPTIONS = {"layer": 0, "ksplit": 1, "l2pf": 2, "stack": 3, "stack_ro": 4, "stack_fuse": 6, "f32_layer": 7}


class HipError(RuntimeError):
    pass


class pd_wavenet_dims(C.Structure):
    _fields_ = [("in_dims", C.c_int), ("hidden_size", C.c_int), ("residual_layers", C.c_int),
                ("residual_channels", C.c_int), ("dilation_cycle_length", C.c_int)]


class fd_dims(C.Structure):
    _fields_ = [("audio_channels", C.c_int), ("inner_channels", C.c_int),
                ("cond_channels", C.c_int), ("num_blocks", C.c_int),
                ("upsample_ratios", C.c_int * 4), ("lvc_layers_each_block", C.c_int),
                ("lvc_kernel_size", C.c_int), ("kpnet_hidden_channels", C.c_int),
                ("kpnet_conv_size", C.c_int), ("step_embed_in", C.c_int),
                ("step_embed_mid", C.c_int), ("step_embed_out", C.c_int)]


class nsf_dims(C.Structure):
    _fields_ = [("num_mels", C.c_int), ("upsample_initial_channel", C.c_int), ("num_upsamples", C.c_int),
                ("upsample_rates", C.c_int * 6), ("upsample_kernel_sizes", C.c_int * 6), ("resblock", C.c_int),
                ("num_kernels", C.c_int), ("resblock_kernel_sizes", C.c_int * 4), ("num_dilations", C.c_int),
                ("resblock_dilation_sizes", (C.c_int * 4) * 4), ("sampling_rate", C.c_int),
                ("harmonic_num", C.c_int)]


class pd_cond_dims(C.Structure):
    _fields_ = [("vocab_size", C.c_int), ("hidden_size", C.c_int), ("enc_layers", C.c_int),
                ("enc_ffn_kernel_size", C.c_int), ("num_heads", C.c_int), ("num_spk", C.c_int),
                ("num_langs", C.c_int), ("use_dur_embed", C.c_int), ("use_spk_id", C.c_int),
                ("use_gender_id", C.c_int), ("use_lang_id", C.c_int), ("use_voicing_embed", C.c_int),
                ("use_breath_embed", C.c_int), ("rel_pos", C.c_int)]


class pd_cond_inputs(C.Structure):
    _fields_ = [("txt_tokens", C.c_void_p), ("mel2ph", C.c_void_p), ("f0", C.c_void_p), ("lang_seq", C.c_void_p),
                ("spk_embed_id", C.c_void_p), ("spk_mix_embed", C.c_void_p), ("spk_mix_frames", C.c_int),
                ("gender_embed_id", C.c_void_p), ("gender_mix_embed", C.c_void_p), ("gender_mix_frames", C.c_int),
                ("voicing", C.c_void_p), ("breath", C.c_void_p), ("txt_lens", C.c_void_p)]


_VP = C.c_void_p
_SIGS = {
    "pd_last_error": (C.c_char_p, []),
    "pd_version": (C.c_int, []),
    "pd_build_config": (C.c_char_p, []),
    "pd_profile_enable": (C.c_int, [C.c_int]),
    "pd_profile_summary": (C.c_int, [C.c_char_p, C.c_int]),
    "pd_profile_filter": (C.c_int, [C.c_char_p]),
    "pd_wavenet_create": (C.c_int, [C.POINTER(pd_wavenet_dims), C.POINTER(_VP), C.c_int, _VP, C.POINTER(_VP)]),
    "pd_wavenet_destroy": (None, [_VP]),
    "pd_wavenet_set_option": (C.c_int, [_VP, C.c_int, C.c_int]),
    "pd_wavenet_workspace_size": (C.c_size_t, [_VP, C.c_int, C.c_int, C.c_int]),
    "pd_wavenet_forward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, C.c_int, C.c_int, _VP, C.c_size_t, _VP]),
    "pd_prodiff_sample": (C.c_int, [_VP, _VP, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                    C.POINTER(C.c_float), C.c_int, _VP, _VP, C.c_ulonglong, _VP, _VP, _VP,
                                    C.c_int, C.c_int, _VP, C.c_size_t, _VP]),
    "pd_reflow_workspace_size": (C.c_size_t, [_VP, C.c_int, C.c_int, C.c_int, C.c_int]),
    "pd_reflow_sample": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_float, _VP, C.c_ulonglong, _VP, _VP, _VP,
                                   C.c_int, C.c_int, _VP, C.c_size_t, _VP]),
    "pd_reflow_denorm": (C.c_int, [_VP, _VP, _VP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                   _VP, _VP]),
    "fd_create": (C.c_int, [C.POINTER(fd_dims), C.POINTER(_VP), C.c_int, _VP, C.POINTER(_VP)]),
    "fd_destroy": (None, [_VP]),
    "fd_hop": (C.c_int, [_VP]),
    "fd_workspace_size": (C.c_size_t, [_VP, C.c_int, C.c_int, C.c_int]),
    "fd_set_option": (C.c_int, [_VP, C.c_int, C.c_int]),
    "fd_fold_weight_norm": (C.c_int, [_VP, _VP, _VP, C.c_int, C.c_int, _VP]),
    "fd_forward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, C.c_int, C.c_int, _VP, C.c_size_t, _VP]),
    "fd_sample": (C.c_int, [_VP, _VP, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                            C.POINTER(C.c_float), C.c_int, _VP, _VP, C.c_ulonglong, _VP, _VP, _VP, C.c_int,
                            C.c_int, _VP, C.c_size_t, _VP]),
    "fd_sample_coefs": (C.c_int, [_VP, _VP, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                  C.POINTER(C.c_float), C.c_int, _VP, _VP, C.c_ulonglong, _VP, _VP, C.c_int, _VP,
                                  C.c_int, C.c_int, _VP, C.c_size_t, _VP]),
    "fd_draw_x_T": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_ulonglong, _VP, _VP]),
    "pd_cond_num_params": (C.c_int, [C.POINTER(pd_cond_dims)]),
    "pd_cond_create": (C.c_int, [C.POINTER(pd_cond_dims), C.POINTER(_VP), C.c_int, _VP, C.POINTER(_VP)]),
    "pd_cond_destroy": (None, [_VP]),
    "pd_cond_workspace_size": (C.c_size_t, [_VP, C.c_int, C.c_int, C.c_int]),
    "pd_cond_forward": (C.c_int, [_VP, C.POINTER(pd_cond_inputs), _VP, _VP, C.c_int, C.c_int, C.c_int, _VP,
                                  C.c_size_t, _VP]),
    "nsf_num_params": (C.c_int, [C.POINTER(nsf_dims)]),
    "nsf_create": (C.c_int, [C.POINTER(nsf_dims), C.POINTER(_VP), C.c_int, _VP, C.POINTER(_VP)]),
    "nsf_destroy": (None, [_VP]),
    "nsf_hop": (C.c_int, [_VP]),
    "nsf_workspace_size": (C.c_size_t, [_VP, C.c_int, C.c_int]),
    "nsf_set_option": (C.c_int, [_VP, C.c_int, C.c_int]),
    "nsf_forward": (C.c_int, [_VP, _VP, C.c_float, _VP, _VP, _VP, C.c_ulonglong, _VP, _VP, _VP, C.c_int, C.c_int,
                              _VP, C.c_size_t, _VP]),
}
EXPORTS = tuple(_SIGS)

_lib = None


def lib():
    """Load (once) and return the library; raise loudly if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(f"libprodiff_hip.so not found at {LIB_PATH}: run "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().pd_last_error().decode(errors="replace")
        raise HipError(f"libprodiff_hip error {rc}: {msg}")


def fptr(t):
    """Device pointer of a contiguous float32 CUDA(HIP) tensor, or None."""
    if t is None:
        return None
    import torch
    if not t.is_cuda:
        raise HipError("libprodiff_hip needs device tensors (got a CPU tensor)")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise HipError(f"expected contiguous float32 tensor, got {t.dtype} contiguous={t.is_contiguous()}")
    return C.c_void_p(t.data_ptr())


def lptr(t):
    """Device pointer of a contiguous int64 (torch.long) CUDA tensor, or None."""
    if t is None:
        return None
    import torch
    if not t.is_cuda:
        raise HipError("libprodiff_hip needs device tensors (got a CPU tensor)")
    if t.dtype != torch.int64 or not t.is_contiguous():
        raise HipError(f"expected contiguous int64 tensor, got {t.dtype} contiguous={t.is_contiguous()}")
    return C.c_void_p(t.data_ptr())


_UTT_CACHE = {}


def _device_rows(vals, B, device, name, lo, hi):
    """B host ints (checked in [lo, hi]) or a device tensor -> device int32 tensor (cached by value,
    see utt_ids)."""
    import torch
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if torch.is_tensor(vals) and vals.is_cuda:
        t = vals.reshape(-1)
        if t.numel() != B:
            raise HipError(f"{name} holds {t.numel()} values for a batch of {B}")
        if t.device != dev:
            t = t.to(dev)
        return t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()
    t = torch.as_tensor(vals).reshape(-1)
    if t.numel() != B:
        raise HipError(f"{name} holds {t.numel()} values for a batch of {B}")
    if t.numel() and (int(t.min()) < lo or int(t.max()) > hi):
        raise HipError(f"{name} must lie in [{lo}, {hi}]")
    key = (name, str(dev), tuple(int(v) for v in t.tolist()))
    d = _UTT_CACHE.get(key)   # (device tensor, pinned host source)
    if d is None:
        if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise HipError(f"{name}: host values not seen before cannot be copied to the device during a "
                           "graph capture; pass a device int32 tensor (or call once before capturing)")
        if len(_UTT_CACHE) >= 256:
            _UTT_CACHE.pop(next(iter(_UTT_CACHE)))
        h = t.to(torch.int32).contiguous()
        ev = None
        if dev.type == "cuda":
            # pinned source + non_blocking: a pageable copy would block the host until the stream
            # drains (no queuing ahead, no overlap of batches on other streams); the pinned host
            # buffer lives in the cache entry, so it outlives the copy.  The event marks the copy's
            # end on the stream that issued it: a later hit on ANOTHER stream waits for it (ADVICE
            # r05: a job on stream B reusing the key job k just created on a busy stream A read the
            # lengths / utterance ids before A's copy had landed)
            h = h.pin_memory()
            d = h.to(device=dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
        else:
            d = h
        _UTT_CACHE[key] = [d, h, ev]
    else:
        ent = d
        d = ent[0]
        if dev.type == "cuda":
            cur = torch.cuda.current_stream(dev)
            ev = ent[2]
            if ev is not None:
                if ev.query():
                    ent[2] = None           # the copy has landed: no stream needs to wait any more
                elif not torch.cuda.is_current_stream_capturing():
                    cur.wait_event(ev)
                else:
                    raise HipError(f"{name}: the device copy of these values is still in flight on "
                                   "another stream; synchronize before capturing a graph")
            d.record_stream(cur)
    return d


def lens(vals, B, T, device):
    """Ragged batch: each row's utterance length in frames (include/prodiff_hip.h), None (every
    row T frames), B host ints in [1, T], or a device tensor (not range-checked: the kernels clamp
    to T) -> device int32 tensor or None.  All equal to T -> None (the dense path)."""
    if vals is None:
        return None
    import torch
    if not (torch.is_tensor(vals) and vals.is_cuda):
        v = [int(x) for x in (vals.tolist() if torch.is_tensor(vals) else vals)]
        if len(v) == B and all(x == T for x in v):
            return None
        vals = v
    return _device_rows(vals, B, device, "lens", 1, T)


def utt_ids(ids, B, device):
    """Per-row utterance ids for the samplers' Philox draws (include/prodiff_hip.h): None
    (ids 0..B-1) or B ints -> (device int32 tensor or None).  Keep the tensor alive until
    the call's stream work is done (a captured graph keeps it).

    A device int32 tensor must live on the sampler's device (a tensor on another GPU is
    copied there); its values are NOT range-checked (that would read it back to the host),
    and a negative id draws the same noise as the id it wraps to as uint32.  Host ids are
    checked here and their device copy is cached by value: a pageable host-to-device copy
    blocks the host until the stream drains, which left the GPU idle while the host queued
    the next launches (C3 trace r03: ~50 us per sampler call).  Cached tensors are marked
    as in use by the current stream on every hit (record_stream), so an evicted entry is
    not reused by the allocator while another stream's kernels still read it; a cache
    miss is refused while the current stream is capturing a graph (the H2D copy would be
    captured): pass a device tensor or warm the cache before the capture."""
    if ids is None:
        return None
    return _device_rows(ids, B, device, "utt_ids", 0, 2 ** 31 - 1)


def iptr(t):
    """Device pointer of a contiguous int32 tensor, or None."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def farr(vals):
    arr = (C.c_float * len(vals))(*[float(v) for v in vals])
    return arr


def stream_ptr(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def profile_enable(on=True):
    check(lib().pd_profile_enable(1 if on else 0))


def profile_filter(tags=None):
    """Record only these tags (None = all)."""
    check(lib().pd_profile_filter(",".join(tags).encode() if tags else None))


def profile_summary():
    """{tag: (launch count, total ms)} of the launches recorded since profile_enable."""
    l = lib()
    n = l.pd_profile_summary(None, 0)
    if n < 0:
        raise HipError(l.pd_last_error().decode())
    buf = C.create_string_buffer(n + 16)
    l.pd_profile_summary(buf, n + 16)
    out = {}
    for line in buf.value.decode().splitlines():
        tag, cnt, ms = line.split()
        out[tag] = (int(cnt), float(ms))
    return out


class Workspace:
    """Grow-only device scratch buffers (torch caching allocator), one per (device, stream): the
    library's calls are stream-ordered, so calls on different streams -- distributed_synthesize
    runs ragged batches side by side -- must not share scratch (include/prodiff_hip.h: "concurrent
    calls on different streams need separate workspaces").  ``per_stream=False``: one buffer per
    device whatever the stream (a captured graph's workspace: sized by an eager warm-up call, then
    reused by the capture on torch's capture stream; the caller orders the two)."""

    def __init__(self, per_stream=True):
        self.bufs = {}
        self.per_stream = per_stream

    def get(self, nbytes, device):
        import torch
        device = torch.device(device)
        sid = (torch.cuda.current_stream(device).cuda_stream
               if device.type == "cuda" and self.per_stream else 0)
        key = (str(device), sid)
        buf = self.bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self.bufs[key] = buf
        return C.c_void_p(buf.data_ptr()), buf.numel()
