"""SVS teacher with the condition stage on the GPU, drop-in for the reference.

``ProDiffTeacher`` replaces modules/svs/prodiff_teacher.py:10-168: the same
constructor ``(vocab_size, hparams)``, the same child modules and state-dict keys
(``encoder.layers.N.op.self_attn.in_proj_weight``, ``dur_embed.weight``, ...,
``diffusion.denoise_fn.*``), so ``load_ckpt(model, ckpt_dir, 'model')``
(utils/ckpt_utils.py:28-68) fills it unchanged.  ``forward_condition`` -- the
FastspeechEncoder (modules/fastspeech/tts_modules.py:291-330), mel2ph_to_dur,
the length-regulator gather and the pitch / speaker / gender / voicing / breath
embeddings -- runs in ``pd_cond_forward`` (include/prodiff_hip.h), the reverse
process in ``pd_prodiff_sample`` / ``pd_reflow_sample``.  The nn children are
parameter containers; nothing here computes on the CPU and every call raises if
the HIP library is unavailable.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib
from .prodiff import GaussianDiffusion, WaveNet
from .reflow import RectifiedFlow


# ---------------------------------------------------------------- parameter containers
class MultiheadAttention(nn.Module):
    """common_layers.py:172-215 with bias=False, self-attention (qkv_same_dim)."""

    def __init__(self, embed_dim, num_heads):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=False)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.xavier_uniform_(self.out_proj.weight)


class TransformerFFNLayer(nn.Module):
    """common_layers.py:542-555 (SAME padding, gelu)."""

    def __init__(self, hidden_size, filter_size, kernel_size):
        super().__init__()
        self.kernel_size = kernel_size
        self.ffn_1 = nn.Conv1d(hidden_size, filter_size, kernel_size, padding=kernel_size // 2)
        self.ffn_2 = nn.Linear(filter_size, hidden_size)


class EncSALayer(nn.Module):
    """common_layers.py:625-648 (norm 'ln': LayerNorm eps 1e-5, :76-83)."""

    def __init__(self, c, num_heads, kernel_size):
        super().__init__()
        self.layer_norm1 = nn.LayerNorm(c, eps=1e-5)
        self.self_attn = MultiheadAttention(c, num_heads)
        self.layer_norm2 = nn.LayerNorm(c, eps=1e-5)
        self.ffn = TransformerFFNLayer(c, 4 * c, kernel_size)


class TransformerEncoderLayer(nn.Module):
    """tts_modules.py:16-31."""

    def __init__(self, hidden_size, kernel_size, num_heads):
        super().__init__()
        self.op = EncSALayer(hidden_size, num_heads, kernel_size)


class SinusoidalPositionalEmbedding(nn.Module):
    """common_layers.py:94-109: the table is computed on the fly; only the buffer is state."""

    def __init__(self, embedding_dim, padding_idx=0):
        super().__init__()
        self.embedding_dim, self.padding_idx = embedding_dim, padding_idx
        self.register_buffer("_float_tensor", torch.FloatTensor(1))


class RelPositionalEncoding(nn.Module):
    """espnet_positional_embedding.py:89-115: no parameters or buffers (its table is a plain
    attribute there); the encoder kernel computes the table (pd_cond_dims.rel_pos)."""

    def __init__(self, d_model, dropout_rate=0.0, max_len=5000):
        super().__init__()
        self.d_model, self.max_len = d_model, max_len
        # rows of the reference's table: extend_pe (:24-45) regrows it for a longer input and
        # keeps the longer table, so later, shorter batches count their reversed positions from
        # the largest length seen so far; tracked here and passed as pd_cond_dims.rel_pos
        self.pe_len = max_len

    def extend(self, T):
        self.pe_len = max(self.pe_len, int(T))


class FastspeechEncoder(nn.Module):
    """tts_modules.py:291-330 (use_pos_embed False, use_last_norm; rel_pos selects the
    RelPositionalEncoding embedding)."""

    def __init__(self, vocab_size, hidden_size, num_layers, kernel_size, dropout=0.1, num_heads=2, rel_pos=False):
        super().__init__()
        self.rel_pos = bool(rel_pos)
        self.hidden_size, self.num_layers, self.kernel_size, self.num_heads = hidden_size, num_layers, kernel_size, num_heads
        self.layers = nn.ModuleList([TransformerEncoderLayer(hidden_size, kernel_size, num_heads)
                                     for _ in range(num_layers)])
        self.layer_norm = nn.LayerNorm(hidden_size)
        self.embed_tokens = nn.Embedding(vocab_size, hidden_size, padding_idx=0)
        self.embed_scale = math.sqrt(hidden_size)
        self.padding_idx = 0
        self.embed_positions = (RelPositionalEncoding(hidden_size) if self.rel_pos
                                else SinusoidalPositionalEmbedding(hidden_size, 0))

    def ordered_params(self):
        out = []
        for layer in self.layers:
            op = layer.op
            out += [op.layer_norm1.weight, op.layer_norm1.bias, op.self_attn.in_proj_weight,
                    op.self_attn.out_proj.weight, op.layer_norm2.weight, op.layer_norm2.bias,
                    op.ffn.ffn_1.weight, op.ffn.ffn_1.bias, op.ffn.ffn_2.weight, op.ffn.ffn_2.bias]
        return out + [self.layer_norm.weight, self.layer_norm.bias, self.embed_tokens.weight]


# ---------------------------------------------------------------- the teacher
class ProDiffTeacher(nn.Module):
    def __init__(self, vocab_size, hparams):
        super().__init__()
        H = hparams["hidden_size"]
        self.mel_bins = hparams["audio_num_mel_bins"]
        self.vocab_size = vocab_size
        self.encoder = FastspeechEncoder(vocab_size, H, hparams["enc_layers"], hparams["enc_ffn_kernel_size"],
                                         hparams.get("dropout", 0.1), hparams["num_heads"],
                                         rel_pos=hparams.get("rel_pos", False))
        self.with_dur_embed = hparams.get("use_dur_embed", True)
        if self.with_dur_embed:
            self.dur_embed = nn.Linear(1, H)
        self.with_spk_embed = hparams.get("use_spk_id", True)
        if self.with_spk_embed:
            self.spk_embed = nn.Embedding(hparams["num_spk"], H)
        self.with_gender_embed = hparams.get("use_gender_id", False)
        if self.with_gender_embed:
            self.gender_embed = nn.Embedding(2, H)
        self.with_lang_embed = hparams.get("use_lang_id", True)
        if self.with_lang_embed:
            self.lang_embed = nn.Embedding(len(hparams["languages"]) + 1, H, 0)
        self.pitch_embed = nn.Linear(1, H)
        self.with_voicing_embed = hparams.get("use_voicing_embed", False)
        if self.with_voicing_embed:
            self.voicing_embed = nn.Linear(1, H)
        self.with_breath_embed = hparams.get("use_breath_embed", False)
        if self.with_breath_embed:
            self.breath_embed = nn.Linear(1, H)
        self.diffusion_type = hparams.get("diff_type", "prodiff")
        if self.diffusion_type in ("prodiff", "reflow"):
            wn = WaveNet(hparams["audio_num_mel_bins"], H, hparams["residual_layers"], hparams["residual_channels"],
                         hparams["dilation_cycle_length"])
            if self.diffusion_type == "prodiff":
                self.diffusion = GaussianDiffusion(out_dims=hparams["audio_num_mel_bins"], denoise_fn=wn,
                                                   timesteps=hparams["timesteps"], time_scale=hparams["timescale"],
                                                   schedule_type=hparams["schedule_type"],
                                                   max_beta=hparams.get("max_beta", 0.06),
                                                   spec_min=hparams["spec_min"], spec_max=hparams["spec_max"])
            else:
                self.diffusion = RectifiedFlow(out_dims=hparams["audio_num_mel_bins"], denoise_fn=wn,
                                               time_scale=hparams["timescale"], num_features=1,
                                               sampling_algorithm=hparams.get("sampling_algorithm", "euler"),
                                               spec_min=hparams["spec_min"], spec_max=hparams["spec_max"])
        self.compute_dtype = "fp32"
        self._h = None
        self._sig = None
        self._ws = _lib.Workspace()

    def set_compute_dtype(self, dtype):
        """'fp32' (the parity path) or 'bf16' (bf16 MFMA GEMMs, fp32 accumulate) for the condition
        stage and the diffusion."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(dtype)
        self.compute_dtype = dtype
        if hasattr(self, "diffusion"):
            self.diffusion.set_compute_dtype(dtype)
        return self

    # ----------------------------------------------------------- packing
    def cond_dims(self):
        e = self.encoder
        return _lib.pd_cond_dims(
            self.vocab_size, e.hidden_size, e.num_layers, e.kernel_size, e.num_heads,
            self.spk_embed.num_embeddings if self.with_spk_embed else 0,
            self.lang_embed.num_embeddings if self.with_lang_embed else 0,
            int(self.with_dur_embed), int(self.with_spk_embed), int(self.with_gender_embed),
            int(self.with_lang_embed), int(self.with_voicing_embed), int(self.with_breath_embed),
            e.embed_positions.pe_len if e.rel_pos else 0)

    def ordered_cond_params(self):
        """Tensors in the include/prodiff_hip.h pd_cond order (== reference state-dict order)."""
        out = self.encoder.ordered_params()
        if self.with_dur_embed:
            out += [self.dur_embed.weight, self.dur_embed.bias]
        if self.with_spk_embed:
            out.append(self.spk_embed.weight)
        if self.with_gender_embed:
            out.append(self.gender_embed.weight)
        if self.with_lang_embed:
            out.append(self.lang_embed.weight)
        out += [self.pitch_embed.weight, self.pitch_embed.bias]
        if self.with_voicing_embed:
            out += [self.voicing_embed.weight, self.voicing_embed.bias]
        if self.with_breath_embed:
            out += [self.breath_embed.weight, self.breath_embed.bias]
        return out

    def cond_handle(self):
        ps = self.ordered_cond_params()
        sig = (self.compute_dtype, self.cond_dims().rel_pos) + tuple((p.data_ptr(), p._version) for p in ps)
        if self._h is not None and sig == self._sig:
            return self._h
        L = _lib.lib()
        dev = ps[0].device
        if dev.type != "cuda":
            raise _lib.HipError("ProDiffTeacher parameters must live on the GPU (call .cuda())")
        tensors = [p.detach().float().contiguous() for p in ps]
        dims = self.cond_dims()
        if L.pd_cond_num_params(_lib.C.byref(dims)) != len(tensors):
            raise _lib.HipError("parameter count does not match pd_cond_num_params")
        arr = (_lib.C.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
        h = _lib.C.c_void_p()
        dt = _lib.PD_DTYPE_BF16 if self.compute_dtype == "bf16" else _lib.PD_DTYPE_F32
        _lib.check(L.pd_cond_create(_lib.C.byref(dims), arr, dt, _lib.stream_ptr(dev), _lib.C.byref(h)))
        self._release()
        self._h, self._sig = h, sig
        self._keep = tensors
        return h

    def _release(self):
        if self._h is not None:
            torch.cuda.synchronize()
            _lib.lib().pd_cond_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            if self._h is not None:
                _lib.lib().pd_cond_destroy(self._h)
        except Exception:
            pass

    # ----------------------------------------------------------- forward
    @torch.no_grad()
    def forward_condition(self, txt_tokens, mel2ph, f0, lang_seq=None, spk_embed_id=None, spk_mix_embed=None,
                          gender_embed_id=None, gender_mix_embed=None, voicing=None, breath=None,
                          return_encoder=False, txt_lens=None):
        """prodiff_teacher.py:103-146 -> condition [B, T_mel, H].  ``return_encoder`` (not in the
        reference) also returns the FastspeechEncoder output [B, T_txt, H].  ``txt_lens`` (not in the
        reference): each row's phoneme count in a token-padded batch -- every row then equals the
        segment encoded alone (pd_cond_inputs.txt_lens)."""
        if self.with_lang_embed and lang_seq is None:
            raise AssertionError("use_lang_embed is True, lang_seq is required")
        if self.with_spk_embed and spk_embed_id is None and spk_mix_embed is None:
            raise AssertionError("spk_embed_id or spk_mix_embed is required")
        if self.with_gender_embed and gender_embed_id is None and gender_mix_embed is None:
            raise AssertionError("gender_embed_id or gender_mix_embed is required")
        if self.encoder.rel_pos:
            self.encoder.embed_positions.extend(txt_tokens.shape[1])
        h = self.cond_handle()
        dev = txt_tokens.device
        B, Tt = txt_tokens.shape
        Tm = mel2ph.shape[1]
        H = self.encoder.hidden_size
        lng = lambda t: None if t is None else t.to(dev).long().reshape(t.shape[0], -1).contiguous()
        flt = lambda t: None if t is None else t.to(dev).float().contiguous()
        tok, m2p, lang = lng(txt_tokens), lng(mel2ph), lng(lang_seq)
        spk_id = None if spk_embed_id is None else spk_embed_id.to(dev).long().reshape(B).contiguous()
        gen_id = None if gender_embed_id is None else gender_embed_id.to(dev).long().reshape(B).contiguous()
        smix = None if spk_mix_embed is None else flt(spk_mix_embed.reshape(B, -1, H))
        gmix = None if gender_mix_embed is None else flt(gender_mix_embed.reshape(B, -1, H))
        f0_, vo, br = flt(f0), flt(voicing), flt(breath)
        tl = _lib.lens(txt_lens, B, Tt, dev)
        keep = (tok, m2p, lang, spk_id, gen_id, smix, gmix, f0_, vo, br, tl)
        vp = lambda t: None if t is None else t.data_ptr()
        ins = _lib.pd_cond_inputs(vp(tok), vp(m2p), vp(f0_), vp(lang), vp(spk_id), vp(smix),
                                  0 if smix is None else smix.shape[1], vp(gen_id), vp(gmix),
                                  0 if gmix is None else gmix.shape[1], vp(vo), vp(br), vp(tl))
        cond = torch.empty(B, Tm, H, device=dev, dtype=torch.float32)
        enc = torch.empty(B, Tt, H, device=dev, dtype=torch.float32) if return_encoder else None
        L = _lib.lib()
        nbytes = L.pd_cond_workspace_size(h, B, Tt, Tm)
        ws, wsb = self._ws.get(nbytes, dev)
        _lib.check(L.pd_cond_forward(h, _lib.C.byref(ins), _lib.fptr(cond), _lib.fptr(enc), B, Tt, Tm, ws, wsb,
                                     _lib.stream_ptr(dev)))
        del keep
        return (cond, enc) if return_encoder else cond

    def forward(self, txt_tokens, mel2ph, f0, lang_seq=None, spk_embed_id=None, spk_mix_embed=None,
                gender_embed_id=None, gender_mix_embed=None, voicing=None, breath=None, gt_spec=None, infer=False):
        """prodiff_teacher.py:148-168 (inference only)."""
        if not infer:
            raise NotImplementedError("training (infer=False) is out of scope")
        condition = self.forward_condition(txt_tokens, mel2ph, f0, lang_seq=lang_seq, spk_embed_id=spk_embed_id,
                                           spk_mix_embed=spk_mix_embed, gender_embed_id=gender_embed_id,
                                           gender_mix_embed=gender_mix_embed, voicing=voicing, breath=breath)
        return self.diffusion(condition, infer=True)
