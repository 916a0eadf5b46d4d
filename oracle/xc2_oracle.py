"""CPU oracle for the XCodec2 codec decoder (TEST INFRASTRUCTURE ONLY).

Restates ``AudioTokenizer.decode`` (reference data/tokenizer.py:117-123 -> pip
xcodec2 0.1.7 ``decode_code``) in plain fp32 PyTorch CPU ops, following the
transformers port that SURVEY 8(c)#4 names as the architecture oracle
([tf] = transformers/models/xcodec2/modeling_xcodec2.py, transformers 5.15):

  decode                     [tf] Xcodec2Model.decode :1028-1049
  fsq_codes                  [tf] Xcodec2FiniteScalarQuantization._indices_to_codes :692-700
  project_out / fc / embed   [tf] Xcodec2Quantizer.from_codes :806-809, Xcodec2Decoder :838-843
  resnet_block               [tf] Xcodec2ResNetBlock.forward :650-661
  transformer layer          [tf] Xcodec2DecoderLayer :344-373, Xcodec2Attention :268-310,
                             RMSNorm :322-327, MLP :164-168, RoPE over heads :855-857
  istft_head                 [tf] Xcodec2ISTFTHead.forward :763-796

Pinning: tests/golden/make_golden_codec.py runs the transformers Xcodec2Model itself on
the same seeded weights and commits its waveforms; tests/test_codec_cpu.py checks this
restatement against them. Parity against the pip xcodec2 package itself is UNPINNED
(package and checkpoints absent; the reference holds no codec fixtures).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this file.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F

F32 = torch.float32


def fsq_codes(idx: torch.Tensor, levels: Sequence[int]) -> torch.Tensor:
    """ids -> per-dimension codes in [-1, 1] ([tf] :692-700). Ids reduce modulo
    prod(levels) by the digit formula (pip package behaviour; the HF port's
    ``codebook[idx]`` would raise for ids >= 65536)."""
    lv = torch.tensor(list(levels), dtype=torch.int64)
    basis = torch.cumprod(torch.tensor([1] + list(levels[:-1]), dtype=torch.int64), 0)
    digits = (idx.long().unsqueeze(-1) // basis) % lv
    half = lv // 2
    return (digits - half) / half          # int / int -> float32 true division


def rms_norm(x, w, eps):
    v = x.pow(2).mean(-1, keepdim=True)
    return w * (x * torch.rsqrt(v + eps))


def resnet_block(x, sd, p, eps=1e-6):
    """x [B, T, C] -> [B, T, C]; GroupNorm(32) + SiLU + Conv1d(k3, pad 1), twice, + residual."""
    h = x.transpose(1, 2)
    r = h
    h = F.silu(F.group_norm(h, 32, sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps))
    h = F.conv1d(h, sd[p + "conv1.weight"], sd[p + "conv1.bias"], padding=1)
    h = F.silu(F.group_norm(h, 32, sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps))
    h = F.conv1d(h, sd[p + "conv2.weight"], sd[p + "conv2.bias"], padding=1)
    return (h + r).transpose(1, 2)


def head_rope(n_heads: int, head_dim: int, theta: float):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=F32) / head_dim))
    pos = torch.arange(n_heads, dtype=F32)
    fr = (inv[None, :, None] @ pos[None, None, :]).transpose(1, 2)      # [1, H, hd/2]
    emb = torch.cat((fr, fr), -1)
    return emb.cos(), emb.sin()                                          # [1, H, hd]


def rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), -1)


def attention_layer(x, sd, p, n_heads, cos, sin, eps):
    B, T, Cd = x.shape
    hd = Cd // n_heads
    h = rms_norm(x, sd[p + "input_layernorm.weight"], eps)
    q = (h @ sd[p + "self_attn.q_proj.weight"].T).view(B, T, n_heads, hd).transpose(1, 2)
    k = (h @ sd[p + "self_attn.k_proj.weight"].T).view(B, T, n_heads, hd).transpose(1, 2)
    v = (h @ sd[p + "self_attn.v_proj.weight"].T).view(B, T, n_heads, hd).transpose(1, 2)
    c, s = cos.unsqueeze(2), sin.unsqueeze(2)          # [1, H, 1, hd]: angle depends on the head
    q = q * c + rotate_half(q) * s
    k = k * c + rotate_half(k) * s
    a = F.scaled_dot_product_attention(q, k, v, scale=hd ** -0.5)
    a = a.transpose(1, 2).reshape(B, T, Cd)
    x = x + a @ sd[p + "self_attn.o_proj.weight"].T
    h = rms_norm(x, sd[p + "post_attention_layernorm.weight"], eps)
    h = F.silu(h @ sd[p + "mlp.fc1.weight"].T) @ sd[p + "mlp.fc2.weight"].T
    return x + h


def istft_head(x, sd, n_fft: int, hop: int):
    """x [B, T, C] -> wav [B, T * hop] ([tf] :763-796)."""
    spec = (x @ sd["acoustic_decoder.head.linear.weight"].T + sd["acoustic_decoder.head.linear.bias"])
    spec = spec.transpose(1, 2)
    mag, ph = spec.chunk(2, dim=1)
    mag = torch.exp(mag).clamp(max=1e2)
    S = torch.polar(mag, ph)
    frames = torch.fft.irfft(S, n_fft, dim=1, norm="backward")
    win = torch.hann_window(n_fft, dtype=F32)
    frames = frames * win[None, :, None]
    T = S.shape[-1]
    pad = (n_fft - hop) // 2
    out_size = (T - 1) * hop + n_fft
    audio = F.fold(frames, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0, pad:-pad]
    env = F.fold(win.square().expand(1, T, -1).transpose(1, 2), output_size=(1, out_size),
                 kernel_size=(1, n_fft), stride=(1, hop)).squeeze()[pad:-pad]
    return audio / env.clamp(min=1e-11)


@torch.no_grad()
def decode(sd: Dict[str, torch.Tensor], codes: torch.Tensor, cfg, lens: Optional[Sequence[int]] = None):
    """codes [B, T] int -> wav [B, 1, T * hop] fp32 (rows past lens[b] * hop are zero:
    each row is decoded on its own, as the reference decodes one utterance at a time)."""
    sd = {k: v.to(F32) for k, v in sd.items()}
    B, T = codes.shape
    if lens is not None:
        out = torch.zeros(B, 1, T * cfg.hop_length)
        for b in range(B):
            n = int(lens[b])
            out[b, :, :n * cfg.hop_length] = decode(sd, codes[b:b + 1, :n], cfg)[0]
        return out
    x = fsq_codes(codes, cfg.quantization_levels)
    x = x @ sd["quantizer.project_out.weight"].T + sd["quantizer.project_out.bias"]
    x = x @ sd["acoustic_decoder.fc.weight"].T + sd["acoustic_decoder.fc.bias"]
    x = F.conv1d(x.transpose(1, 2), sd["acoustic_decoder.embed.weight"], sd["acoustic_decoder.embed.bias"],
                 padding=3).transpose(1, 2)
    for i in range(2):
        x = resnet_block(x, sd, f"acoustic_decoder.prior_net.{i}.")
    cos, sin = head_rope(cfg.num_attention_heads, cfg.head_dim, cfg.rope_theta)
    for i in range(cfg.num_hidden_layers):
        x = attention_layer(x, sd, f"acoustic_decoder.layers.{i}.", cfg.num_attention_heads, cos, sin,
                            cfg.rms_norm_eps)
    for i in range(2):
        x = resnet_block(x, sd, f"acoustic_decoder.post_net.{i}.")
    x = F.layer_norm(x, (x.shape[-1],), sd["acoustic_decoder.norm.weight"], sd["acoustic_decoder.norm.bias"], 1e-6)
    return istft_head(x, sd, cfg.n_fft, cfg.hop_length).unsqueeze(1)
