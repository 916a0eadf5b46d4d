"""CPU oracle for the T5Gemma-TTS generate() hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The product path
(``t5gemma_tts_amd``) never imports, links or executes anything under ``oracle/``.

It is a from-scratch restatement, in plain PyTorch CPU ops, of the reference
algorithm (tori29umai0123/T5Gemma-TTS @ 2025-12-26):

* ``T5GemmaVoiceForConditionalGeneration.inference_tts``
  (``hf_export/modeling_t5gemma_voice.py:565-862``; identical copy
  ``models/t5gemma.py:835-1129``) -- encoder, prefill, AR loop, stop rules;
* the sampler ``topk_sampling`` / ``top_k_top_p_filtering`` (``:84-138``,
  ``models/utils.py:53-122``) with ``torch.multinomial(p, 1)`` restated as
  ``argmax(p / q)``, ``q = empty_like(p).exponential_(1)`` (ATen's own
  single-sample algorithm), so the noise can be injected and uploaded to the GPU;
* the T5Gemma backbone arithmetic of transformers' T5Gemma modules
  (third-party; reference pins 4.57.3, this container runs 5.15):
  RMSNorm(1+w), GeGLU-tanh MLP, GQA attention via SDPA (softcap only on the
  eager path), RoPE with *float* PM-RoPE progress positions
  (``:516-531, :669-681, :817-832``), PM cross-attention (``:141-253``).

Parity pinning: ``tests/golden/make_golden.py`` imports the reference itself in
this container and records token ids / logits; ``tests/test_oracle_golden.py``
checks this oracle reproduces them bit-for-bit.

Every op is chosen to issue the same ATen kernel the reference issues (same
dtype, same SDPA argument pattern incl. mask-None / ``enable_gqa``), so results
are bitwise identical to the reference for the same thread count.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


# ----------------------------------------------------------------------------
# backbone primitives ([tf] modeling_t5gemma.py)
# ----------------------------------------------------------------------------
def _acc(dt: torch.dtype) -> torch.dtype:
    """The type the reference's fp32 steps run in: fp32, or fp64 for the fp64 restatement."""
    return torch.float64 if dt == torch.float64 else torch.float32


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """T5GemmaRMSNorm ([tf] :61-78): fp32 normalise, scale by (1 + w), cast back."""
    ct = _acc(x.dtype)
    xf = x.to(ct)
    out = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    out = out * (1.0 + w.to(ct))
    return out.type_as(x)


def inv_freq_table(head_dim: int, theta: float, dtype=torch.float) -> torch.Tensor:
    """Default RoPE inverse frequencies ([tf] :114-137)."""
    return 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=dtype) / head_dim))


def rope_cos_sin(inv_freq: torch.Tensor, pos: torch.Tensor, dtype=BF16) -> Tuple[torch.Tensor, torch.Tensor]:
    """T5GemmaRotaryEmbedding.forward ([tf] :138-151) on float positions [B, T]."""
    B = pos.shape[0]
    ct = _acc(dtype)
    inv = inv_freq[None, :, None].to(ct).expand(B, -1, 1)
    p = pos[:, None, :].to(ct)
    freqs = (inv @ p).transpose(1, 2)
    emb = torch.cat((freqs, freqs), dim=-1)
    cos = emb.cos() * 1.0
    sin = emb.sin() * 1.0
    return cos.to(dtype), sin.to(dtype)


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B,H,T,D], cos/sin [B,T,D] -> x*cos + rotate_half(x)*sin (bf16 ops)."""
    c = cos.unsqueeze(1)
    s = sin.unsqueeze(1)
    return (x * c) + (rotate_half(x) * s)


def repeat_kv(x: torch.Tensor, n_rep: int) -> torch.Tensor:
    if n_rep == 1:
        return x
    b, h, s, d = x.shape
    return x[:, :, None, :, :].expand(b, h, n_rep, s, d).reshape(b, h * n_rep, s, d)


def attention(q, k, v, *, scale: float, softcap: float, n_rep: int,
              mask: Optional[torch.Tensor], is_causal: bool, impl: str) -> torch.Tensor:
    """Attention as the reference dispatches it.

    * ``impl == 'sdpa'``: transformers' ``sdpa_attention_forward`` -- GQA via
      ``enable_gqa`` when the mask is None, else ``repeat_kv``; softcap ignored.
    * ``impl == 'eager'``: ``eager_attention_forward`` ([tf] :199-230) with tanh softcap.
    ``mask``: bool [1,1,Tq,Tk] (True = attend) or None. Returns [B, Tq, H*D].
    """
    B, H, Tq, D = q.shape
    if impl == "sdpa":
        kw = {}
        if n_rep > 1:
            if mask is None and k.shape[-1] <= 256:
                kw = {"enable_gqa": True}
            else:
                k = repeat_kv(k, n_rep)
                v = repeat_kv(v, n_rep)
        causal = bool(is_causal and Tq > 1 and mask is None)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=0.0,
                                           scale=scale, is_causal=causal, **kw)
    else:
        k = repeat_kv(k, n_rep)
        v = repeat_kv(v, n_rep)
        w = torch.matmul(q, k.transpose(2, 3)) * scale
        if softcap:
            w = w / softcap
            w = torch.tanh(w)
            w = w * softcap
        if mask is None and is_causal and Tq > 1:
            Tk = k.shape[2]
            mask = (torch.arange(Tq)[:, None] + (Tk - Tq) >= torch.arange(Tk)[None, :]).view(1, 1, Tq, Tk)
        if mask is not None:
            add = torch.zeros(mask.shape, dtype=w.dtype)
            add = add.masked_fill(~mask, torch.finfo(w.dtype).min)
            w = w + add
        w = F.softmax(w, dim=-1, dtype=_acc(q.dtype)).to(q.dtype)
        o = torch.matmul(w, v)
    return o.transpose(1, 2).reshape(B, Tq, H * D)


# ----------------------------------------------------------------------------
# sampler (hf_export/modeling_t5gemma_voice.py:84-138, 702-786)
# ----------------------------------------------------------------------------
def top_k_top_p_filtering(logits: torch.Tensor, top_k: int = 0, top_p: float = 1.0,
                          min_p: float = 0.0, filter_value: float = -float("inf"),
                          min_tokens_to_keep: int = 1) -> torch.Tensor:
    """Restatement of ``top_k_top_p_filtering`` (:84-130), 1-D or [B, V] logits.

    NB: like the reference, the top-k step fills ``logits`` IN PLACE.
    """
    if 0.0 < min_p < 1.0:
        probs = F.softmax(logits, dim=-1)
        remove = probs < min_p
        if torch.all(remove.sum(-1) < logits.size(-1)):
            logits = logits.masked_fill(remove, filter_value)
            top_k = 0
            top_p = 1.0
    if isinstance(top_k, int) and top_k > 0:
        k = min(max(top_k, min_tokens_to_keep), logits.size(-1))
        thr = torch.topk(logits, k, dim=-1)[0][..., -1, None]
        logits[logits < thr] = filter_value
    if top_p < 1.0:
        s_logits, s_idx = torch.sort(logits, descending=True)
        cum = torch.cumsum(F.softmax(s_logits, dim=-1), dim=-1)
        s_remove = cum > top_p
        if min_tokens_to_keep > 1:
            s_remove[..., :min_tokens_to_keep] = 0
        s_remove[..., 1:] = s_remove[..., :-1].clone()
        s_remove[..., 0] = 0
        remove = torch.zeros_like(logits, dtype=torch.bool)
        remove.scatter_(dim=-1, index=s_idx, src=s_remove)
        logits = logits.masked_fill(remove, filter_value)
    return logits


def draw_noise(gen: torch.Generator, V: int) -> torch.Tensor:
    """The exponential draw ``torch.multinomial(p, 1)`` makes internally on CPU
    (``q = at::empty_like(self).exponential_(1, gen)``, self = bf16 probs [V])."""
    return torch.empty(V, dtype=BF16).exponential_(1, generator=gen)


def multinomial_from_noise(probs: torch.Tensor, noise: torch.Tensor) -> int:
    """``torch.multinomial(probs, 1)`` given its exponential draw: argmax(p / q)."""
    return int(torch.argmax(probs / noise).item())


@dataclasses.dataclass
class SamplerParams:
    top_k: Union[int, List[int]] = 30
    top_p: float = 0.9
    min_p: float = 0.0
    temperature: float = 0.8
    stop_repetition: int = 3
    silence_tokens: Sequence[int] = ()
    # throughput mode: never accept EOS before the time budget
    eos_disabled: bool = False


@dataclasses.dataclass
class RowState:
    """Per-utterance AR-loop state (the locals of ``inference_tts``)."""
    cur_num_gen: int = 0
    current_length: int = 0
    prompt_offset: int = 0
    target_total: Optional[int] = None
    est_total: int = 0
    prev_token: int = -1
    consec_silence: int = 0
    first_input_len: int = 0


def sample_helper(logits: torch.Tensor, p: SamplerParams, st: RowState, noise: torch.Tensor,
                  *, eos: int, encodec_sr: float, extra_cutoff: float,
                  text_guard_frames_per_token: int = 0) -> Tuple[int, Dict]:
    """One AR sampling step (:702-786). ``logits`` bf16 [V] is edited in place.

    Returns (token_id, info) and advances the silence state in ``st``
    (cur_num_gen / current_length are advanced by the caller, like the reference).
    """
    effective_length = max(0, st.current_length - st.prompt_offset)
    la = logits
    if effective_length == 0:
        la[eos] = -1e9
    kk = p.top_k[min(len(p.top_k) - 1, st.cur_num_gen)] if isinstance(p.top_k, list) else p.top_k
    if st.cur_num_gen <= encodec_sr // 5:
        la[eos] = -10000.0
    if p.eos_disabled:
        la[eos] = -float("inf")
    if (p.stop_repetition > 0 and st.prev_token in p.silence_tokens
            and st.consec_silence > p.stop_repetition):
        f = st.consec_silence - (p.stop_repetition - 1)
        if la[st.prev_token] < 0:
            la[st.prev_token] = la[st.prev_token] * f
        else:
            la[st.prev_token] = la[st.prev_token] / f
    # topk_sampling (:133-138)
    x = la
    if p.temperature != 1.0:
        x = x / p.temperature
    x = top_k_top_p_filtering(x, top_k=kk, top_p=p.top_p, min_p=p.min_p)
    probs = F.softmax(x, dim=-1)
    token = multinomial_from_noise(probs, noise)
    argmax_tok = int(torch.argmax(logits).item())
    force = token == eos or argmax_tok == eos
    if text_guard_frames_per_token > 0:
        force = force or effective_length > max(1, st.first_input_len) * text_guard_frames_per_token
    budget = st.target_total is not None and st.cur_num_gen > (
        st.target_total - st.prompt_offset + int(encodec_sr) * extra_cutoff)
    sampled = token
    if force or budget:
        token = eos
    if token in set(p.silence_tokens) and token == st.prev_token:
        st.consec_silence += 1
    else:
        st.consec_silence = 0
    st.prev_token = token
    return token, {"sampled": sampled, "argmax": argmax_tok, "force": force, "budget": budget}


# ----------------------------------------------------------------------------
# the model
# ----------------------------------------------------------------------------
class T5GemmaTTSOracle:
    """Encoder / decoder / head of T5Gemma-TTS on CPU in bf16 (reference numerics).

    ``dtype=torch.float64``: the same graph with every tensor and every fp32 step in fp64 --
    the noise-floor yardstick of tests/test_gpu_noise_floor.py (not a reference run)."""

    def __init__(self, cfg, sd: Dict[str, torch.Tensor], dtype: torch.dtype = BF16):
        self.cfg = cfg
        self.bb = cfg.backbone
        self.dt = dtype
        self.w = {k: v.to(dtype).contiguous() for k, v in sd.items()}
        self.inv_freq = inv_freq_table(self.bb.head_dim, self.bb.rope_theta, _acc(dtype))
        self.n_rep = self.bb.num_attention_heads // self.bb.num_key_value_heads
        self.enc_types = self.bb.layer_types("encoder")
        self.dec_types = self.bb.layer_types("decoder")
        self.normalizer = torch.tensor(self.bb.hidden_size ** 0.5, dtype=dtype)

    # -- helpers -----------------------------------------------------------
    def _lin(self, x, name, bias=None):
        return F.linear(x, self.w[name], self.w[bias] if bias else None)

    def _mlp(self, x, p):
        g = self._lin(x, f"{p}.mlp.gate_proj.weight")
        u = self._lin(x, f"{p}.mlp.up_proj.weight")
        return self._lin(F.gelu(g, approximate="tanh") * u, f"{p}.mlp.down_proj.weight")

    def _heads(self, x, n):
        B, T, _ = x.shape
        return x.view(B, T, n, self.bb.head_dim).transpose(1, 2)

    def _attn(self, q, k, v, mask, causal):
        return attention(q, k, v, scale=self.bb.attn_scale, softcap=self.bb.softcap,
                         n_rep=self.n_rep, mask=mask, is_causal=causal,
                         impl=self.bb.attn_implementation)

    # -- positions (:508-531, :669-681, :817-832) ----------------------------
    def encoder_positions(self, x_len: int, T: int) -> torch.Tensor:
        lengths = torch.tensor([x_len])
        pos = torch.arange(T, dtype=torch.float32)[None, :]
        denom = (lengths.clamp(min=2).to(torch.float32) - 1.0)[:, None]
        position_ids = pos / denom * self.cfg.progress_scale
        mask = pos < lengths[:, None]
        return position_ids.masked_fill(~mask, 0.0)

    def prefill_positions(self, cur_len: int, est_total: int) -> torch.Tensor:
        base = torch.arange(cur_len, dtype=torch.float32).unsqueeze(0)
        return base / max(1, est_total - 1) * self.cfg.progress_scale

    def step_position(self, current_length: int, est_total: int) -> torch.Tensor:
        v = float(current_length - 1) / max(1, est_total - 1) * self.cfg.progress_scale
        v = min(v, self.cfg.progress_scale)
        return torch.tensor([[v]], dtype=torch.float32)

    # -- encoder ([tf] T5GemmaEncoder.forward :648-702) ----------------------
    def encode(self, x_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """x_ids int64 [T] (no padding). Returns memory [1,T,d] bf16, enc positions [1,T]."""
        T = int(x_ids.shape[0])
        pos = self.encoder_positions(T, T)
        h = F.embedding(x_ids[None], self.w["backbone.model.encoder.embed_tokens.weight"])
        h = h * self.normalizer
        cos, sin = rope_cos_sin(self.inv_freq, pos, self.dt)
        eps = self.bb.rms_norm_eps
        W = self.bb.sliding_window
        for i, lt in enumerate(self.enc_types):
            p = f"backbone.model.encoder.layers.{i}"
            r = h
            x = rms_norm(h, self.w[f"{p}.pre_self_attn_layernorm.weight"], eps)
            q = self._heads(self._lin(x, f"{p}.self_attn.q_proj.weight"), self.bb.num_attention_heads)
            k = self._heads(self._lin(x, f"{p}.self_attn.k_proj.weight"), self.bb.num_key_value_heads)
            v = self._heads(self._lin(x, f"{p}.self_attn.v_proj.weight"), self.bb.num_key_value_heads)
            q = apply_rope(q, cos, sin)
            k = apply_rope(k, cos, sin)
            mask = None
            if lt == "sliding_attention" and T >= W:
                idx = torch.arange(T)
                mask = ((idx[:, None] - idx[None, :]).abs() <= W).view(1, 1, T, T)
            a = self._attn(q, k, v, mask, False)
            a = self._lin(a, f"{p}.self_attn.o_proj.weight")
            h = r + rms_norm(a, self.w[f"{p}.post_self_attn_layernorm.weight"], eps)
            r = h
            x = rms_norm(h, self.w[f"{p}.pre_feedforward_layernorm.weight"], eps)
            x = self._mlp(x, p)
            h = r + rms_norm(x, self.w[f"{p}.post_feedforward_layernorm.weight"], eps)
        h = rms_norm(h, self.w["backbone.model.encoder.norm.weight"], eps)
        return h, pos

    # -- decoder ([tf] T5GemmaDecoder.forward :732-812 + PMDecoderLayer) -------
    def new_cache(self):
        n = self.bb.num_decoder_layers
        return {"k": [None] * n, "v": [None] * n, "ck": [None] * n, "cv": [None] * n, "len": 0}

    def decode(self, emb: torch.Tensor, pos: torch.Tensor, memory: torch.Tensor,
               enc_pos: torch.Tensor, cache) -> torch.Tensor:
        """emb bf16 [1,T,d] (already audio_embedding rows), pos fp32 [1,T] PM positions.
        Appends to ``cache``; returns last hidden [1,T,d] after the final norm."""
        T = emb.shape[1]
        past = cache["len"]
        h = emb * self.normalizer
        cos, sin = rope_cos_sin(self.inv_freq, pos, self.dt)
        eps = self.bb.rms_norm_eps
        W = self.bb.sliding_window
        Hq, Hk = self.bb.num_attention_heads, self.bb.num_key_value_heads
        for i, lt in enumerate(self.dec_types):
            p = f"backbone.model.decoder.layers.{i}"
            # self-attention with cache append
            r = h
            x = rms_norm(h, self.w[f"{p}.pre_self_attn_layernorm.weight"], eps)
            q = self._heads(self._lin(x, f"{p}.self_attn.q_proj.weight"), Hq)
            k = self._heads(self._lin(x, f"{p}.self_attn.k_proj.weight"), Hk)
            v = self._heads(self._lin(x, f"{p}.self_attn.v_proj.weight"), Hk)
            q = apply_rope(q, cos, sin)
            k = apply_rope(k, cos, sin)
            if cache["k"][i] is None:
                cache["k"][i], cache["v"][i] = k, v
            else:
                cache["k"][i] = torch.cat([cache["k"][i], k], dim=-2)
                cache["v"][i] = torch.cat([cache["v"][i], v], dim=-2)
            K, Vv = cache["k"][i], cache["v"][i]
            L = K.shape[2]
            mask = None
            if lt == "sliding_attention" and L >= W:
                # DynamicSlidingWindowLayer keeps the last W-1 keys (+ current): same math
                qi = torch.arange(past, past + T)[:, None]
                ki = torch.arange(L)[None, :]
                mask = ((ki <= qi) & (ki > qi - W)).view(1, 1, T, L)
                if T == 1:
                    # DynamicSlidingWindowLayer.update returns the last W-1 cached keys
                    # + the new one; the mask over them is all-true but still explicit
                    K, Vv, mask = K[:, :, L - W:], Vv[:, :, L - W:], mask[..., L - W:]
            a = self._attn(q, K, Vv, mask, True)
            a = self._lin(a, f"{p}.self_attn.o_proj.weight")
            h = r + rms_norm(a, self.w[f"{p}.post_self_attn_layernorm.weight"], eps)
            # PM cross-attention (:167-253)
            r = h
            x = rms_norm(h, self.w[f"{p}.pre_cross_attn_layernorm.weight"], eps)
            q = self._heads(self._lin(x, f"{p}.cross_attn.q_proj.weight"), Hq)
            if self.cfg.use_pm_rope:
                q = apply_rope(q, cos, sin)
            if cache["ck"][i] is None:
                ck = self._heads(self._lin(memory, f"{p}.cross_attn.k_proj.weight"), Hk)
                if self.cfg.use_pm_rope:
                    ec, es = rope_cos_sin(self.inv_freq, enc_pos, self.dt)
                    ck = apply_rope(ck, ec, es)
                cv = self._heads(self._lin(memory, f"{p}.cross_attn.v_proj.weight"), Hk)
                cache["ck"][i], cache["cv"][i] = ck, cv
            a = self._attn(q, cache["ck"][i], cache["cv"][i], None, False)
            a = self._lin(a, f"{p}.cross_attn.o_proj.weight")
            h = r + rms_norm(a, self.w[f"{p}.post_cross_attn_layernorm.weight"], eps)
            # MLP
            r = h
            x = rms_norm(h, self.w[f"{p}.pre_feedforward_layernorm.weight"], eps)
            x = self._mlp(x, p)
            h = r + rms_norm(x, self.w[f"{p}.post_feedforward_layernorm.weight"], eps)
        cache["len"] = past + T
        return rms_norm(h, self.w["backbone.model.decoder.norm.weight"], eps)

    def embed_audio(self, ids: torch.Tensor) -> torch.Tensor:
        return F.embedding(ids, self.w["audio_embedding.0.weight"])

    def head(self, hidden: torch.Tensor) -> torch.Tensor:
        """predict_layer[0] (:469-478): Linear -> GELU(erf) -> Linear. [.., d] -> [.., V]."""
        h = self._lin(hidden, "predict_layer.0.0.weight", "predict_layer.0.0.bias")
        h = F.gelu(h)
        return self._lin(h, "predict_layer.0.2.weight", "predict_layer.0.2.bias")

    # -- the generate loop (:565-862), one utterance -------------------------
    def prepare(self, x_ids, y_prompt, tgt_y_len: Optional[int], prompt_frames: Optional[int] = None):
        cfg = self.cfg
        x_ids = torch.as_tensor(x_ids, dtype=torch.long).view(-1)
        y = torch.as_tensor(y_prompt, dtype=torch.long).view(-1)
        if cfg.special_first:
            y = y + int(cfg.n_special)
        memory, enc_pos = self.encode(x_ids)
        y_len = int(y.shape[0])
        pf = y_len if prompt_frames is None else int(prompt_frames)
        cated = torch.cat([torch.tensor([cfg.empty_token]), y])
        cur_len = int(cated.shape[0])
        st = RowState(current_length=cur_len, prompt_offset=pf + 1,
                      target_total=None if tgt_y_len is None else int(tgt_y_len),
                      first_input_len=int(x_ids.shape[0]))
        if st.target_total is not None:
            est = st.target_total + 1
        else:
            est = int(cur_len + int(cfg.encodec_sr) * cfg.progress_lookahead_secs)
        st.est_total = max(est, cur_len)
        cache = self.new_cache()
        pos = self.prefill_positions(cur_len, st.est_total)
        hid = self.decode(self.embed_audio(cated[None]), pos, memory, enc_pos, cache)
        return {"memory": memory, "enc_pos": enc_pos, "cache": cache, "last": hid[:, -1:, :],
                "state": st, "y": y}

    def advance(self, ctx, token_id: int) -> None:
        st = ctx["state"]
        pos = self.step_position(st.current_length, st.est_total)
        emb = self.embed_audio(torch.tensor([[token_id]]))
        ctx["last"] = self.decode(emb, pos, ctx["memory"], ctx["enc_pos"], ctx["cache"])

    def step_logits(self, ctx) -> torch.Tensor:
        return self.head(ctx["last"]).squeeze(0).squeeze(0)

    def generate(self, x_ids, y_prompt, tgt_y_len, params: SamplerParams, seed: Optional[int] = None,
                 noise_fn=None, prompt_frames=None, record_logits: bool = False,
                 max_steps: Optional[int] = None):
        """inference_tts for one utterance. Noise: torch CPU generator reseeded with
        ``seed`` right before the loop (SURVEY a14' step 8), or ``noise_fn(step)``.
        Returns dict(res, gen, logits?)."""
        cfg = self.cfg
        eos = cfg.eog_inference
        gen = None
        if noise_fn is None:
            gen = torch.Generator().manual_seed(int(seed))
        ctx = self.prepare(x_ids, y_prompt, tgt_y_len, prompt_frames)
        st = ctx["state"]
        out: List[int] = []
        logs = []
        while True:
            logits = self.step_logits(ctx)
            if record_logits:
                logs.append(logits.clone())
            noise = noise_fn(st.cur_num_gen) if noise_fn else draw_noise(gen, logits.shape[-1])
            tok, _ = sample_helper(logits, params, st, noise, eos=eos, encodec_sr=cfg.encodec_sr,
                                   extra_cutoff=cfg.extra_cutoff,
                                   text_guard_frames_per_token=cfg.text_guard_frames_per_token)
            out.append(tok)
            st.cur_num_gen += 1
            st.current_length += 1
            if tok == eos:
                break
            if max_steps is not None and st.cur_num_gen >= max_steps:
                break
            self.advance(ctx, tok)
        gen_t = torch.tensor(out, dtype=torch.long)
        res = torch.cat([ctx["y"], gen_t])
        if cfg.special_first:
            res = res - int(cfg.n_special)
            gen_t = gen_t - int(cfg.n_special)
        r = {"res": res.view(1, 1, -1), "gen": gen_t.view(1, 1, -1)}
        if record_logits:
            r["logits"] = torch.stack(logs) if logs else torch.zeros(0)
        return r
