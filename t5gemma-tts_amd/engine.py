"""Python host mirror of the reference's generate() hot path, over libt5gtts.so.

``T5GemmaTTSEngine`` owns device weights (packed once into the P16 MFMA layout)
and a native engine handle; ``generate`` runs a batch of utterances.
``T5GemmaVoiceForConditionalGeneration`` keeps the reference's model API
(hf_export/modeling_t5gemma_voice.py:338-862): ``from_pretrained`` and
``inference_tts(x, x_lens, y, tgt_y_lens, top_k, top_p, min_p, temperature,
stop_repetition, silence_tokens, multi_trial, **kwargs) -> (res, gen)`` with the
same shapes, errors and token semantics -- and batch > 1 accepted (row i is the
reference run alone on utterance i).

Host-side work is only the reference's index/position plumbing (done with the
same torch fp32 ops the reference uses, so positions are bit-identical); all
arithmetic on activations runs in the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import _lib
from .config import VoiceConfig
from .noise import DeviceNoise
from .weights import check_state_dict

BF16 = torch.bfloat16
MAX_AUDIO = 12288   # cache capacity of both kernel sets: 24 aten kv blocks of 512 keys (t5g_kernels.h)


@dataclass
class SamplingParams:
    """``topk_sampling`` / ``sample_helper`` knobs of one utterance (:565-580)."""
    top_k: Union[int, List[int]] = 30
    top_p: float = 0.9
    min_p: float = 0.0
    temperature: float = 0.8
    stop_repetition: int = 3
    silence_tokens: Sequence[int] = ()
    eos_disabled: bool = False


@dataclass
class Utterance:
    x: Sequence[int]                 # text token ids (no padding)
    y: Sequence[int] = ()            # prompt audio codes incl. y_sep (may be empty)
    tgt_y_len: Optional[int] = None  # tgt_y_lens
    prompt_frames: Optional[int] = None


def reference_noise(seed, steps: int, V: int) -> torch.Tensor:
    """The exponential draws torch.multinomial(p, 1) makes on CPU for ``steps``
    consecutive calls (parity mode, SURVEY a14' 6): after ``torch.manual_seed(seed)``
    for an int ``seed``, or continuing a ``torch.Generator`` (its state is not
    consumed: the draws come from a copy, see ``consume_noise``)."""
    if isinstance(seed, torch.Generator):
        g = torch.Generator()
        g.set_state(seed.get_state())
    else:
        g = torch.Generator().manual_seed(int(seed))
    out = torch.empty(steps, V, dtype=BF16)
    for s in range(steps):
        out[s] = torch.empty(V, dtype=BF16).exponential_(1, generator=g)
    return out


def consume_noise(gen: torch.Generator, steps: int, V: int) -> None:
    """Advance ``gen`` past ``steps`` multinomial calls over V probabilities, exactly as
    the reference's AR loop leaves torch's global generator (:744-751, one
    ``exponential_`` of V bf16 draws per step, EOS step included)."""
    for _ in range(steps):
        torch.empty(V, dtype=BF16).exponential_(1, generator=gen)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class T5GemmaTTSEngine:
    """One engine per GPU: packed weights + KV arena + sampler state in HBM."""

    def __init__(self, cfg: VoiceConfig, state_dict: Dict[str, torch.Tensor], device="cuda:0",
                 max_batch: int = 8, max_text: int = 128, max_audio: int = 1024, max_gen: Optional[int] = None,
                 free_source: bool = False, shared_from: Optional["T5GemmaTTSEngine"] = None):
        """``shared_from``: reuse another engine's packed weights on the same device (e.g. a
        second KV arena / batch slot set without a second 10.6 GB weight copy)."""
        if not torch.cuda.is_available():
            raise RuntimeError("T5GemmaTTSEngine needs a ROCm GPU (MI355X); there is no CPU fallback")
        self.L = _lib.lib()
        self.cfg = cfg
        self.bb = bb = cfg.backbone
        self.device = torch.device(device)
        self.V = cfg.n_audio_tokens
        if not 0 < max_audio <= MAX_AUDIO:
            raise ValueError(f"max_audio {max_audio} outside 1..{MAX_AUDIO} (the decode attention kernels' capacity: "
                             "a 100 s prompt plus the 120 s duration cap)")
        self.max_batch, self.max_text, self.max_audio = max_batch, max_text, max_audio
        self.max_gen = max_gen or max_audio
        dev = self.device
        if shared_from is not None:
            if shared_from.device != dev or shared_from.cfg != cfg:
                raise ValueError("shared_from must be an engine of the same config on the same device")
            self._keep = shared_from._keep
            self._enc, self._dec, self._weights = shared_from._enc, shared_from._dec, shared_from._weights
            self._create(cfg, shared_from._weights)
            return
        check_state_dict(cfg, state_dict)
        self._keep: List[torch.Tensor] = []

        def w(name):
            t = state_dict[name]
            if t.device != dev or t.dtype != BF16:
                t = t.to(device=dev, dtype=BF16)
            return t.contiguous()

        def keep(t):
            self._keep.append(t)
            return t.data_ptr()

        stream = _stream(dev)

        def pack(mat: torch.Tensor) -> int:
            N, K = mat.shape
            nbytes = self.L.t5g_packed_bytes(N, K)
            dst = torch.empty(nbytes // 2, dtype=BF16, device=dev)
            _lib.check(self.L.t5g_pack_weight(_ptr(mat), N, K, K, _ptr(dst), stream), "pack")
            return keep(dst)

        d, f = bb.hidden_size, bb.intermediate_size

        def interleave_gate_up(gate, up):
            # 16-row P16 groups of 8 gate rows then the same 8 features' up rows: one
            # MFMA tile holds gate and up of its features (GeGLU epilogue, gemm.hip)
            return torch.stack([gate.view(f // 8, 8, d), up.view(f // 8, 8, d)], dim=1).reshape(2 * f, d)

        def layer(side: str, i: int) -> _lib.LayerWeights:
            p = f"backbone.model.{side}.layers.{i}"
            lw = _lib.LayerWeights()
            lw.qkv = pack(torch.cat([w(f"{p}.self_attn.q_proj.weight"), w(f"{p}.self_attn.k_proj.weight"),
                                     w(f"{p}.self_attn.v_proj.weight")], 0))
            lw.o = pack(w(f"{p}.self_attn.o_proj.weight"))
            lw.gate_up = pack(interleave_gate_up(w(f"{p}.mlp.gate_proj.weight"), w(f"{p}.mlp.up_proj.weight")))
            lw.down = pack(w(f"{p}.mlp.down_proj.weight"))
            names = ["pre_self_attn_layernorm", "post_self_attn_layernorm", "pre_cross_attn_layernorm",
                     "post_cross_attn_layernorm", "pre_feedforward_layernorm", "post_feedforward_layernorm"]
            for j, nm in enumerate(names):
                key = f"{p}.{nm}.weight"
                lw.norms[j] = keep(w(key)) if key in state_dict else None
            if side == "decoder":
                lw.cross_q = pack(w(f"{p}.cross_attn.q_proj.weight"))
                lw.cross_kv = pack(torch.cat([w(f"{p}.cross_attn.k_proj.weight"),
                                              w(f"{p}.cross_attn.v_proj.weight")], 0))
                lw.cross_o = pack(w(f"{p}.cross_attn.o_proj.weight"))
            return lw

        self._enc = (_lib.LayerWeights * bb.num_encoder_layers)(
            *[layer("encoder", i) for i in range(bb.num_encoder_layers)])
        self._dec = (_lib.LayerWeights * bb.num_decoder_layers)(
            *[layer("decoder", i) for i in range(bb.num_decoder_layers)])
        W = _lib.Weights()
        W.enc_embed = keep(w("backbone.model.encoder.embed_tokens.weight"))
        W.audio_embed = keep(w("audio_embedding.0.weight"))
        W.enc_final_norm = keep(w("backbone.model.encoder.norm.weight"))
        W.dec_final_norm = keep(w("backbone.model.decoder.norm.weight"))
        W.head1 = pack(w("predict_layer.0.0.weight"))
        W.head1_bias = keep(w("predict_layer.0.0.bias"))
        W.head2 = pack(w("predict_layer.0.2.weight"))
        W.head2_bias = keep(w("predict_layer.0.2.bias"))
        inv = 1.0 / (bb.rope_theta ** (torch.arange(0, bb.head_dim, 2, dtype=torch.float) / bb.head_dim))
        W.inv_freq = keep(inv.to(dev))
        W.enc_layers = self._enc
        W.dec_layers = self._dec
        self._weights = W
        if free_source:
            state_dict.clear()
        self._create(cfg, W)

    def _create(self, cfg: VoiceConfig, W) -> None:
        bb, dev = cfg.backbone, self.device
        d, f = bb.hidden_size, bb.intermediate_size
        max_batch, max_text, max_audio = self.max_batch, self.max_text, self.max_audio
        c = _lib.Config()
        c.hidden, c.intermediate = d, f
        c.n_enc_layers, c.n_dec_layers = bb.num_encoder_layers, bb.num_decoder_layers
        c.n_heads, c.n_kv_heads, c.head_dim = bb.num_attention_heads, bb.num_key_value_heads, bb.head_dim
        c.text_vocab, c.n_audio_tokens = bb.text_vocab_size, self.V
        c.attn_scale = bb.attn_scale
        c.softcap = bb.softcap
        c.rms_eps = bb.rms_norm_eps
        c.normalizer = float(torch.tensor(d ** 0.5, dtype=BF16).item())
        c.sliding_window = int(bb.sliding_window)
        for i, lt in enumerate(bb.layer_types("encoder")):
            c.enc_sliding[i] = 1 if lt == "sliding_attention" else 0
        for i, lt in enumerate(bb.layer_types("decoder")):
            c.dec_sliding[i] = 1 if lt == "sliding_attention" else 0
        c.max_batch, c.max_text, c.max_audio, c.max_gen = max_batch, max_text, max_audio, self.max_gen
        c.eos = cfg.eog_inference
        c.eos_guard = cfg.eos_guard_steps
        c.budget_extra = float(cfg.extra_budget)
        c.text_guard = int(cfg.text_guard_frames_per_token)
        c.progress_scale = float(cfg.progress_scale)
        self._cfg = c
        torch.cuda.synchronize(dev)
        h = C.c_void_p()
        _lib.check(self.L.t5g_engine_create(C.byref(c), C.byref(W), C.byref(h)), "engine_create")
        self.h = h
        ld = C.c_int32()
        self._logits_ptr = self.L.t5g_logits_ptr(h, C.byref(ld))
        self.logits_ld = ld.value
        self._noise = DeviceNoise(self.V, self.device)

    def set_fused(self, enable: bool) -> None:
        """Fast-path decode layer after the self attention (o-proj, norm, cross-q, cross
        attention, cross-o, norm, gate/up, down, norm, the next q|k|v) as one persistent
        launch (default; 17-32 rows: the MLP half) or as per-op launches; bitwise equal
        (csrc/fused.hip). In parity mode the same switch selects the exact-order persistent
        layer (csrc/xlayer.hip; 1-8 rows of <= 64 text keys), bitwise equal to the per-op
        exact launches."""
        _lib.check(self.L.t5g_engine_set_fused(self.h, 1 if enable else 0), "set_fused")

    def xlayer_launches(self) -> int:
        """Parity-mode persistent layer launches issued so far (test / bench hook; a launch
        captured into a graph counts once)."""
        n = C.c_int64()
        _lib.check(self.L.t5g_engine_xlayer_launches(self.h, C.byref(n)), "xlayer_launches")
        return n.value

    def set_attn_in_block(self, mode) -> None:
        """Fast-path decode self attention inside the persistent layer launch (csrc/fused.hip
        stage S): 0 / False its own flash launch, 1 in front of the launch's o-projection,
        2 / True (default) at the end of the previous layer's launch after its q|k|v stage,
        with that layer's o-projection. Bitwise equal in every mode; a call past the tail's
        chunk-slot bound takes mode 1 (two passes of slots, rows up to 3 072 keys at 8 rows),
        past that the separate launch."""
        m = 2 if mode is True else 0 if mode is False else int(mode)
        _lib.check(self.L.t5g_engine_set_attn_in_block(self.h, m), "set_attn_in_block")

    def attn_in_block_mode(self) -> int:
        """Where the last fast-path decode step ran the self attention: 2 at the end of the
        previous layer's launch, 1 in front of the layer's o-projection, 0 its own launch."""
        m = C.c_int32()
        _lib.check(self.L.t5g_engine_attn_in_block_mode(self.h, C.byref(m)), "attn_in_block_mode")
        return m.value

    def attn_in_block_launches(self) -> int:
        """Fast-path persistent layer launches issued with the self attention inside (test /
        bench hook; a launch captured into a graph counts once)."""
        n = C.c_int64()
        _lib.check(self.L.t5g_engine_attn_in_block_launches(self.h, C.byref(n)), "attn_in_block_launches")
        return n.value

    def set_attn_flash(self, enable: bool) -> None:
        """Fast-path decode self attention as one split-key launch with an online-softmax
        combine (default) or as the two-launch aten-order form (scores, then P.V / combine);
        parity mode is unaffected (csrc/attn.hip)."""
        _lib.check(self.L.t5g_engine_set_attn_flash(self.h, 1 if enable else 0), "set_attn_flash")

    def close(self):
        if getattr(self, "h", None):
            self.L.t5g_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def workspace_bytes(self) -> int:
        return int(self.L.t5g_engine_workspace_bytes(self.h))

    # ------------------------------------------------------------------
    def _positions_encoder(self, T: int) -> torch.Tensor:
        # _build_position_ids (:516-531) for one unpadded row
        lengths = torch.tensor([T])
        pos = torch.arange(T, dtype=torch.float32)[None, :]
        denom = (lengths.clamp(min=2).to(torch.float32) - 1.0)[:, None]
        p = pos / denom * self.cfg.progress_scale
        return p.masked_fill(~(pos < lengths[:, None]), 0.0)[0]

    def _positions_prefill(self, cur_len: int, est_total: int) -> torch.Tensor:
        base = torch.arange(cur_len, dtype=torch.float32).unsqueeze(0)
        return (base / max(1, est_total - 1) * self.cfg.progress_scale)[0]

    def logits(self, B: int) -> torch.Tensor:
        """Copy of the current logits [B, V] (bf16, device)."""
        t = torch.empty(B, self.logits_ld, dtype=BF16, device=self.device)
        _lib.check(self.L.t5g_copy_logits(self.h, _ptr(t), B, _stream(self.device)), "copy_logits")
        return t[:, :self.V]

    # ------------------------------------------------------------------
    def set_exact(self, enable: bool) -> None:
        """Switch the engine to the exact-order kernels (csrc/exact.hip: every sum in the
        reference host's CPU order) or back to the fast kernels."""
        if bool(enable) == getattr(self, "_exact", False):
            return
        tab = _lib.gelu_erf_table() if enable else None
        if enable and self.cfg.backbone.softcap != 0.0 and not getattr(self, "_tanh_set", False):
            # eager attention: the reference host's bf16 tanh (csrc/eager.hip)
            _lib.check(self.L.t5g_engine_set_tanh_lut(self.h, _lib.tanh_table()), "set_tanh_lut")
            self._tanh_set = True
        _lib.check(self.L.t5g_engine_set_exact(self.h, 1 if enable else 0, tab, _lib.EXACT_THREADS), "set_exact")
        if enable and getattr(self, "_rope_exc", None) is None:
            self._rope_exc = np.ascontiguousarray(_lib.rope_exc_table())
            _lib.check(self.L.t5g_engine_set_rope_exc(self.h, self._rope_exc.ctypes.data, len(self._rope_exc)),
                       "set_rope_exc")
        self._exact = bool(enable)

    def generate(self, utts: Sequence[Utterance], params: Union[SamplingParams, Sequence[SamplingParams]],
                 seeds: Optional[Sequence[int]] = None, parity: bool = False, use_graph: bool = True,
                 chunk: int = 32, record_logits: bool = False,
                 generators: Optional[Sequence[torch.Generator]] = None, exact: Optional[bool] = None):
        """Run inference_tts on a batch. ``parity=True`` is the reference-reproduction mode:
        the exact-order kernels (logits bit-identical to the reference host's CPU run), the
        reference's CPU RNG stream (MT19937 on the device, csrc/noise.hip) and torch.sort's
        tie order for top-p cuts inside tie groups (csrc/sort_emu.h; the host's std::sort for
        the rare step the device cannot reproduce), in graph-replayed chunks. The stream of row i is ``torch.manual_seed(seeds[i])`` or, with
        ``generators``, the continuation of ``generators[i]`` (e.g. ``torch.default_generator``
        after ``seed_everything``), which is then advanced by exactly the draws the reference
        would have made. ``exact`` (default: = parity) selects the kernel set on its own.
        Returns dict(res=[...], gen=[...], steps, ambiguous)."""
        if generators is not None and not parity:
            raise ValueError("generators= drives the reference RNG stream: parity=True only")
        if exact is None:
            exact = parity
        if exact and not _lib.eager_restated(self.cfg.backbone):
            # eager (softcap) attention is restated for the reference model's call shape (8
            # query heads of 256, csrc/eager.hip); another shape would not be reproduced bit
            # for bit -- refuse instead of degrading
            raise ValueError("parity mode restates eager attention (attn_implementation='eager', logit softcap) "
                             "for 8 query heads of head_dim 256 only (the reference's oneDNN picks its matmul "
                             "kernels by shape): run with parity=False (fast kernels, tolerance parity)")
        if exact:
            for u in utts:
                n_y = len(u.y) + 1
                if len(u.x) > _lib.EXACT_MAX_TOKENS or n_y > _lib.EXACT_MAX_TOKENS:
                    raise ValueError(f"parity mode: text {len(u.x)} / prompt {n_y} tokens exceed the measured "
                                     f"reference K-split table ({_lib.EXACT_MAX_TOKENS})")
        self.set_exact(exact)
        stream = _stream(self.device)
        gen_state = [g.get_state() for g in generators] if generators is not None else None
        try:
            out = self._generate_once(utts, params, seeds, generators, parity, use_graph, chunk, record_logits, stream)
        except _lib.FusedHandoffError:
            # the fused decode launch could not have all its workgroups resident (another
            # process on this GPU): rerun this call on the per-op launches (the same bits),
            # then restore the persistent launch for the next calls
            import warnings
            warnings.warn("fused decode launch gave up waiting (GPU shared?): call rerun on the per-op launches")
            self.set_fused(False)
            if gen_state is not None:
                for g, st_ in zip(generators, gen_state):
                    g.set_state(st_)
            try:
                out = self._generate_once(utts, params, seeds, generators, parity, use_graph, chunk, record_logits,
                                          stream)
            finally:
                self.set_fused(True)
        if generators is not None:
            # where the reference's loop leaves torch's generator: after len(gen) draws of V
            self._noise.advance_generators(generators, [len(row) for row in out["gen"]])
        return out

    def _generate_once(self, utts, params, seeds, generators, parity, use_graph, chunk, record_logits, stream):
        ctx = self._prepare(utts, params, generators if generators is not None else seeds, parity, stream)
        if parity:
            self._run_parity(ctx, stream, record_logits, chunk, use_graph)
        else:
            while not self._decode_chunk(ctx, chunk, use_graph, stream):
                pass
        return self._collect(ctx, stream)

    # -- phases ------------------------------------------------------------------
    def _prepare(self, utts, params, seeds, parity, stream):
        cfg, dev = self.cfg, self.device
        B = len(utts)
        if B < 1:
            raise ValueError("empty batch")
        if B > self.max_batch:
            raise ValueError(f"batch {B} > engine max_batch {self.max_batch}")
        if isinstance(params, SamplingParams):
            params = [params] * B
        seeds = list(seeds) if seeds is not None else list(range(1, B + 1))
        if len(seeds) < B:
            raise ValueError(f"{len(seeds)} seeds for {B} rows")
        # ---- host plumbing: packed text / audio tokens and float PM positions
        ids, trow, tt, tpos, tlen = [], [], [], [], []
        aid, arow, at, apos, alen, last = [], [], [], [], [], []
        states = (_lib.SamplerState * B)()
        rows = (_lib.SamplerRow * B)()
        topk_list: List[int] = []
        silence: List[int] = []
        y_rows = []
        max_steps = 1
        budgets: List[int] = []
        for b, u in enumerate(utts):
            x = [int(v) for v in u.x]
            if len(x) == 0:
                raise ValueError("empty text")
            if len(x) > self.max_text:
                raise ValueError(f"text length {len(x)} > max_text {self.max_text}")
            n_text = cfg.backbone.text_vocab_size
            if min(x) < 0 or max(x) >= n_text:
                # nn.Embedding in the reference: "index out of range in self"
                raise IndexError(f"text id out of range [0, {n_text}): index out of range in self")
            ids += x
            trow += [b] * len(x)
            tt += list(range(len(x)))
            tpos.append(self._positions_encoder(len(x)))
            tlen.append(len(x))
            y = [int(v) for v in u.y]
            if cfg.special_first:
                y = [v + int(cfg.n_special) for v in y]
            if y and (min(y) < 0 or max(y) >= self.V):
                raise IndexError(f"audio token out of range [0, {self.V}) (codec codes must match the model's "
                                 "audio vocabulary): index out of range in self")
            y_rows.append(y)
            cated = [cfg.empty_token] + y
            cur_len = len(cated)
            pf = len(y) if u.prompt_frames is None else int(u.prompt_frames)
            tgt = None if u.tgt_y_len is None else int(u.tgt_y_len)
            if tgt is not None:
                est = tgt + 1
            else:
                est = int(cur_len + int(cfg.encodec_sr) * cfg.progress_lookahead_secs)
            est = max(est, cur_len)
            if getattr(self, "_exact", False) and est > _lib.ROPE_EXC_MAX_LEN:
                raise ValueError(f"parity mode: estimated length {est} exceeds the RoPE cos / sin table's "
                                 f"coverage ({_lib.ROPE_EXC_MAX_LEN}, tools/cpu_order/make_rope_table.py)")
            last.append(len(aid) + cur_len - 1)
            aid += cated
            arow += [b] * cur_len
            at += list(range(cur_len))
            apos.append(self._positions_prefill(cur_len, est))
            alen.append(cur_len)
            st = states[b]
            st.cur_num_gen, st.current_length, st.prompt_offset = 0, cur_len, pf + 1
            st.target_total = -1 if tgt is None else tgt
            st.est_total, st.prev_token, st.consec_silence = est, -1, 0
            st.first_input_len, st.done, st.ambiguous_steps, st.last_token, st.next_pos = len(x), 0, 0, -1, 0.0
            if tgt is not None:
                budget = min(int(math.floor(tgt - (pf + 1) + cfg.extra_budget)) + 2, self.max_gen)
                if cur_len + budget > self.max_audio:
                    raise ValueError(f"row {b}: prompt {cur_len} + budget {budget} > max_audio {self.max_audio}")
            else:
                # no tgt_y_lens (:624): the reference has no time budget, only EOS; the
                # engine's cache capacity bounds the row (EOS forced at the last slot)
                budget = min(self.max_gen, self.max_audio - cur_len)
                if budget < 1:
                    raise ValueError(f"row {b}: prompt {cur_len} leaves no room in max_audio {self.max_audio}")
            max_steps = max(max_steps, budget)
            budgets.append(budget)
            p = params[b]
            r = rows[b]
            if isinstance(p.top_k, (list, tuple)):
                r.top_k, r.top_k_list_len, r.top_k_list_off = 0, len(p.top_k), len(topk_list)
                topk_list += [int(k) for k in p.top_k]
            else:
                r.top_k, r.top_k_list_len, r.top_k_list_off = int(p.top_k), 0, 0
            r.top_p, r.min_p, r.temperature = float(p.top_p), float(p.min_p), float(p.temperature)
            r.stop_repetition = int(p.stop_repetition)
            r.n_silence, r.silence_off = len(p.silence_tokens), len(silence)
            silence += [int(s) for s in p.silence_tokens]
            r.eos_disabled = int(bool(p.eos_disabled))
            sd = int(seeds[b].initial_seed()) if isinstance(seeds[b], torch.Generator) else int(seeds[b])
            r.seed_lo, r.seed_hi = sd & 0xFFFFFFFF, (sd >> 32) & 0xFFFFFFFF
        i32 = dict(dtype=torch.int32, device=dev)
        d_ids, d_trow, d_tt = (torch.tensor(v, **i32) for v in (ids, trow, tt))
        d_tpos = torch.cat(tpos).to(dev)
        d_tlen = torch.tensor(tlen, **i32)
        d_aid, d_arow, d_at = (torch.tensor(v, **i32) for v in (aid, arow, at))
        d_apos = torch.cat(apos).to(dev)
        d_alen, d_last = torch.tensor(alen, **i32), torch.tensor(last, **i32)
        L = self.L
        _lib.check(L.t5g_engine_set_text_max(self.h, max(tlen)), "set_text_max")
        # the call's key bound (every row's prompt + budget, rounded up to a 64-key flash chunk;
        # calls with the same bound keep the captured graphs): the decode attention grids
        # cover it, not max_audio
        key_bound = min(self.max_audio, -(-(max(a + b for a, b in zip(alen, budgets)) + 1) // 64) * 64)
        _lib.check(L.t5g_engine_set_audio_max(self.h, key_bound), "set_audio_max")
        if parity:
            # the reference's multinomial draws, one stream step per sampler call (up to the row
            # budget, plus the step at which a cap forces EOS): MT19937 streams generated on a
            # side stream (csrc/noise.hip) while the encoder and prefill run
            # buffer rows sized from this call's steps (2 V int32 per step and row: 0.5 MB),
            # in power-of-two buckets so repeated calls keep the captured graphs' pointer
            cap = min(self.max_gen + 1, max(64, 1 << (max_steps + 1 - 1).bit_length()))
            self._noise.generate(seeds[:B], max_steps + 1, cap, snapshots=isinstance(seeds[0], torch.Generator))
            _lib.check(L.t5g_engine_set_noise_mt(self.h, C.c_void_p(self._noise.raw.data_ptr()), cap),
                       "set_noise_mt")
        else:
            _lib.check(L.t5g_engine_set_noise_mt(self.h, None, 0), "set_noise_mt")
        # the host tensors above were filled on torch's current stream: order them first
        torch.cuda.current_stream(dev).synchronize()
        _lib.check(L.t5g_encode(self.h, B, len(ids), _ptr(d_ids), _ptr(d_trow), _ptr(d_tt), _ptr(d_tpos),
                                _ptr(d_tlen), stream), "encode")
        _lib.check(L.t5g_prefill(self.h, B, len(aid), _ptr(d_aid), _ptr(d_arow), _ptr(d_at), _ptr(d_apos),
                                 _ptr(d_alen), _ptr(d_last), stream), "prefill")
        tk = (C.c_int32 * max(1, len(topk_list)))(*topk_list)
        sl = (C.c_int32 * max(1, len(silence)))(*silence)
        _lib.check(L.t5g_sampler_setup(self.h, B, rows, states, tk, len(topk_list), sl, len(silence),
                                       None, 0, stream), "sampler_setup")
        if parity:
            self._noise.wait()   # the first sampler call reads the draws
        return {"B": B, "rows": rows, "tk": tk, "sl": sl, "y_rows": y_rows, "budgets": budgets, "key_bound": key_bound,
                "max_steps": max_steps, "steps": 0, "ambiguous_fixed": 0, "rec": None,
                "cur": (_lib.SamplerState * B)(), "keep": (d_ids, d_trow, d_tt, d_tpos, d_tlen, d_aid, d_arow, d_at,
                                                          d_apos, d_alen, d_last)}

    def _decode_chunk(self, ctx, chunk: int, use_graph: bool, stream) -> bool:
        """Enqueue up to ``chunk`` graph-replayed decode steps, then read the row states
        (one host sync). Returns True when every row is done."""
        n = max(1, min(chunk, ctx["max_steps"] + 1 - ctx["steps"]))
        _lib.check(self.L.t5g_decode(self.h, n, 1 if use_graph else 0, stream), "decode")
        ctx["steps"] += n
        return self._poll(ctx, stream)

    def _poll(self, ctx, stream) -> bool:
        B, cur = ctx["B"], ctx["cur"]
        _lib.check(self.L.t5g_read_state(self.h, cur, B, stream), "read_state")
        if all(cur[b].done for b in range(B)):
            return True
        if ctx["steps"] > ctx["max_steps"] + 2:
            raise RuntimeError("decode did not terminate within the time budget")
        return False

    def _run_parity(self, ctx, stream, record_logits: bool, chunk: int, use_graph: bool) -> None:
        """The AR loop in parity mode: graph-replayed chunks of sampler + exact decoder steps,
        with the reference's draws and torch.sort's tie order on the device. A row whose tie
        order the device cannot reproduce (csrc/sort_emu.h bails out, or the single-block
        sampler path) stalls without committing its step (state.done == 2); after the chunk
        the host re-runs that step with std::sort (t5g_host_sample), writes the state back
        and runs one decoder step so the row's next logits follow its token.
        record_logits: one step per chunk, every sampled logits row kept."""
        L, B = self.L, ctx["B"]
        rows, tk, sl = ctx["rows"], ctx["tk"], ctx["sl"]
        eos = self.cfg.eog_inference
        rec = [] if record_logits else None
        cur = ctx["cur"]
        budget = ctx["budgets"]
        _lib.check(L.t5g_read_state(self.h, cur, B, stream), "read_state")
        limit = ctx["max_steps"] + 2
        while True:
            active = [b for b in range(B) if cur[b].done != 1]
            if not active:
                break
            stalled = [b for b in active if cur[b].done == 2]
            if stalled:
                lg = self.logits(B).cpu()
                for b in stalled:
                    st_in = _lib.SamplerState()
                    C.memmove(C.byref(st_in), C.byref(cur[b]), C.sizeof(st_in))
                    st_in.done = 0
                    nz = self._noise.q_row(b, st_in.cur_num_gen)
                    out_st = _lib.SamplerState()
                    tok = C.c_int32()
                    _lib.check(L.t5g_host_sample(
                        _ptr(lg[b].contiguous()), self.V, C.byref(rows[b]), tk, sl, C.byref(st_in), _ptr(nz), eos,
                        self._cfg.eos_guard, self._cfg.budget_extra, self._cfg.text_guard,
                        self._cfg.progress_scale, self.max_gen, ctx["key_bound"], C.byref(out_st), C.byref(tok)),
                        "host_sample")
                    out_st.ambiguous_steps = st_in.ambiguous_steps + 1
                    _lib.check(L.t5g_write_state(self.h, C.byref(out_st), b, st_in.cur_num_gen, tok.value, stream),
                               "write_state")
                    ctx["ambiguous_fixed"] += 1
                    limit += 1
                # the resolved rows' next logits (the other rows recompute theirs: same inputs)
                _lib.check(L.t5g_step_only(self.h, stream), "step")
                _lib.check(L.t5g_read_state(self.h, cur, B, stream), "read_state")
                continue
            if rec is not None:
                rec.append(self.logits(B).clone())
                n = 1
            else:
                n = max(1, min(chunk, max(budget[b] + 1 - cur[b].cur_num_gen for b in active)))
            _lib.check(L.t5g_decode(self.h, n, 1 if use_graph else 0, stream), "decode")
            ctx["steps"] += n
            _lib.check(L.t5g_read_state(self.h, cur, B, stream), "read_state")
            if ctx["steps"] > limit + chunk:
                raise RuntimeError("parity decode did not terminate within the time budget")
        ctx["rec"] = rec

    def _collect(self, ctx, stream):
        cfg, B, cur = self.cfg, ctx["B"], ctx["cur"]
        toks = (C.c_int32 * (B * self.max_gen))()
        _lib.check(self.L.t5g_read_tokens(self.h, toks, B, stream), "read_tokens")
        res, gen = [], []
        for b in range(B):
            n = cur[b].cur_num_gen
            g = [toks[b * self.max_gen + i] for i in range(n)]
            gt = torch.tensor(g, dtype=torch.long)
            rt = torch.cat([torch.tensor(ctx["y_rows"][b], dtype=torch.long), gt])
            if cfg.special_first:
                rt = rt - int(cfg.n_special)
                gt = gt - int(cfg.n_special)
            res.append(rt)
            gen.append(gt)
        out = {"res": res, "gen": gen, "steps": ctx["steps"],
               "ambiguous": [cur[b].ambiguous_steps for b in range(B)], "ambiguous_fixed": ctx["ambiguous_fixed"]}
        if ctx["rec"] is not None:
            out["logits"] = ctx["rec"]
        return out


# ----------------------------------------------------------------------------
class T5GemmaVoiceForConditionalGeneration:
    """Drop-in for the reference's HF model class on the generate() path.

    ``from_pretrained(model_dir)`` reads the HF export (config.json +
    safetensors, no pickle); ``inference_tts`` keeps the reference signature
    and return shapes (:565-862)."""

    def __init__(self, cfg: VoiceConfig, state_dict, device="cuda:0", **engine_kw):
        self.config = cfg
        self.args = cfg
        self.engine = T5GemmaTTSEngine(cfg, state_dict, device=device, **engine_kw)

    @classmethod
    def from_pretrained(cls, model_dir: str, device="cuda:0", **engine_kw):
        from .weights import load_hf_checkpoint
        cfg = VoiceConfig.from_pretrained(model_dir)
        return cls(cfg, load_hf_checkpoint(model_dir), device=device, **engine_kw)

    def eval(self):
        return self

    def to(self, *a, **k):
        return self

    @torch.inference_mode()
    def inference_tts(self, x, x_lens, y, tgt_y_lens, top_k=-100, top_p=1.0, min_p=0.0, temperature=1.0,
                      stop_repetition=3, silence_tokens=None, multi_trial=None, parity=None, seeds=None,
                      **kwargs):
        """Reference signature and RNG contract (:565-862). With the defaults the noise of
        every step is drawn from torch's global CPU generator exactly as the reference's
        ``torch.multinomial`` draws it (:137), so ``seed_everything(s)`` followed by this
        call returns the reference's tokens and leaves the global generator where the
        reference leaves it. ``parity=False`` is the fast path (on-device Philox noise,
        graph-replayed loop); its per-row seeds are drawn from the global generator
        unless ``seeds`` is given. Batch > 1 (not allowed by the reference, :594) gives
        row i its own stream: ``seeds[i]``, or a seed drawn from the global generator."""
        cfg = self.config
        if parity is None:
            # the drop-in default: token-exact parity where it is restated (sdpa attention);
            # an eager / softcap checkpoint runs the fast kernels, and says so once
            parity = _lib.eager_restated(cfg.backbone)
            if not parity and not getattr(self, "_warned_eager", False):
                import warnings
                warnings.warn("eager (softcap) attention checkpoint of an unmeasured shape: inference_tts runs the "
                              "fast kernels (logits within tolerance of the reference, tokens may differ); the "
                              "bit-exact parity mode covers sdpa attention and eager attention with 8 query heads "
                              "of 256")
                self._warned_eager = True
        if multi_trial:
            import warnings
            warnings.warn("multi_trial is not supported and will be ignored")   # :585-586
        if int(getattr(cfg, "n_codebooks", 1)) != 1:
            raise ValueError("XCodec2 inference expects n_codebooks=1.")
        B = x.shape[0]
        if y.dim() != 3 or y.shape[2] != 1:
            raise ValueError(f"y must be [B, T, 1], got {tuple(y.shape)}")
        pf = kwargs.get("prompt_frames", None)
        utts = []
        for b in range(B):
            xl = int(x_lens[b])
            utts.append(Utterance(x=x[b, :xl].tolist(), y=y[b, :, 0].tolist(),
                                  tgt_y_len=None if tgt_y_lens is None else int(tgt_y_lens[b]),
                                  prompt_frames=pf))
        params = SamplingParams(top_k=top_k, top_p=top_p, min_p=min_p, temperature=temperature,
                                stop_repetition=stop_repetition, silence_tokens=tuple(silence_tokens or ()))
        generators = None
        if seeds is None:
            if parity and B == 1:
                generators = [torch.default_generator]
            else:
                seeds = [int(s) for s in torch.randint(0, 2 ** 62, (B,), dtype=torch.int64).tolist()]
        out = self.engine.generate(utts, params, seeds=seeds, parity=parity, generators=generators)
        n = max(len(g) for g in out["gen"])
        if B == 1:
            return out["res"][0].view(1, 1, -1), out["gen"][0].view(1, 1, -1)
        # batched: right-pad with eos so rows stack (per-row lengths in .lengths)
        eos = cfg.eog_inference
        gen = torch.full((B, 1, n), eos, dtype=torch.long)
        res = torch.full((B, 1, max(len(r) for r in out["res"])), eos, dtype=torch.long)
        for b in range(B):
            gen[b, 0, :len(out["gen"][b])] = out["gen"][b]
            res[b, 0, :len(out["res"][b])] = out["res"][b]
        return res, gen
