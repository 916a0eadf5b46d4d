"""Host plumbing around generate(): the reference's ``inference_one_sample``
(inference_tts_utils.py:140-378) restated over this build's engine and codec.

SURVEY 8(a) rows covered here:
  a17  token plumbing: text ids = [bos] + prefix + [x_sep] + target + [eos]
       (:253-273), prompt codes + repeat_prompt + [y_sep] (:179-243), tgt_y_lens
       (:279-285);
  a15  output assembly ``_strip_sep_and_eos`` (:323-357);
  and the codec call on the concatenated / generated frames (:359-366).

Text normalisation and duration estimation are text.py; the prompt audio is encoded by
the codec's XCodec2 encoder (codec_enc.py) when ``audio_fn`` is a path. A missing
reference transcript is produced by the Whisper recognizer (whisper_asr.py) in cli.py,
as the reference CLI does (inference_commandline_hf.py:144-150).

``inference_batch`` is the batched form the reference lacks (its batch is asserted to
1, :288): many utterances through one engine call and one batched codec decode.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import torch

IntList = Union[Sequence[int], torch.Tensor]


def build_text_tokens(target: Union[str, IntList], prefix: Optional[Union[str, IntList]] = None,
                      text_tokenizer=None, x_sep_token: Optional[int] = None, add_eos_token: int = 0,
                      add_bos_token: int = 0) -> List[int]:
    """inference_tts_utils.py:253-273."""
    def enc(t):
        if isinstance(t, str):
            if text_tokenizer is None:
                raise ValueError("text given as a string but no text_tokenizer")
            return list(text_tokenizer.encode(t.strip(), add_special_tokens=False))
        if isinstance(t, list) and t and isinstance(t[0], str):
            return enc(" ".join(t))
        return [int(v) for v in (t.tolist() if isinstance(t, torch.Tensor) else t)]

    ids = enc(target)
    if prefix:
        p = enc(prefix)
        ids = p + [int(x_sep_token)] + ids if x_sep_token is not None else p + ids
    if add_eos_token:
        ids.append(int(add_eos_token))
    if add_bos_token:
        ids = [int(add_bos_token)] + ids
    return ids


def build_prompt(prompt_codes: Optional[IntList], y_sep_token: Optional[int], codec_sr: float,
                 target_generation_length: float, repeat_prompt: Union[int, str] = 0,
                 audio_max_length: float = 40.0) -> torch.Tensor:
    """Prompt frames -> original_audio [1, T_p, 1] (inference_tts_utils.py:179-243).
    ``prompt_codes`` None / empty = no reference audio (no y_sep is inserted)."""
    if prompt_codes is None:
        frames = torch.empty(1, 1, 0, dtype=torch.long)
    else:
        frames = (prompt_codes.detach().cpu() if isinstance(prompt_codes, torch.Tensor)
                  else torch.as_tensor(prompt_codes)).long()
        if frames.ndim == 1:
            frames = frames.view(1, 1, -1)
        elif frames.ndim == 2:
            frames = frames.unsqueeze(0)
        if frames.ndim != 3 or frames.shape[0] != 1:
            raise ValueError(f"Unexpected prompt shape {tuple(frames.shape)}")
        if frames.shape[2] == 1:
            frames = frames.transpose(1, 2).contiguous()
        if frames.shape[1] != 1:
            raise ValueError(f"Expected a single codebook axis, got shape {tuple(frames.shape)}")
    has_ref = frames.shape[2] > 0
    single = frames.clone()
    if isinstance(repeat_prompt, int) and repeat_prompt > 0:
        for _ in range(repeat_prompt):
            frames = torch.cat([frames, single], dim=2)
    elif isinstance(repeat_prompt, str) and repeat_prompt.lower() == "max":
        while frames.shape[2] + codec_sr * target_generation_length + single.shape[2] < audio_max_length * codec_sr:
            frames = torch.cat([frames, single], dim=2)
            if single.shape[2] == 0:
                break
    if y_sep_token is not None and has_ref and frames.shape[2] > 0:
        frames = torch.cat([frames, torch.full((1, 1, 1), int(y_sep_token), dtype=torch.long)], dim=2)
    return frames.transpose(2, 1).contiguous()


def target_length(prompt_frames: int, codec_sr: float, target_generation_length: float,
                  parallel_pattern: int = 0) -> int:
    """inference_tts_utils.py:279-285 (effective_delay_inc = 0)."""
    extra = 2 if parallel_pattern else 0
    return int(prompt_frames + codec_sr * target_generation_length + extra)


def strip_sep_and_eos(frames: torch.Tensor, sep_token: Optional[int], eos_token: Optional[int]) -> torch.Tensor:
    """Drop y_sep / EOS ids from [B, K, T] frames (inference_tts_utils.py:323-354). When
    rows keep different counts, every row is cut (or padded with sep) to the minimum."""
    mask = torch.ones_like(frames, dtype=torch.bool)
    if sep_token is not None:
        mask &= frames.ne(sep_token)
    if eos_token is not None:
        mask &= frames.ne(eos_token)
    if bool(mask.all()):
        return frames
    keep = mask.sum(dim=2)
    if not bool(torch.all(keep.eq(keep[..., :1]))):
        n = int(keep.min())
        rows = []
        for b in range(frames.shape[0]):
            per = []
            for k in range(frames.shape[1]):
                v = frames[b, k][mask[b, k]]
                if v.numel() < n:
                    v = torch.nn.functional.pad(v, (0, n - v.numel()), value=sep_token if sep_token is not None else 0)
                per.append(v[:n].unsqueeze(0))
            rows.append(torch.cat(per, 0).unsqueeze(0))
        return torch.cat(rows, 0).to(frames.device)
    n = int(keep[0, 0])
    return frames[mask].view(frames.size(0), frames.size(1), n)


CODEC_INPUT_SR = 16000     # XCodec2 encodes 16 kHz audio (data/tokenizer.py:125-143)
CODEC_INPUT_HOP = 320      # input samples per code at 16 kHz


def prompt_frames_for_samples(n_samples: int, sample_rate: int) -> int:
    """Codes XCodec2's encoder emits for the first ``n_samples`` of a ``sample_rate`` file.

    The reference truncates the reference audio to ``prompt_end_frame`` samples at the
    file's own rate (``torchaudio.load(num_frames=...)``, data/tokenizer.py:127-128, with
    ``prompt_end_frame = int(cut_off_sec * sr)``, inference_commandline_hf.py:181),
    resamples to 16 kHz (torchaudio: ceil(n * 16000 / sr) samples) and encodes; the
    encoder pads one sample and then up to a multiple of the 320-sample hop
    ([tf] feature_extraction_xcodec2.py "acoustic encoder padding"), i.e. n16 // 320 + 1
    codes."""
    n16 = -(-int(n_samples) * CODEC_INPUT_SR // int(sample_rate))
    return n16 // CODEC_INPUT_HOP + 1


def _eos_token(model_args):
    return getattr(model_args, "eos", getattr(model_args, "eog", None))


def parse_silence_tokens(v):
    """decode_config["silence_tokens"] may be a list or its string form ("[1, 2]"); the
    reference eval()s the string (inference_tts_utils.py:175-176) -- a literal parse here."""
    if isinstance(v, str):
        import ast
        v = ast.literal_eval(v.strip() or "[]")
    return [int(s) for s in (v or [])]


def _no_audio(audio_fn) -> bool:
    return audio_fn is None or (isinstance(audio_fn, str) and audio_fn.strip().lower() in {"", "none", "null"})


def prompt_codes_from(audio_fn, audio_tokenizer, prompt_end_frame: int, prompt_sample_rate: int):
    """The reference prompt as codec ids [1, 1, T] (inference_tts_utils.py:182-206).

    ``audio_fn`` is, as in the reference, a path to the reference audio -- loaded, cut to
    ``prompt_end_frame`` samples (its own rate, > 0), resampled to 16 kHz and encoded by
    ``audio_tokenizer.encode`` (data/tokenizer.py:125-143) -- or, in this build, already
    encoded codec ids (list / 1-D / [1, T] / [1, 1, T] / [1, T, 1]), cut to the codes those
    samples encode to at ``prompt_sample_rate``."""
    if isinstance(audio_fn, str):
        from .audio import load_audio, resample
        n = int(prompt_end_frame) if prompt_end_frame and prompt_end_frame > 0 else -1
        wav, sr = load_audio(audio_fn, num_frames=n)
        target = int(getattr(audio_tokenizer, "encode_sample_rate", 16000))
        if sr != target:
            wav = resample(wav.float(), sr, target)
        if wav.shape[0] == 2:
            wav = wav.mean(dim=0, keepdim=True)
        return audio_tokenizer.encode(wav.unsqueeze(0))
    frames = torch.as_tensor(audio_fn, dtype=torch.long)
    if prompt_end_frame and prompt_end_frame > 0:
        flat = frames.reshape(-1)
        frames = flat[:prompt_frames_for_samples(int(prompt_end_frame), int(prompt_sample_rate))]
    return frames


@torch.no_grad()
def inference_one_sample(model, model_args, text_tokenizer, audio_tokenizer, audio_fn, target_text, lang,
                         device, decode_config, prompt_end_frame, target_generation_length, prefix_transcript=None,
                         quiet=False, repeat_prompt=0, multi_trial=None, return_frames=False, seed=None,
                         parity=True, prompt_sample_rate=CODEC_INPUT_SR):
    """Same arguments, errors and returns as the reference (inference_tts_utils.py:141-379).

    ``audio_fn``: the reference audio (path, encoded by ``audio_tokenizer.encode``) or its
    codec ids (see ``prompt_codes_from``); None / "none" for no reference.
    ``prompt_end_frame`` keeps the reference's units -- a count of audio SAMPLES of the
    reference file (``int(cut_off_sec * sr)``); for code input the file's rate is
    ``prompt_sample_rate``. Text is normalised like the reference (Japanese only, the
    language resolved once, ``text.normalize_text_with_lang``). ``parity=True`` (default)
    draws the sampling noise from torch's global generator like the reference; ``seed``
    gives the row its own ``manual_seed`` stream instead. ``device`` is accepted for
    signature compatibility (the engine's device wins)."""
    from .text import normalize_text_with_lang
    multi_trial = multi_trial or []
    if int(getattr(model_args, "n_codebooks", 1)) != 1:
        raise ValueError("XCodec2 backend supports only n_codebooks=1.")
    codec_sr = int(decode_config["codec_sr"])
    silence = parse_silence_tokens(decode_config.get("silence_tokens", []))
    has_ref = not _no_audio(audio_fn)
    prompt_codes = prompt_codes_from(audio_fn, audio_tokenizer, prompt_end_frame, prompt_sample_rate) \
        if has_ref else None
    original_audio = build_prompt(prompt_codes, getattr(model_args, "y_sep_token", None), codec_sr,
                                  target_generation_length, repeat_prompt,
                                  float(getattr(model_args, "audio_max_length", 40.0)))
    prompt_frames = original_audio.shape[1]
    if isinstance(target_text, str):
        target_text, lang = normalize_text_with_lang(target_text, lang)
    if prefix_transcript and isinstance(prefix_transcript, str):
        prefix_transcript, _ = normalize_text_with_lang(prefix_transcript, lang)
    ids = build_text_tokens(target_text, prefix_transcript, text_tokenizer, getattr(model_args, "x_sep_token", None),
                            getattr(model_args, "add_eos_to_text", 0), getattr(model_args, "add_bos_to_text", 0))
    if int(decode_config.get("sample_batch_size", 1) or 1) > 1:
        raise AssertionError("sample_batch_size must be <= 1 (inference_tts_utils.py:288)")
    if multi_trial:
        raise AssertionError("multi_trial is not supported (reference asserts multi_trial == [])")
    x = torch.LongTensor(ids).unsqueeze(0)
    x_lens = torch.LongTensor([x.shape[-1]])
    tgt = torch.LongTensor([target_length(prompt_frames, codec_sr, target_generation_length,
                                          getattr(model_args, "parallel_pattern", 0))])
    t0 = time.time()
    concat_frames, gen_frames = model.inference_tts(
        x, x_lens, original_audio, tgt_y_lens=tgt, top_k=decode_config["top_k"], top_p=decode_config["top_p"],
        min_p=decode_config.get("min_p", 0.0), temperature=decode_config["temperature"],
        stop_repetition=decode_config.get("stop_repetition", 3), silence_tokens=silence,
        prompt_frames=prompt_frames, **({} if seed is None else {"seeds": [int(seed)]}),
        **({} if parity else {"parity": False}))
    dt = time.time() - t0
    n = gen_frames.shape[-1]
    if not quiet:
        print(f"[Speed] {n / dt if dt > 0 else 0.0:.2f} tokens/s | RTF: {n / codec_sr / dt if dt > 0 else 0.0:.2f}x | "
              f"Generated {n} tokens in {dt:.2f}s")
    y_sep, eos = getattr(model_args, "y_sep_token", None), _eos_token(model_args)
    concat_frames = strip_sep_and_eos(concat_frames, y_sep, eos)
    gen_frames = strip_sep_and_eos(gen_frames, y_sep, eos)
    concat_sample = audio_tokenizer.decode(concat_frames) if has_ref and concat_frames.shape[-1] > 0 else None
    gen_sample = audio_tokenizer.decode(gen_frames)
    if concat_sample is None:
        concat_sample = gen_sample
    if return_frames:
        return concat_sample, gen_sample, concat_frames.detach().cpu(), gen_frames.detach().cpu()
    return concat_sample, gen_sample


@dataclass
class TTSRequest:
    target: Union[str, IntList]
    duration_s: float
    prefix: Optional[Union[str, IntList]] = None
    prompt_codes: Optional[IntList] = None
    seed: int = 1


@torch.no_grad()
def inference_batch(engine, model_args, audio_tokenizer, requests: Sequence[TTSRequest], decode_config,
                    text_tokenizer=None, parity=False):
    """Batched text -> waveform: one generate() over all requests, then one batched codec
    decode of the stripped generated frames (ragged lengths via the codec's lens).
    Returns (list of wav [1, n * hop] tensors, list of generated frame tensors, stats)."""
    from .engine import SamplingParams, Utterance
    codec_sr = float(decode_config["codec_sr"])
    utts = []
    for r in requests:
        oa = build_prompt(r.prompt_codes, getattr(model_args, "y_sep_token", None), codec_sr, r.duration_s)
        ids = build_text_tokens(r.target, r.prefix, text_tokenizer, getattr(model_args, "x_sep_token", None),
                                getattr(model_args, "add_eos_to_text", 0), getattr(model_args, "add_bos_to_text", 0))
        utts.append(Utterance(x=ids, y=oa[0, :, 0].tolist(), tgt_y_len=target_length(oa.shape[1], codec_sr,
                                                                                     r.duration_s)))
    params = SamplingParams(top_k=decode_config["top_k"], top_p=decode_config["top_p"],
                            min_p=decode_config.get("min_p", 0.0), temperature=decode_config["temperature"],
                            stop_repetition=decode_config.get("stop_repetition", 3),
                            silence_tokens=tuple(decode_config.get("silence_tokens", []) or ()))
    t0 = time.time()
    out = engine.generate(utts, params, seeds=[r.seed for r in requests], parity=parity)
    t_gen = time.time() - t0
    y_sep, eos = getattr(model_args, "y_sep_token", None), _eos_token(model_args)
    frames = [strip_sep_and_eos(g.view(1, 1, -1), y_sep, eos)[0, 0] for g in out["gen"]]
    lens = [max(1, int(f.numel())) for f in frames]
    T = max(lens)
    codes = torch.zeros(len(frames), T, dtype=torch.long)
    for b, f in enumerate(frames):
        codes[b, :f.numel()] = f
    t1 = time.time()
    wav = audio_tokenizer.codec.decode(codes, lens=lens)
    torch.cuda.synchronize(wav.device)
    t_codec = time.time() - t1
    hop = audio_tokenizer.codec.cfg.hop_length
    wavs = [wav[b, :, :lens[b] * hop] for b in range(len(frames))]
    n_tok = sum(len(g) for g in out["gen"])
    stats = {"tokens": n_tok, "t_generate": t_gen, "t_codec": t_codec,
             "audio_s": sum(lens) / codec_sr, "rtf": sum(lens) / codec_sr / (t_gen + t_codec)}
    return wavs, frames, stats
