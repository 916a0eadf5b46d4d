"""End-to-end text ids -> waveform on the GPU (tiny voice model + tiny codec) through
the reference-shaped entry points: ``inference_one_sample`` (inference_tts_utils.py:140)
and the batched ``inference_batch``. The frames must equal a direct engine.generate()
of the same utterance (plumbing exactness) whose every step is verified against the CPU
oracle by teacher forcing (the method of test_gpu_parity.py); waveforms must be within
the 1e-4 RMS bar of the codec oracle."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DC = {"top_k": 30, "top_p": 0.9, "min_p": 0.0, "temperature": 0.8, "stop_repetition": 3, "codec_sr": 50,
      "silence_tokens": [], "sample_batch_size": 1}


def _setup():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd.codec import AudioTokenizer, codec_tiny, synthetic_codec_weights
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import T5GemmaVoiceForConditionalGeneration
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 21)
    model = T5GemmaVoiceForConditionalGeneration(cfg, sd, device="cuda:0", max_batch=4, max_text=32, max_audio=256,
                                                 max_gen=160)
    ccfg = codec_tiny()
    csd = synthetic_codec_weights(ccfg, 22)
    tok = AudioTokenizer(device="cuda:0", cfg=ccfg, state_dict=csd, max_batch=4, max_frames=256)
    return cfg, sd, model, ccfg, csd, tok


def _rms(a, b):
    return float(((a.double().cpu() - b.double().cpu()) ** 2).mean().sqrt())


def _oracle_check(cfg, sd, x, y, tgt, seed, model):
    from oracle.t5g_oracle import SamplerParams
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from tests.test_gpu_parity import teacher_forced_check
    utt = Utterance(x=x, y=y, tgt_y_len=tgt)
    out = model.engine.generate([utt], SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3),
                                seeds=[seed], parity=True, record_logits=True)
    teacher_forced_check(cfg, sd, utt, SamplerParams(top_k=30, top_p=0.9, min_p=0.0, temperature=0.8,
                                                     stop_repetition=3, silence_tokens=()), seed, out, rtol=0.02)
    return out


def test_inference_one_sample_matches_oracles():
    from oracle import xc2_oracle
    from t5gemma_tts_amd.pipeline import inference_one_sample, strip_sep_and_eos
    cfg, sd, model, ccfg, csd, tok = _setup()
    prompt = [3, 60, 12, 9, 41]
    text, prefix = [5, 17, 301, 44], [120, 33, 7]
    cs, gs, cf, gf = inference_one_sample(model, cfg, None, tok, prompt, text, None, "cuda:0", DC,
                                          prompt_end_frame=0, target_generation_length=0.4,
                                          prefix_transcript=prefix, quiet=True, return_frames=True, seed=5,
                                          parity=True)
    x = prefix + [cfg.x_sep_token] + text
    y = prompt + [cfg.y_sep_token]
    ref = _oracle_check(cfg, sd, x, y, len(y) + 20, 5, model)
    assert gf.tolist() == strip_sep_and_eos(ref["gen"][0].view(1, 1, -1), cfg.y_sep_token, cfg.eos).tolist()
    assert cf.tolist() == strip_sep_and_eos(ref["res"][0].view(1, 1, -1), cfg.y_sep_token, cfg.eos).tolist()
    wref = xc2_oracle.decode(csd, gf[0], ccfg)
    assert gs.shape == wref.shape and _rms(gs, wref) <= 1e-4
    assert _rms(cs, xc2_oracle.decode(csd, cf[0], ccfg)) <= 1e-4


def test_inference_batch_rows_match_single_runs():
    from oracle import xc2_oracle
    from t5gemma_tts_amd.pipeline import TTSRequest, inference_batch, strip_sep_and_eos
    cfg, sd, model, ccfg, csd, tok = _setup()
    reqs = [TTSRequest(target=[5, 17, 301], duration_s=0.3, prompt_codes=[3, 60], seed=1),
            TTSRequest(target=[44, 9], duration_s=0.5, prefix=[11, 12], prompt_codes=None, seed=2),
            TTSRequest(target=[7, 8, 9, 10, 11], duration_s=0.2, prompt_codes=[1, 2, 3, 4], seed=3)]
    wavs, frames, stats = inference_batch(model.engine, cfg, tok, reqs, DC, parity=True)
    for r, w, f in zip(reqs, wavs, frames):
        x = (list(r.prefix) + [cfg.x_sep_token] if r.prefix else []) + list(r.target)
        y = list(r.prompt_codes) + [cfg.y_sep_token] if r.prompt_codes else []
        ref = _oracle_check(cfg, sd, x, y, len(y) + int(50 * r.duration_s), r.seed, model)
        want = strip_sep_and_eos(ref["gen"][0].view(1, 1, -1), cfg.y_sep_token, cfg.eos)[0, 0]
        assert f.tolist() == want.tolist()
        if f.numel():
            assert _rms(w, xc2_oracle.decode(csd, f.view(1, -1), ccfg)[0]) <= 1e-4
    assert stats["tokens"] > 0 and stats["t_codec"] > 0


def test_drop_in_inference_tts_global_rng_contract():
    """The reference seeds torch's global generator (seed_everything,
    inference_commandline_hf.py:62-69, 95) and every AR step's torch.multinomial draws
    from it (hf_export/modeling_t5gemma_voice.py:137). The drop-in inference_tts with
    its default arguments must do the same: the tokens equal the engine's run on the
    stream torch.manual_seed(s) starts (the reference's, pinned by the tiny goldens), and
    the global generator ends where the reference leaves it (one V-draw per step)."""
    from t5gemma_tts_amd.engine import SamplingParams, Utterance, consume_noise
    cfg, sd, model, *_ = _setup()
    V = cfg.n_audio_tokens
    for seed, x, y, tgt in [(5, [5, 17, 301, 44, 9], [3, 60, cfg.y_sep_token], 24),
                            (77, [8, 9, 10, 11, 12, 13, 14], [], 18)]:
        kw = dict(top_k=30, top_p=0.9, min_p=0.0, temperature=0.8, stop_repetition=3, silence_tokens=[])
        torch.manual_seed(seed)
        res, gen = model.inference_tts(torch.tensor([x]), torch.tensor([len(x)]),
                                       torch.tensor(y, dtype=torch.long).view(1, -1, 1),
                                       tgt_y_lens=torch.tensor([tgt]), prompt_frames=len(y), **kw)
        after = torch.rand(3)
        ref = model.engine.generate([Utterance(x=x, y=y, tgt_y_len=tgt)], SamplingParams(**kw), seeds=[seed],
                                    parity=True)
        assert gen.view(-1).tolist() == ref["gen"][0].tolist()
        assert res.view(-1).tolist() == y + ref["gen"][0].tolist()
        torch.manual_seed(seed)
        consume_noise(torch.default_generator, gen.shape[-1], V)
        assert torch.equal(torch.rand(3), after)
