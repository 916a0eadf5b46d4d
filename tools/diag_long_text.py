"""Diagnostic: tiny engine generate() with long text prompts (T_x > 64) at several
max_text capacities, parity and fast sampler modes."""
import sys, os, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    for max_text in (256, 512, 1024, 2048):
        for tx in (60, 100, 150, 300):
            if tx > max_text:
                continue
            for parity in (True, False):
                try:
                    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=max_text, max_audio=256,
                                           max_gen=64)
                    x = [3 + (i * 7) % 250 for i in range(tx)]
                    out = eng.generate([Utterance(x=x, y=[], tgt_y_len=20)], SamplingParams(top_k=20, top_p=0.9),
                                       seeds=[1], parity=parity)
                    torch.cuda.synchronize()
                    print("ok", max_text, tx, parity, len(out["gen"][0]), flush=True)
                except Exception as e:
                    print("FAIL", max_text, tx, parity, repr(e), flush=True)
                    return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
