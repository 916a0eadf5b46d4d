"""Debug: parity logits of the persistent exact layer (xlayer.hip) vs the per-op exact
launches on the mid config, per step: max |diff| and count of differing logits."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
from test_gpu_xlayer import _mid_engine, _utts  # noqa: E402


def main():
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(16)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    utts = _utts(cfg, B, 90 + B, max_text=64)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    outs = []
    for fused in (True, False):
        eng.set_fused(fused)
        outs.append(eng.generate(utts, p, seeds=list(range(700, 700 + B)), parity=True, record_logits=True))
    for s, (a, b) in enumerate(zip(outs[0]["logits"], outs[1]["logits"])):
        a = a.float()
        b = b.float()
        d = (a - b).abs()
        print(f"step {s}: differing {(d > 0).sum().item()} / {d.numel()}, max {d.max().item():.4g}, "
              f"ref absmax {b.abs().max().item():.4g}")
        if s >= 3:
            break


if __name__ == "__main__":
    main()
