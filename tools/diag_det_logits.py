"""Where the rare last-row difference starts: R host-loop runs (fast kernels, logits of every
step recorded) of the same utterances and seeds at B rows; per run, for each row whose
logits ever differ from the first run, the first step where they do and the largest
difference. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from test_gpu_fused import _mid_engine, _utts
    from t5gemma_tts_amd.engine import SamplingParams
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    Bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 12]
    cfg, eng = _mid_engine(32)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    for B in Bs:
        utts = _utts(cfg, B, 40 + B)
        seeds = list(range(300, 300 + B))
        for fused in (False, True):
            eng.set_fused(fused)
            runs = [eng.generate(utts, p, seeds=seeds, parity=True, exact=False, record_logits=True)
                    for _ in range(R)]
            out = {"B": B, "fused": fused, "steps": len(runs[0]["logits"]), "diffs": []}
            for r in range(1, R):
                d = []
                n = min(len(runs[0]["logits"]), len(runs[r]["logits"]))
                for b in range(B):
                    first, mx = None, 0.0
                    for s in range(n):
                        l0, l1 = runs[0]["logits"][s], runs[r]["logits"][s]
                        if b < l0.shape[0] and b < l1.shape[0]:
                            x, y = l0[b].float(), l1[b].float()
                            if not torch.equal(x, y):
                                if first is None:
                                    first = s
                                mx = max(mx, float((x - y).abs().max()))
                    if first is not None:
                        d.append([b, first, mx])
                out["diffs"].append(d)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
