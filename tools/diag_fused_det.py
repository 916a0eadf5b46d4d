"""Determinism of the fused decode launch: at B rows of the mid-width (true 2b-2b widths,
2 + 2 layers) engine, one per-op run and R fused runs of the same utterances and seeds;
prints, per run, the rows whose tokens differ from the per-op run and the first step where
they do. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    from test_gpu_fused import _mid_engine, _utts
    from t5gemma_tts_amd.engine import SamplingParams
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    Bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [12, 16, 8]
    cfg, eng = _mid_engine(32)
    if os.environ.get("DET_SAMPLER_SINGLE"):   # the single-block sampler kernel only
        from t5gemma_tts_amd import _lib
        _lib.check(_lib.lib().t5g_engine_set_sampler_path(eng.h, 1), "set_sampler_path")
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    for B in Bs:
        utts = _utts(cfg, B, 40 + B)
        seeds = list(range(300, 300 + B))
        eng.set_fused(False)
        ref = eng.generate(utts, p, seeds=seeds)
        res = {"B": B, "fused": [], "per_op": []}
        for r in range(R):
            for mode in ("fused", "per_op"):
                eng.set_fused(mode == "fused")
                out = eng.generate(utts, p, seeds=seeds)
                bad = []
                for b in range(B):
                    a, c = ref["gen"][b].tolist(), out["gen"][b].tolist()
                    if a != c:
                        first = next((i for i in range(min(len(a), len(c))) if a[i] != c[i]), min(len(a), len(c)))
                        bad.append([b, first, len(a), len(c)])
                res[mode].append(bad)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
