"""Reduce the two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of a driver script to a
profiles/*.json: HBM bytes per launch (or per call of a multi-kernel op) with the gfx950
corrections of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of 16 B/lane
streaming reads: x2; WRITE_SIZE exact; both in KiB).

  python tools/pmc_summarize.py gate_up   gpurun_out/pmc_gu   profiles/r02_pmc_gate_up.json
  python tools/pmc_summarize.py attention gpurun_out/pmc_attn profiles/r02_pmc_attention.json
"""
import csv
import json
import os
import sys

OPS = {
    "gate_up": {"kernels": ["gemv_rx_kernel<12, 1, 3, 6"],
                "algorithmic": 2 * 9216 * 2304 * 2 + 8 * 2304 * 2 + 8 * 9216 * 2,
                "what": "decode gate/up GEGLU GEMV, M=8, N=18432, K=2304 (tools/pmc_gateup.py: 26 weight sets "
                        "rotated, 2.2 GB > 256 MiB Infinity Cache)"},
    "fused_mlp": {"kernels": ["fused_mlp_kernel<1>"],
                  "algorithmic": 2 * 9216 * 2304 * 2 + 2304 * 9216 * 2 + 4 * 8 * 2304 * 4 + 8 * 2304 * 2 + 2 * 2304 * 2
                  + 8 * 2304 * 2 + 8 * 8 * 2304 * 4,
                  "what": "fused decode MLP half (norm -> gate/up GeGLU -> down), M=8, 2b-2b widths "
                          "(tools/pmc_fused.py: 26 layers' weights rotated, 3.3 GB > 256 MiB Infinity Cache); "
                          "algorithmic = weights + cross-o slabs, h, norm weights in + h, down slabs out"},
    "fused_block": {"kernels": ["fused_block_kernel"],
                    "algorithmic": None,   # _lib.fused_block_bytes(8, 60): the average over a step's 26 layers
                    "what": "fused decode block after the self-attention o-projection (norm -> cross-q -> PM cross "
                            "attention -> cross-o -> norm -> gate/up GeGLU -> down -> norm -> next q|k|v), M=8, "
                            "T_x=60, 2b-2b widths (tools/pmc_fused.py: 26 layers rotated, 4.3 GB > 256 MiB Infinity "
                            "Cache); algorithmic = weights + cross K/V + o slabs, h, norm weights, RoPE rows in + h, "
                            "q|k|v slabs out"},
    "fused_block_s": {"kernels": ["fused_block_kernel<2>"],
                      "algorithmic": None,   # tools/pmc_fused.py --self writes it (keys of the run)
                      "what": "fast-path persistent decode layer WITH the next layer's self attention at its end "
                              "(norm -> cross-q -> PM cross attention -> cross-o -> norm -> gate/up GeGLU -> down -> "
                              "norm -> next q|k|v -> stage S: flash chunks over the next layer's cached K / V + "
                              "append -> next o-proj), M=8, T_x=60, L = 903 (the rows' "
                              "final length, where bench.py times it), "
                              "2b-2b widths (tools/pmc_fused.py --self: 26 layers rotated); algorithmic = weights + "
                              "self K/V read + appended K/V + q|k|v slabs + cross K/V + h, norm weights, RoPE rows in "
                              "+ h, q|k|v slabs out"},
    "xlayer": {"kernels": ["xlayer_kernel"],
               "algorithmic": None,   # _lib.xlayer_bytes(8, bb, 60, 26): the average over a step's 26 layers
               "what": "parity mode's persistent decode layer after the self attention (o-proj -> norm -> cross-q "
                       "-> PM cross attention -> cross-o -> norm -> gate/up GeGLU -> down in the reference's K "
                       "parts -> norm -> next q|k|v; exact fp32 orders on the f32 MFMA), M=8, T_x=60, 2b-2b widths "
                       "(tools/pmc_xlayer.py: 26 layers rotated, 4.5 GB > 256 MiB Infinity Cache); algorithmic = "
                       "weights + cross K/V + self-attention output, h in and out, in-launch hand-offs"},
    "attention": {"kernels": ["attn_decode_kernel<256, 2, false>", "attn_pvc_kernel<256, 2, 32>"],
                  "algorithmic": None,
                  "what": "decode self attention (scores + P.V/combine launches), 8 rows x 8/4 heads x 256, L ~ 527 "
                          "(tools/pmc_attention.py: 26 KV caches, 436 MB > 256 MiB Infinity Cache)"},
    "attention_flash": {"kernels": ["attn_decode_kernel<256, 2, true, true>"],
                        "algorithmic": None,
                        "what": "decode self attention, the fast path's one-launch flash form (per-chunk "
                                "online-softmax partials, last-arriving chunk combines), 8 rows x 8/4 heads x 256, "
                                "L ~ 527 (tools/pmc_attention.py --flash: 26 KV caches, 436 MB > 256 MiB Infinity "
                                "Cache)"},
}


def per_call(path, kernels):
    tot = {}
    for r in csv.DictReader(open(path)):
        for k in kernels:
            if k in r["Kernel_Name"]:
                tot.setdefault(k, []).append(float(r["Counter_Value"]))
    n = min(len(v) for v in tot.values())
    return sum(sum(v) / len(v) for v in tot.values()), n, {k: sum(v) / len(v) for k, v in tot.items()}


def main(op, out_dir, dst):
    spec = OPS[op]
    alg = spec["algorithmic"]
    if alg is None and op == "xlayer":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import t5gemma_tts_amd  # noqa: F401
        from t5gemma_tts_amd._lib import xlayer_bytes
        from t5gemma_tts_amd.config import config_2b2b
        bb = config_2b2b().backbone
        alg = xlayer_bytes(8, bb, 60, bb.num_decoder_layers)
    elif alg is None and op == "fused_block_s":
        alg = json.load(open(os.path.join(out_dir, "alg.json")))["algorithmic"]
    elif alg is None and op == "fused_block":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import t5gemma_tts_amd  # noqa: F401
        from t5gemma_tts_amd._lib import fused_block_bytes
        alg = fused_block_bytes(8, 60)
    elif alg is None:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pmc_attention import algorithmic_bytes
        alg = algorithmic_bytes()
    f, nf, fk = per_call(os.path.join(out_dir, "fetch", "pmc_counter_collection.csv"), spec["kernels"])
    w, nw, wk = per_call(os.path.join(out_dir, "write", "pmc_counter_collection.csv"), spec["kernels"])
    hbm = f * 1024 * 2 + w * 1024
    res = {"op": op, "kernels": spec["kernels"], "what": spec["what"], "launches_per_kernel": nf,
           "FETCH_SIZE_KiB_per_call": f, "WRITE_SIZE_KiB_per_call": w,
           "FETCH_SIZE_KiB_by_kernel": fk, "WRITE_SIZE_KiB_by_kernel": wk,
           "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE is half of 16B/lane reads)",
           "hbm_bytes_per_call": int(hbm), "algorithmic_bytes_per_call": int(alg),
           "traffic_over_algorithmic": round(hbm / alg, 4)}
    # the digest of the kernel sources measured (bench.py quotes this traffic only while the
    # tree's sources still hash the same)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd._lib import PMC_SOURCES, kernel_source_digest
    if op in PMC_SOURCES:
        res["source_digest"] = kernel_source_digest(op)
        res["source_files"] = PMC_SOURCES[op]
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
