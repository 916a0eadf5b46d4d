"""Write t5gemma-tts_amd/data/rope_trig_exc.bin: the RoPE angles of this model at which the
reference host's cos / sin, after the bf16 cast, differ from the correctly rounded value.

The reference evaluates RoPE's cos / sin with torch 2.10 on CPU ([tf] T5GemmaRotaryEmbedding,
emb.cos() / emb.sin() on fp32, then .to(bf16)). torch is built with USE_MKL=ON, so float
cos / sin run MKL VML's vmsCos / vmsSin (VML_HA) -- a proprietary implementation within
~0.6 ulp that cannot be restated. The kernels (csrc/exact_math.h) evaluate cos / sin in
double (correctly rounded float) and consult this table, which lists every angle of the
enumerable angle set where the two disagree after the bf16 cast:
  angle = fp32(inv_freq[i] * pos)  (the K = 1 fp32 matmul of the rotary embedding),
  inv_freq[i] = 1 / theta ** (arange(0, D, 2) / D) in fp32 (:114-137), and pos from the
  reference's three position formulas (hf_export/modeling_t5gemma_voice.py):
  * encoder / prefill (:516-531, :653-681): fp32(fp32(t / (e - 1)) * 2000), 0 <= t < e;
  * decode step (:817-823): fp32(min((L - 1) / (e - 1) * 2000, 2000)) in Python double;
  for every length e <= E_MAX (the estimated total length / text length; parity mode
  refuses longer ones, engine.py).
Format: little-endian uint32 pairs sorted by angle bits: (angle bits, mkl_cos_bf16 |
mkl_sin_bf16 << 16). Run here only (the build container is the reference host).
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "t5gemma-tts_amd", "data", "rope_trig_exc.bin")
E_MAX = 12288   # a 100 s prompt (5 003 tokens) + the 120 s duration cap (duration_estimator.py:79)
SCALE = 2000.0


def positions(e_max: int, e_min: int = 2) -> np.ndarray:
    out = [np.array([0.0, SCALE], np.float32)]
    for e in range(max(2, e_min), e_max + 1):
        t = torch.arange(e, dtype=torch.float32)
        out.append(((t / (e - 1)) * SCALE).numpy())                       # encoder / prefill
        d = np.arange(e, dtype=np.float64) / float(e - 1) * SCALE          # decode (Python double)
        out.append(np.minimum(d, SCALE).astype(np.float32))
    return np.unique(np.concatenate(out))


def main():
    torch.set_num_threads(8)
    sys.path.insert(0, REPO)
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd.config import named_config
    bb = named_config("2b2b").backbone
    D, theta = bb.head_dim, bb.rope_theta
    inv = (1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float) / D))).numpy()
    t0 = time.time()
    # --extend E0: keep the existing table (lengths <= E0) and add the angles of the lengths
    # E0 < e <= E_MAX (the union is the table of every length <= E_MAX)
    e0 = int(sys.argv[sys.argv.index("--extend") + 1]) if "--extend" in sys.argv else 0
    exc = {}
    if e0:
        old = np.fromfile(OUT, dtype="<u4").reshape(-1, 2)
        exc = {int(k): int(v) for k, v in old}
        print(f"extending the table of lengths <= {e0} ({len(exc)} exceptions)", flush=True)
    pos = positions(E_MAX, e0 + 1 if e0 else 2)
    print(f"{pos.size} distinct positions ({time.time() - t0:.0f} s)", flush=True)
    n_ang = 0
    for i, f in enumerate(inv):
        ang = np.unique((np.float32(f) * pos).astype(np.float32))   # fp32 products
        n_ang += ang.size
        at = torch.from_numpy(ang)
        for which, tf, nf in ((0, torch.cos, np.cos), (1, torch.sin, np.sin)):
            mk = tf(at).to(torch.bfloat16).view(torch.int16).numpy().astype(np.uint16)
            cr = torch.from_numpy(nf(ang.astype(np.float64)).astype(np.float32)).to(torch.bfloat16)
            cr = cr.view(torch.int16).numpy().astype(np.uint16)
            for k in np.nonzero(mk != cr)[0]:
                a = ang[k]
                key = int(a.view(np.uint32))
                if key not in exc:
                    c = torch.cos(torch.tensor([a])).to(torch.bfloat16).view(torch.int16).item() & 0xFFFF
                    s = torch.sin(torch.tensor([a])).to(torch.bfloat16).view(torch.int16).item() & 0xFFFF
                    exc[key] = c | (s << 16)
        if i % 16 == 0:
            print(f"freq {i}: {len(exc)} exceptions so far ({time.time() - t0:.0f} s)", flush=True)
    keys = np.array(sorted(exc), np.uint32)
    tab = np.stack([keys, np.array([exc[int(k)] for k in keys], np.uint32)], 1).astype("<u4")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tab.tofile(OUT)
    print(f"wrote {OUT}: {len(keys)} exceptions over {n_ang} angles ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
