mkdir -p gpurun_out
timeout -k 10 300 python -u - > gpurun_out/r4_fastcap.log 2>&1 <<'PY'
import sys; sys.path.insert(0, '.')
import t5gemma_tts_amd
from t5gemma_tts_amd.config import named_config
from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
from t5gemma_tts_amd.weights import synthetic_weights
from bench import make_batch
cfg = named_config("2b2b")
sd = synthetic_weights(cfg, 7)
eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=64, max_audio=4200, max_gen=64)
x, y, tgt = make_batch(cfg, 1, seed=1, T_x=60, T_p=30)[0]
u = [Utterance(x=x, y=y, tgt_y_len=len(y) + 10)]
try:
    eng.generate(u, SamplingParams(), seeds=[1])
    print("FAST: ran")
except ValueError as e:
    print("FAST refused:", e)
out = eng.generate(u, SamplingParams(), seeds=[1], parity=True)
print("PARITY ok", out["gen"][0].tolist()[:8])
PY
