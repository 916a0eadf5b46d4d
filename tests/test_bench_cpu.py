"""bench.py argument plumbing (CPU): every BASELINE config is selectable and builds the
workload SURVEY 8(d) describes; the CPU baseline's step sampler works on a tiny model."""
import json
import os

import pytest

from conftest import REPO


def test_workloads_cover_baseline_configs():
    import bench
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert {v[4] for v in bench.WORKLOADS.values()} == {1, 2, 3, 4}
    for name, (b, tx, tp, e2e, idx) in bench.WORKLOADS.items():
        desc = base["configs"][idx]
        assert ("batch 1" in desc) == (b == 1), (name, desc)
        assert e2e == ("decoder" in desc and "RTF" in desc), (name, desc)


@pytest.mark.parametrize("wl", ["c2", "c3", "c3p10", "c4", "c5"])
def test_make_batch_shapes(wl):
    import bench
    from t5gemma_tts_amd.config import config_2b2b
    cfg = config_2b2b()
    b, tx, tp, _, _ = bench.WORKLOADS[wl]
    rows = bench.make_batch(cfg, b, seed=20251226, T_x=tx, T_p=tp)
    assert len(rows) == b
    for x, y, tgt in rows:
        assert len(x) == tx and len(y) == tp and tgt == tp + bench.DUR_FRAMES
        if tp:
            assert x[28] == cfg.x_sep_token and y[-1] == cfg.y_sep_token
            assert all(0 <= v < cfg.audio_vocab_size for v in y[:-1])
        assert all(3 <= v < cfg.backbone.text_vocab_size - 1 or v == cfg.x_sep_token for v in x)
    # c3 keeps the rows the golden_long fixture was made from
    if wl == "c3":
        meta = json.load(open(os.path.join(REPO, "tests", "golden", "golden_long.json")))
        assert rows[0][0] == meta["cases"][0]["x"] and rows[0][1] == meta["cases"][0]["y"]


def test_cli_flags(monkeypatch):
    """--workload and --parity reach main() (parse only: no GPU work happens)."""
    import argparse
    import sys
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "c4", "--parity", "--steps", "1"])
    ap_cls = argparse.ArgumentParser
    orig = ap_cls.parse_args

    def checking_parse(self, args=None, namespace=None):
        ns = orig(self, args, namespace)
        assert ns.workload == "c4" and ns.parity and ns.steps == 1
        raise SystemExit(0)
    monkeypatch.setattr(ap_cls, "parse_args", checking_parse)
    with pytest.raises(SystemExit):
        bench.main()


def test_cpu_baseline_tiny():
    """The CPU baseline times one whole utterance end to end on a tiny model (and reports its
    sample)."""
    import bench
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    x = [5, 6, 7, 8, 9]
    y = [1, 2, 3, cfg.y_sep_token]
    r = bench.cpu_baseline(cfg, sd, (x, y, len(y) + 20), 30)
    assert r["value"] > 0 and r["kind"] == "port" and "timed whole" in r["sample"]


def test_c3p10_rows_pass_1024_keys():
    """--workload c3p10 (round 6): C3's rows with a 10 s prompt (500 codes + y_sep), so every
    row's keys pass 1 024 -- the stage-S range past one combine batch."""
    import bench
    b, tx, tp, e2e, idx = bench.WORKLOADS["c3p10"]
    assert (b, tx, e2e, idx) == bench.WORKLOADS["c3"][:2] + (False, 2) and tp == 501
    from t5gemma_tts_amd.config import config_2b2b
    n_tok_row = bench.DUR_FRAMES + int(config_2b2b().extra_budget) + 1   # bench.py: tokens a row generates
    assert 1 + tp + n_tok_row > 1024 >= 1 + bench.WORKLOADS["c3"][2] + n_tok_row
