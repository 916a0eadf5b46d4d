"""The bench line's quoted evidence refuses stale files (_lib.pmc_traffic for
roofline.traffic, _lib.fast_token_agreement for the fast path's teacher-forced agreement):
a file is quoted only while the kernel sources it was measured on hash the same as this
tree's. CPU only: temporary report files, no library load."""
import json
import os

from conftest import GOLDEN  # noqa: F401  (sys.path set-up)
from t5gemma_tts_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(tmp_path, name, obj):
    p = tmp_path / name
    p.write_text(json.dumps(obj))
    return str(p)


def test_source_digest_is_stable_and_per_op():
    a = _lib.kernel_source_digest("fused_block_s")
    assert a == _lib.kernel_source_digest("fused_block_s") and len(a) == 16
    assert a != _lib.kernel_source_digest("xlayer")
    assert a != _lib.kernel_source_digest("fast_path")


def test_pmc_traffic_quotes_only_a_fresh_file_of_the_same_kernel(tmp_path):
    dig = _lib.kernel_source_digest("fused_block_s")
    fresh = _write(tmp_path, "fresh.json", {"source_digest": dig, "kernels": ["fused_block_kernel<2>"],
                                            "hbm_bytes_per_call": 220.9e6})
    b, info = _lib.pmc_traffic(fresh, "fused_block_s", "fused_block_kernel<2>")
    assert b == 220.9e6 and info["traffic_source_digest"] == dig == info["kernel_source_digest"]
    stale = _write(tmp_path, "stale.json", {"source_digest": "0" * 16, "kernels": ["fused_block_kernel<2>"],
                                            "hbm_bytes_per_call": 1.0})
    b, info = _lib.pmc_traffic(stale, "fused_block_s", "fused_block_kernel<2>")
    assert b is None and info["traffic_note"].startswith("stale")
    nodig = _write(tmp_path, "nodig.json", {"kernels": ["fused_block_kernel<2>"], "hbm_bytes_per_call": 1.0})
    assert _lib.pmc_traffic(nodig, "fused_block_s", "fused_block_kernel<2>")[0] is None
    other = _write(tmp_path, "other.json", {"source_digest": dig, "kernels": ["xlayer_kernel"],
                                            "hbm_bytes_per_call": 1.0})
    b, info = _lib.pmc_traffic(other, "fused_block_s", "fused_block_kernel<2>")
    assert b is None and "another kernel" in info["traffic_note"]
    b, info = _lib.pmc_traffic(str(tmp_path / "missing.json"), "fused_block_s")
    assert b is None and info["traffic_note"] == "no PMC file"


def test_fast_token_agreement_sums_teacher_forced_rows_of_a_fresh_report(tmp_path):
    dig = _lib.kernel_source_digest("fast_path")
    rows = {"golden_0": {"steps": 16}, "tf_a": {"steps": 300, "ref_sampler_same_token": 280},
            "tf_b": {"steps": 247, "ref_sampler_same_token": 220}}
    fresh = _write(tmp_path, "pf.json", {"source_digest": dig, "rows": rows})
    r = _lib.fast_token_agreement(fresh)
    assert (r["agree"], r["steps"], r["rate"]) == (500, 547, round(500 / 547, 4))
    stale = _write(tmp_path, "pf_stale.json", {"source_digest": "f" * 16, "rows": rows})
    r = _lib.fast_token_agreement(stale)
    assert "rate" not in r and r["note"].startswith("stale")
    none = _write(tmp_path, "pf_none.json", {"source_digest": dig, "rows": {"golden_0": {"steps": 16}}})
    assert _lib.fast_token_agreement(none)["note"] == "no teacher-forced rows"
    assert _lib.fast_token_agreement(str(tmp_path / "missing.json"))["note"] == "no report"


def test_committed_reports_name_their_digests():
    """The committed round-6 evidence files carry the digest field the refusal reads."""
    for name in ("r06_pmc_fused_block_s.json", "r06_pmc_xlayer.json", "r06_parity_full.json"):
        p = os.path.join(REPO, "profiles", name)
        assert os.path.exists(p), name
        d = json.load(open(p))
        assert isinstance(d.get("source_digest"), str) and len(d["source_digest"]) == 16, name
