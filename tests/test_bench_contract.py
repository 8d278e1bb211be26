"""The committed bench lines (profiles/r01_bench_*.json, written by `python bench.py [--workload …]`
on an MI355X) carry every field of the driver's JSON contract, with the roofline and CPU-baseline
objects, and a verified result. CPU-only: reads the committed files."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r01_bench_*.json")))

TOP = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
       "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}
ROOF = {"bound", "achieved", "peak", "unit", "frac", "traffic"}
CPU = {"value", "unit", "cores", "kind", "sample"}


def test_bench_files_present():
    names = {os.path.basename(f) for f in FILES}
    assert "r01_bench_config2_sum.json" in names  # the headline (BASELINE.json config 2)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_bench_line_contract(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.strip()]
    assert len(lines) == 1, "one JSON line per run"
    d = json.loads(lines[0])
    assert TOP <= set(d), TOP - set(d)
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["steps"] >= 1
    assert d["n_gpus"] == 1 and d["scaling"] in ("weak", "strong")
    assert d["higher_is_better"] is True
    assert "workload" in d["config"]
    assert ROOF <= set(d["roofline"]), ROOF - set(d["roofline"])
    r = d["roofline"]
    assert 0 < r["frac"] <= 1 and abs(r["achieved"] / r["peak"] - r["frac"]) < 1e-6
    assert CPU <= set(d["cpu_baseline"]), CPU - set(d["cpu_baseline"])
    assert d["cpu_baseline"]["kind"] in ("port", "reference") and d["cpu_baseline"]["cores"] >= 1
    assert d.get("verified") is True


def test_headline_metric_matches_baseline():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    d = json.loads(open(os.path.join(ROOT, "profiles", "r01_bench_config2_sum.json")).read())
    assert d["metric"].startswith("Paillier homomorphic adds/sec (2048-bit key, mod n")
    assert base["metric"].startswith("Paillier homomorphic adds/sec (2048-bit key, mod n")
    assert d["config"]["rows"] == 10_000_000 and d["config"]["key_bits"] == 2048
    assert d["roofline"]["traffic"] is not None
