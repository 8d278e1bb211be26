"""The committed bench lines (profiles/r01_bench_*.json and the round-2 default line, written
by `python bench.py [--workload …]` on an MI355X) carry every field of the driver's JSON contract, with the roofline and CPU-baseline
objects, and a verified result. CPU-only: reads the committed files."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r01_bench_*.json"))) + [
    os.path.join(ROOT, "profiles", "r02_bench_default_final.json")] + [
    os.path.join(ROOT, "profiles", f"r0{r}_{w}.json") for r in (5, 6) for w in ("default", "pf", "order", "es")]

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
    # n_gpus is the rank count the run was asked for (bench.py asserts it equals --gpus before printing)
    assert d["n_gpus"] >= 1 and d["config"]["parallelism"] == f"rows-sharded x{d['n_gpus']}"
    assert d["scaling"] in ("weak", "strong")
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


def test_round2_default_line_carries_configs_3_and_4():
    """The driver-visible default line also carries BASELINE.json configs 3 and 4,
    each with its own roofline and CPU baseline, and the latency lines."""
    d = json.loads(open(os.path.join(ROOT, "profiles", "r02_bench_default_final.json")).read())
    for name in ("config3_product_filter", "config4_encrypt_sum"):
        c = d["configs"][name]
        assert c["value"] > 0 and c.get("verified") is True, name
        r = c["roofline"]
        assert 0 < r["frac"] <= 1 and abs(r["achieved"] / r["peak"] - r["frac"]) < 1e-6, name
        assert CPU <= set(c["cpu_baseline"]), name
    f = d["configs"]["config3_product_filter"]["filter_roofline"]
    assert 0 < f["frac"] <= 1 and f["traffic"] is not None
    assert d["latency"]["pair_sum_route_2048bit"]["matches"] is True
    assert d["latency"]["config1_sumall_10k_1024bit"]["matches"] is True


def test_round5_default_line_boundary_and_latency():
    """The round-5 default line: configs 3 and 4 verified, the host-boundary (end_to_end) routes matching the
    resident fold, the host CPU per fold reported, and the /Sum native line served without errors."""
    d = json.loads(open(os.path.join(ROOT, "profiles", "r05_default.json")).read())
    for name in ("config3_product_filter", "config4_encrypt_sum"):
        assert d["configs"][name].get("verified") is True, name
    e = d["end_to_end"]
    assert e["binary"]["matches"] and e["decimal"]["matches_resident_fold"] and e["strings"]["matches"]
    folds = d["latency"]["host_cpu_per_fold"]["folds"]
    assert [f["rows"] for f in folds] == [10_000, 1_000_000, 10_000_000]
    big = folds[-1]
    assert big["host_cpu_ms"] < 0.1 * big["wall_ms"]  # the long fold's caller sleeps, it does not spin
    n = d["latency"]["pair_sum_route_native_threads_2048bit"]
    assert n["errors"] == 0 and n["matches"] is True


def test_round6_default_line_and_rehearsal():
    """The round-6 default line: configs 3 and 4 verified with their VALU PMC sources, the strong split's
    combine equal to the fold; the two-rank gloo rehearsal through the launcher reports n_gpus 2, verified."""
    d = json.loads(open(os.path.join(ROOT, "profiles", "r06_default.json")).read())
    assert d["roofline"]["valu_pmc"]["source"] == "profiles/r06_pmc_valu_fold.json"
    for name in ("config3_product_filter", "config4_encrypt_sum"):
        c = d["configs"][name]
        assert c.get("verified") is True and c["roofline"]["valu_pmc"]["source"].startswith("profiles/r06_"), name
    assert 0 < d["configs"]["config4_encrypt_sum"]["roofline"]["lane_mad_frac"] <= 1
    assert d["strong_split_1gpu"]["combined_equals_full_fold"] is True
    g = json.loads(open(os.path.join(ROOT, "profiles", "r06_gloo2_rehearsal.json")).read())
    assert g["n_gpus"] == 2 and g["verified"] is True and g["config"]["parallelism"] == "rows-sharded x2"
