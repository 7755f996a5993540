"""The results tables in README.md / BASELINE.md are generated from profiles/results.jsonl
(tools/results_table.py): one source of truth for every headline number."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_results_tables_match_records():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "results_table.py"), "--check"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


def test_results_records_follow_the_bench_contract():
    recs = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "results.jsonl")) if l.strip()]
    keys = {r["key"] for r in recs}
    assert {"c2", "c3", "c4", "c5"} <= keys
    for r in recs:
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "dtype", "data", "config"):
            assert k in r, (r["key"], k)
        assert r["value"] > 0 and r["data"] == "synthetic"


def test_config_yamls_equal_bench_configs():
    """Every configs/*.yaml that says "same as --config X" carries exactly bench.py's CONFIGS[X] (VERDICT r2:
    c3.yaml once named a different pipeline depth than the built-in config)."""
    import glob
    import importlib.util
    import yaml
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = set()
    for p in sorted(glob.glob(os.path.join(ROOT, "configs", "*.yaml"))):
        head = open(p, encoding="utf-8").readline()
        if "same as --config" not in head:
            continue
        doc = yaml.safe_load(open(p, encoding="utf-8"))
        name = doc.pop("name")
        doc.pop("baseline_config", None)
        assert head.split("same as --config")[1].split()[0].strip(";)") == name, p
        assert doc == bench.CONFIGS[name], (p, doc, bench.CONFIGS[name])
        seen.add(name)
    assert seen == set(bench.CONFIGS), seen
