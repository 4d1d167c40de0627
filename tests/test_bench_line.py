"""bench.py's printed JSON line stays parseable by the driver, which reads it from an 8 KB stdout tail
(BENCH_r05's 21.7 KB line was not parsed).  The fixture is the full line round 5's bench printed
(profiles/r5z_bench.log, in the history at commit 76ba74e), the shape `main()` builds before compacting it."""
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

FULL = os.path.join(REPO, "tests", "golden", "bench_line_r05_full.json")


def _full():
    return json.load(open(FULL))


def test_compact_line_fits_the_drivers_tail_and_keeps_the_headline():
    full = _full()
    assert len(json.dumps(full)) > 8192            # the round-5 line the driver could not parse
    line = bench.compact_line(full, "gpurun_out/bench_detail_n1.json")
    s = json.dumps(line)
    assert len(s) <= bench.LINE_LIMIT <= 8192 - 1024, len(s)
    assert json.loads(s) == line
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    assert line["roofline"] == full["roofline"]                      # the headline roofline in full
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert line["cpu_baseline"][k] == full["cpu_baseline"][k]
    assert line["detail"] == "gpurun_out/bench_detail_n1.json"


def test_compact_line_has_one_row_per_config():
    full = _full()
    line = bench.compact_line(full, None)
    assert set(line["configs"]) == set(full["configs"])
    for name, row in line["configs"].items():
        e = full["configs"][name]
        assert row["value"] == e["value"] and row["ms_per_step"] == e["ms_per_step"] and row["steps"] == e["steps"]
        assert row["chains_per_gpu"] == e["chains_per_gpu"]
        assert row["roofline_frac"] == e["roofline"]["frac"]
        assert row["hbm_frac"] == e["roofline"]["hbm"]["frac"]
        assert row["cpu_baseline"] == e["cpu_baseline"]["value"]


def test_compact_line_stays_under_the_limit_when_inflated():
    """Long strings and many configs: optional keys go first, and the line never exceeds LINE_LIMIT."""
    full = _full()
    full["data"] = "x" * 3000
    full["gathered_rhat"] = [1.0] * 200
    for i in range(6):
        full["configs"][f"extra{i}"] = copy.deepcopy(full["configs"]["5"])
    line = bench.compact_line(full, "d.json")
    assert len(json.dumps(line)) <= bench.LINE_LIMIT
    assert line["roofline"] == full["roofline"] and line["value"] == full["value"]
    assert len(line["configs"]) == len(full["configs"])


def test_detail_file_holds_the_full_result(tmp_path):
    full = _full()
    p = bench.write_detail(full, str(tmp_path / "detail.json"))
    assert json.load(open(p)) == full


def test_roofline_is_marked_invalid_when_engines_disagree():
    """engines on different paths make the summed launch arithmetic unphysical; the roofline says so."""
    st = {"step_kernel_launches": 8, "step_kernel_ms": 8.0, "step_ms": 9.0, "step_launches": 8}
    run = {"st": st, "meta": {"model": "sir", "n_population": 200}, "N": 100, "T": 50, "lanes": 1, "steps": 2, "filters": 16,
           "streams": 4, "fused": 1, "dt": 0.01, "cfg": 1, "chains": 8, "paths": [(0, 1), (1, 1)]}
    r = bench.roofline(run, 1e9)
    assert r["valid"] is False and "different paths" in r["invalid_reason"]
    assert r["frac"] is None and r["achieved"] is None
    run["paths"] = [(1, 1)]
    assert bench.roofline(run, 1e9)["valid"] is True


def test_roofline_peak_is_the_measured_loop_ceiling(monkeypatch):
    """The VALU roofline's peak is the SSA loop's measured ceiling (profiles/loop_ceiling.json) when it was taken on
    the library timed here, in lane-events/s; otherwise the flat VALU issue peak."""
    st = {"step_kernel_launches": 8, "step_kernel_ms": 8.0, "step_ms": 9.0, "step_launches": 8}
    run = {"st": st, "meta": {"model": "sir", "n_population": 10000}, "N": 10000, "T": 200, "lanes": 1, "steps": 2,
           "filters": 16, "streams": 4, "dt": 0.01, "cfg": 2, "chains": 8,
           "cst": {"events": 9.0e9, "particle_steps": 1.0e8}}
    ceil = {"lane_events_per_s": 6.0e11, "valu_instr_per_s": 6.3e11, "lane_events_per_s_distinct": 5.0e11}
    monkeypatch.setattr(bench, "loop_ceiling", lambda cfg: (ceil, "profiles/loop_ceiling.json"))
    r = bench.roofline(run, 5.0e9)
    assert r["unit"] == "lane-events/s" and r["peak"] == 6.0e11
    assert abs(r["achieved"] - 5.0e9 * 90.0) < 1.0 and abs(r["frac"] - 0.75) < 1e-12
    monkeypatch.setattr(bench, "loop_ceiling", lambda cfg: ({}, None))
    r = bench.roofline(run, 5.0e9)
    assert r["peak"] == bench.VALU_PEAK and r["peak_kind"].startswith("flat")


def test_committed_loop_ceiling_has_every_config():
    """profiles/loop_ceiling.json (scripts/loop_ceiling.sh) covers every BASELINE config the bench line reports."""
    d = json.load(open(os.path.join(REPO, "profiles", "loop_ceiling.json")))
    for c in ("1", "2", "3", "4", "5"):
        assert d["configs"][c]["uniform"]["lane_events_per_s"] > d["configs"][c]["distinct"]["lane_events_per_s"] > 0
    assert len(d["build_id"]) == 16


def test_roofline_is_one_gpus_share_of_the_job(monkeypatch):
    """At N > 1 ranks `value` is the whole job's rate; the roofline divides it down to this rank's filters."""
    st = {"step_kernel_launches": 8, "step_kernel_ms": 8.0, "step_ms": 9.0, "step_launches": 8}
    run = {"st": st, "meta": {"model": "sir", "n_population": 10000}, "N": 10000, "T": 200, "lanes": 1, "steps": 2,
           "filters": 16, "filters_all": 128, "streams": 4, "dt": 0.01, "cfg": 2, "chains": 8,
           "cst": {"events": 9.0e9, "particle_steps": 1.0e8}}
    ceil = {"lane_events_per_s": 6.0e11, "valu_instr_per_s": 6.3e11}
    monkeypatch.setattr(bench, "loop_ceiling", lambda cfg: (ceil, "profiles/loop_ceiling.json"))
    r = bench.roofline(run, 8 * 5.0e9)
    assert abs(r["frac"] - 0.75) < 1e-12


def test_loop_ceiling_parse_reads_the_runs(tmp_path):
    """scripts/loop_ceiling_parse.py: per (config, variant) the HIP-event rate of the plain run and, from the PMC
    run's counter CSV (one warm-up and three timed launches each), wave64 VALU instr/s and VALU busy of the best."""
    import csv
    import subprocess
    lines = [{"config": 2, "variant": v, "lane_events_per_s": r, "ms": 1.0, "events_per_call": 90.0, "waves": 8192,
              "calls_per_lane": 1, "waves_per_simd_cap": 0} for v, r in (("uniform", 6.0e11), ("distinct", 5.0e11))]
    (tmp_path / "natural.jsonl").write_text("".join(json.dumps(x) + "\n" for x in lines))
    (tmp_path / "pmc").mkdir()
    with open(tmp_path / "pmc" / "run_counter_collection.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Counter_Name", "Counter_Value", "Start_Timestamp",
                                           "End_Timestamp"])
        w.writeheader()
        for d in range(8):
            dur_ns = 1_000_000                                         # 1 ms per launch
            for name, v in (("SQ_INSTS_VALU", 6.0e8 + d), ("SQ_ACTIVE_INST_VALU", 6.0e8),
                            ("SQ_ACTIVE_INST_VALU2", 1.0e8), ("GRBM_GUI_ACTIVE", 8 * 2.4e6)):
                w.writerow({"Dispatch_Id": d + 1, "Counter_Name": name, "Counter_Value": v,
                            "Start_Timestamp": 10_000_000 * d, "End_Timestamp": 10_000_000 * d + dur_ns})
    out = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "loop_ceiling_parse.py"), str(tmp_path)],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    u = d["configs"]["2"]["uniform"]
    assert u["lane_events_per_s"] == 6.0e11 and abs(u["valu_instr_per_s"] - (6.0e8 + 3) / 1e-3) < 1.0
    assert abs(u["clock_ghz"] - 2.4) < 1e-9 and abs(u["valu_busy"] - 4 * 6.0e8 / (1024 * 2.4e6)) < 1e-9
    assert d["configs"]["2"]["distinct"]["valu_instr_per_s"] == (6.0e8 + 7) / 1e-3
