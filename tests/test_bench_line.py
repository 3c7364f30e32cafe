"""bench.py's stdout line fits what the driver captures (the 20,659-byte r4 line
was cut by the driver's ~8 KB stdout tail, so BENCH_r04 was never parsed).  CPU only."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _full():
    return json.load(open(os.path.join(ROOT, "profiles", "r4z_bench.json")))


def test_compact_line_fits_and_has_contract_keys():
    full = _full()
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bench.LINE_MAX
    for k in CONTRACT:
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    assert line["metric"] == bench.METRIC
    r = line["roofline"]
    for k in ("bound", "kernel", "achieved", "peak", "frac", "traffic_ratio", "step_issue_frac"):
        assert k in r, k
    c = line["cpu_baseline"]
    for k in ("value", "cores", "kind", "single_core", "single_socket_estimate", "cpu_model"):
        assert k in c, k
    assert set(line["configs"]) == {"c3", "c4", "c5"}
    for v in line["configs"].values():
        for k in ("value", "ms_per_step", "frac", "step_issue_frac", "output_ok"):
            assert k in v
    assert line["end_to_end"]["value"] == full["end_to_end"]["value"]
    assert line["sharded_stream"]["value"] == full["sharded_stream"]["value"]


def test_compact_line_round6_keys():
    """the CPU baseline carries its spread and scaling health, the roofline
    its fraction of the measured 6.29 TB/s copy rate beside the 8 TB/s spec, and the end-to-end
    block its rank count (every rank runs it under --gpus N)."""
    full = _full()
    full["roofline"]["frac_vs_6p29"] = 0.18
    full["cpu_baseline"].update(reps=3, spread={"best": 300.0, "median": 290.0, "worst": 280.0, "spread": 0.0667},
                                health=0.95, health_ok=True)
    full["end_to_end"]["ranks"] = 8
    line = bench.compact_line(full, "x")
    assert len(json.dumps(line)) <= bench.LINE_MAX
    r = line["roofline"]
    assert r["frac_vs_6p29"] == 0.18 and r["peak_measured_copy"] == bench.HBM_COPY_GBS
    c = line["cpu_baseline"]
    for k in ("reps", "median", "spread", "health", "health_ok"):
        assert k in c, k
    assert c["health_ok"] is True and c["spread"] == 0.0667
    assert line["end_to_end"]["ranks"] == 8
    for v in line["configs"].values():
        assert "frac_vs_6p29" in v and "cpu_health" in v


def test_rate_units_and_line_keys():
    """channel-samples/s and x-realtime beside the interchannel MSamples/s."""
    u = bench.rate_units(153000.0, 2, 44100)
    assert u == {"channel_msamples_per_s": 306000.0, "x_realtime": round(153000e6 / 44100, 1)}
    full = _full()
    full["units"] = u
    for c in full.get("configs") or []:
        c["units"] = bench.rate_units(c["value"], 2, 96000)
    line = bench.compact_line(full, "x")
    assert line["units"] == u and len(json.dumps(line)) <= bench.LINE_MAX
    for v in line["configs"].values():
        assert v["x_realtime"] > 0


def test_compact_line_reports_a_failed_multi_rank_leg():
    """A sharded or node end-to-end leg that raised on every rank leaves the headline in the line,
    its failure named beside it (bench.py main)."""
    full = _full()
    full["sharded_stream"] = {"error": "FlacGpuError: comm_init", "output_ok": False, "ranks": 8}
    full["end_to_end"] = {"error": "RuntimeError: x", "output_ok": False, "ranks": 8}
    line = bench.compact_line(full, "x")
    assert line["value"] == full["value"] and len(json.dumps(line)) <= bench.LINE_MAX
    assert line["sharded_stream"]["error"].startswith("FlacGpuError") and line["sharded_stream"]["output_ok"] is False
    assert line["end_to_end"]["error"] == "RuntimeError: x" and line["end_to_end"]["ranks"] == 8


def test_cpu_pick_cores_one_per_physical_core():
    cpus, info = bench.pick_cores(2, "idle")
    assert len(cpus) == len(set(cpus)) <= 2
    assert set(cpus) <= os.sched_getaffinity(0)
    assert bench.pick_cores(2, "none")[0] is None


def test_cpu_baseline_fields(monkeypatch):
    """A tiny fixed-time CPU leg: best-of-N with spread, health = per-core at P / single-core."""
    import argparse

    args = argparse.Namespace(config="c2", configs="", channels=2, bits=16, rate=44100, lpc=0, cpu_frames=256,
                              cpu_seconds=0.05, cpu_reps=2, cpu_place="idle", cpu_threads=2)
    sub, buf = bench.cpu_input(args, "c2")
    c = bench.cpu_baseline(buf, sub)
    assert c["reps"] == 2 and len(c["spread"]["runs"]) == 2 and c["value"] == c["spread"]["best"]
    assert c["cores"] <= 2 and c["single_core"]["value"] > 0
    assert abs(c["health"] - c["value"] / c["cores"] / c["single_core"]["value"]) < 1e-3
    assert c["health_ok"] == (c["health"] >= bench.HEALTH_MIN)


def test_compact_line_survives_the_driver_tail():
    """The line the driver sees is the last 8,392 characters of stdout: with rank 0's one line the
    whole line is inside it and parses."""
    s = json.dumps(bench.compact_line(_full(), "x")) + "\n"
    tail = s[-8392:]
    assert json.loads(tail.strip())["value"] > 0


def test_compact_line_bounded_even_when_blocks_grow():
    full = _full()
    p0 = full["stream_curve"][1]
    full["stream_curve"] = [dict(p0, streams=i + 1) for i in range(400)]  # absurdly many curve points
    assert len(json.dumps(bench.compact_line(full, "x"))) <= bench.LINE_MAX


def test_detail_sidecar_written(tmp_path, monkeypatch):
    p = tmp_path / "d.json"
    monkeypatch.setenv("FLACGPU_BENCH_DETAIL", str(p))
    full = _full()
    bench.write_detail(full)
    assert json.load(open(p))["value"] == full["value"]
