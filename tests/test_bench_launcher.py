"""bench.py's multi-rank launcher on the CPU (gloo): `--gpus N` without torch.distributed.run spawns N rank
processes, every rank checks the process group size, a failing rank fails the run, and a launcher/--gpus
mismatch is an error."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--backend", "gloo"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1            # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["dry_run"]


def test_failing_rank_fails_the_run():
    r = _run(["--gpus", "2", "--dry-run", "--backend", "gloo"], {"HISEG_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "a rank failed" in r.stderr


def test_gpus_must_match_the_launcher_world():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def _maximal_out():
    """A result object shaped like a full one-GPU run (round 5's 22.5 KB line), with every optional key present
    and long strings everywhere the detail file takes them."""
    big = "x" * 3000
    roof = {"bound": "mfma", "achieved": 1276.7, "peak": 2500.0, "unit": "TFLOP/s", "frac": 0.5107,
            "traffic": 1195599100, "kernel_id": "conv_hwc_128_256x256_roi", "kernel": big, "launches_timed": 90,
            "avg_launch_ms": 0.7266, "flop_per_launch": 927712935936.0, "share_of_step": 0.23,
            "traffic_unit": big}
    leg = {"metric": "train step/s", "value": 13.781, "unit": "steps/s", "ms_per_step": 72.56, "steps": 5,
           "warmup": 3, "pipeline_frac": 0.25, "config": {"workload": big}, "roofline": dict(roof),
           "call_profile": {"classes": {str(i): {"ms": 1.0, "note": big} for i in range(20)}, "top": [big] * 10}}
    out = {"metric": "m" * 80, "value": 15432.2, "unit": "ROI-masks/s", "n_gpus": 1, "steps": 20, "warmup": 5,
           "ms_per_step": 16.589, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "d" * 100, "config": {"workload": "w" * 120, "global_batch": 32, "rois_per_step": 256,
                                         "seq_len": None, "parallelism": "p" * 60, "schedule": "s" * 70},
           "pipeline_tflops": 872.9, "roofline": dict(roof)}
    for k in ("train", "train_c3", "train_c4", "distill", "distill_unfrozen", "eval", "datapath"):
        out[k] = json.loads(json.dumps(leg))
    for k in ("cpu_baseline", "cpu_baseline_train", "cpu_baseline_train_c3"):
        out[k] = {"value": 19.29, "unit": "ROI-masks/s", "cores": 16, "kind": "port", "sample": "s" * 200,
                  "bench_batch": {"sample": big}}
    return out


def test_compact_bench_line_is_bounded_and_keeps_the_contract():
    """the driver parsed nothing from a 22.5 KB line.  The printed line stays <= 4 KB and keeps
    the contract keys, the headline roofline and the CPU baseline; details go to the side file."""
    sys.path.insert(0, ROOT)
    import bench
    out = _maximal_out()
    s = bench.compact_line(out, os.path.join(ROOT, "gpurun_out", "bench_detail.json"))
    assert len(s.encode()) <= bench.LINE_MAX_BYTES
    assert "\n" not in s
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
              "cpu_baseline", "scaling"):
        assert k in line, k
    assert line["roofline"]["frac"] == 0.5107 and "kernel" not in line["roofline"]
    assert line["cpu_baseline"]["cores"] == 16
    assert line["legs"]["train"]["ms_per_step"] == 72.56
    assert line["detail"] == os.path.join("gpurun_out", "bench_detail.json")


def test_compact_bench_line_drops_leg_detail_before_the_headline():
    sys.path.insert(0, ROOT)
    import bench
    out = _maximal_out()
    out["config"]["workload"] = "w" * 2500   # force the fallbacks
    line = json.loads(bench.compact_line(out))
    assert line["value"] == 15432.2 and line["roofline"]["frac"] == 0.5107 and "cpu_baseline" in line
    assert len(json.dumps(line, separators=(",", ":")).encode()) <= bench.LINE_MAX_BYTES
