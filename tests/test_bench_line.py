"""CPU: bench.py's stdout line stays parseable by the driver (round 4's 20 KB line
was lost).  The compact line is built from a full result -- round 4's real 20,216-byte line
(`profiles/r04_bench.json`, every configs sub-line with its rooflines) -- and must be one JSON line
under 4 KB that keeps the headline keys, the trimmed rollout / update rooflines, the CPU
baseline and a summary of every extra shape."""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module level imports nothing heavy)

HEAD = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config")


def _full():
    with open(os.path.join(ROOT, "profiles", "r04_bench.json")) as f:
        return json.load(f)


def test_compact_line_under_4kb_keeps_the_contract():
    full = _full()
    assert len(json.dumps(full)) > 4096  # the case that broke the driver record
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    assert "\n" not in line and len(line) < 4096, len(line)
    out = json.loads(line)
    for k in HEAD:
        assert k in out, k
    assert out["value"] == full["value"] and out["ms_per_step"] == full["ms_per_step"]
    rf = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "peak_no_fma", "frac_no_fma",
              "flop_per_env_step_counted", "mean_launch_ms", "kernel"):
        assert k in rf, k
    assert abs(rf["frac"] - full["roofline"]["frac"]) < 1e-3 * full["roofline"]["frac"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 * rf["frac"]
    ru = out["roofline_update"]
    assert ru["kernel"] == "k_ppo_grad_ws" and "mean_launch_us" in ru and "update_frac" in ru
    cb = out["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "physics_only", "train_ms", "all_cores"):
        assert k in cb, k
    assert cb["all_cores"]["threads"] == 16
    assert set(out["configs"]) == set(full["configs"])
    for name, c in out["configs"].items():
        assert "env_steps_per_s" in c and "frac" in c, name
    assert out["detail_file"] == "gpurun_out/bench_detail.json"


def test_compact_line_drops_optional_parts_before_the_headline():
    full = _full()
    for i in range(40):  # a pathological number of extra shapes
        full["configs"][f"extra_{i}"] = copy.deepcopy(full["configs"]["config3_full_4096"])
    line = bench.compact_line(full)
    assert len(line) < 4096
    out = json.loads(line)
    assert "configs" not in out and out["value"] == full["value"] and "roofline" in out


def test_multirank_line_carries_the_exchange_check():
    full = _full()
    for k in ("configs", "cpu_baseline"):
        full.pop(k)
    full["n_gpus"] = 8
    full["config"]["exchange"] = "ipc"
    full["config"]["exchange_check"] = {"checked": True, "bitwise_equal_to_reference": True,
                                        "replicas_identical": True, "test_round": True}
    out = json.loads(bench.compact_line(full))
    assert out["config"]["exchange"] == "ipc" and out["config"]["exchange_checked"] is True


def test_detail_file_round_trip(tmp_path):
    full = _full()
    p = tmp_path / "sub" / "detail.json"
    rel = bench.write_detail(full, str(p))
    assert rel is not None and json.load(open(p)) == full


def test_valu_ceiling_uses_the_launched_grid():
    """the split kernels launch whole 4-wave blocks; the one-wave ceiling is priced on
    the launched waves, not only on the waves that hold walkers"""
    full = {"lanes_per_walker": 4, "walkers_per_wave": 8, "waves": 1024, "waves_launched": 1024}
    c, why = bench.valu_ceiling_of(full)
    assert c == bench.PEAK_NOFMA_ONE_WAVE and "1024 of 1024" in why
    ragged = {"lanes_per_walker": 4, "walkers_per_wave": 2, "waves": 750, "waves_launched": 752}
    c, why = bench.valu_ceiling_of(ragged)
    assert abs(c - bench.PEAK_NOFMA_ONE_WAVE * 752 / 1024) < 1e-9 and "752 of 1024" in why
    two = {"lanes_per_walker": 2, "walkers_per_wave": 32, "waves": 2048, "waves_launched": 2048}
    assert bench.valu_ceiling_of(two)[0] == bench.PEAK_NOFMA
    old = {"lanes_per_walker": 2, "walkers_per_wave": 32, "waves": 2048}  # a pre-round-5 mapping
    assert bench.valu_ceiling_of(old)[0] == bench.PEAK_NOFMA


def test_compact_line_falls_back_to_the_contract_keys():
    """when the config / CPU baseline / rehearsal themselves push the line past 4 KB,
    the line keeps the contract keys and the detail file, and stays under the limit"""
    full = _full()
    full["config"]["workload"] = "x" * 5000
    full["rehearsal"] = "y" * 3000
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    assert len(line) < 4096, len(line)
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "detail_file"):
        assert k in out, k
    assert out["value"] == full["value"]


def test_xch_stamp_summary():
    """the exchange kernel's per-block stamps -> span / wait / own / gap in us"""
    import numpy as np
    st = np.zeros((3, 2, 4), np.uint64)
    for l in range(3):
        base = 10000 * l
        # block 0: entry, published +100 ticks (1 us), peers seen +300 (3 us wait), exit +150
        st[l, 0] = [base, base + 100, base + 400, base + 550]
        st[l, 1] = [base + 10, base + 120, base + 420, base + 560]
    s = bench.xch_stamp_summary(st)
    assert s["launches"] == 3 and s["blocks"] == 2
    assert abs(s["span_us_median"] - 5.6) < 1e-9
    assert abs(s["wait_us_median"] - 3.0) < 1e-9
    assert abs(s["own_us_median"] - 2.5) < 1e-9  # (1.0 + 1.5, 1.1 + 1.4)
    assert abs(s["gap_us_median"] - (100.0 - 5.6)) < 1e-9
    full = _full()
    full["xch_profile"] = {"per_rank": [s, s]}
    out = json.loads(bench.compact_line(full))
    assert out["xch_profile_us"][1]["wait"] == 3.0
