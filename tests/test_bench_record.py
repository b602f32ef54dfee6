"""bench.py's driver records on CPU: which BASELINE config each N measures, and the fields of the
N > 1 and N = 1 JSON lines (from synthetic per-rank records; the GPU runs fill the same functions)."""
import argparse
import json

import bench


def _args(**kw):
    a = argparse.Namespace(config="auto", steps=20, warmup=5, gather_planes="ids", leaf_size=4, bvh_width=4)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _common(world):
    return {"metric": bench.METRIC, "unit": "Mrays/s", "n_gpus": world, "steps": 20, "warmup": 5,
            "higher_is_better": True, "vs_baseline": None, "dtype": "f32", "data": "synthetic", "source_stamp": "x"}


def test_default_configs_follow_baseline():
    """N = 1: C3 (BASELINE configs[2], north_star's armadillo 1080p target); N > 1: C4 (configs[3], the
    armadillo 4K frame BASELINE names for 2/4/8 GPUs), so the scaling curve has one workload at N >= 2
    and the N = 1 line carries that workload's one-GPU point as c4_armadillo_4k."""
    for world, want in [(1, "c3"), (2, "c4"), (4, "c4"), (8, "c4")]:
        a = _args()
        assert bench.resolve_config(a, world) == want and a.config == want
    a = _args(config="c5")
    assert bench.resolve_config(a, 8) == "c5"
    assert bench.EXTRA_CONFIGS["c4"] == "c4_armadillo_4k" and "c2" in bench.EXTRA_CONFIGS
    assert bench.REFMODE_CONFIG == "c2"


def test_multi_record_fields():
    a = _args()
    bench.resolve_config(a, 8)
    rec = {"elapsed": 0.01, "W": 3840, "H": 2160, "transport": "RCCL send/recv inside libbeam_hip.so", "frame_check": True,
           "checked_planes": ["packed", "rgb", "t", "tri_id"], "build_ms": 0.1, "tris": 278520, "frame_hits": 123,
           "nbuf": 3, "scene": "armadillo_proxy", "eye": [0, 0, 0], "frame_bytes": 5e8,
           "trace_ms": 0.05, "gather_ms": 0.07, "trace_ms_rank0": 0.049}
    out = bench.multi_record(a, rec, 8, _common(8))
    json.dumps(out, allow_nan=False)  # strict JSON
    assert out["n_gpus"] == 8 and out["scaling"] == "strong"
    assert out["config"]["config_id"] == "c4" and out["config"]["width"] == 3840 and out["config"]["height"] == 2160
    assert "c4:" in out["config"]["workload"] and "8 GPUs" in out["config"]["workload"]
    assert out["trace_ms"] == 0.05 and out["gather_ms"] == 0.07
    assert abs(out["ms_per_step"] - 0.5) < 1e-12  # 10 ms over 20 steps
    assert abs(out["value"] - 3840 * 2160 * 20 / 0.01 / 1e6) < 1e-6
    assert out["gather_bytes_per_frame"] == 3840 * 2160 * 4 * 7 // 8
    assert out["roofline"]["unit"] == "GB/s" and out["cpu_baseline"] is None
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out


def test_single_record_value_is_the_configured_workload():
    a = _args()
    bench.resolve_config(a, 1)
    head = {"mrays_s": 30000.0, "ms_per_step": 0.069, "scene": "armadillo_proxy", "tris": 278520, "width": 1920,
            "height": 1080, "frames_in_flight": 3, "build_ms": 0.1, "build_roofline": {}, "trace_kind": "cull+quads",
            "trace_kernel_ms": 0.2, "roofline": {"bound": "latency"}, "single_frame": {}, "per_ray": {},
            "frame_hits": 1, "frame_check": True}
    out = bench.single_record(a, head, {"c4_armadillo_4k": {"mrays_s": 1.0}}, {"kind": "port"}, None, "off",
                              _common(1))
    json.dumps(out, allow_nan=False)
    assert out["config"]["config_id"] == "c3" and out["value"] == 30000.0
    assert out["c4_armadillo_4k"]["mrays_s"] == 1.0 and out["cpu_baseline"]["kind"] == "port"
