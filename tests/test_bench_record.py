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
    rec = {"elapsed": 0.01, "W": 3840, "H": 2160, "transport": "RCCL send/recv inside libbeam_hip.so",
           "transport_id": "rccl_lib", "fallback": False, "frame_check": True,
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
    assert out["config"]["transport"] == "rccl_lib" and out["config"]["fallback"] is False
    # no counter passes at N > 1: no HBM figure, the algorithmic bytes only against the L2 peak
    assert out["roofline"]["frac"] is None and out["roofline"]["traffic"] is None
    assert out["roofline"]["kernel_ms"] <= out["ms_per_step"] + 1e-12
    assert out["roofline"]["levels"]["data"]["peak"] == bench.L2_PEAK_GBS


def test_multi_record_transport_fields():
    """a driver-run N-GPU line names the transport that carried the bands and whether it is
    the fallback, for each of the three paths multi_gpu can take."""
    a = _args()
    bench.resolve_config(a, 2)
    base = {"elapsed": 0.01, "W": 3840, "H": 2160, "frame_check": True, "checked_planes": ["packed"], "build_ms": 0.1,
            "tris": 278520, "frame_hits": 1, "nbuf": 3, "scene": "armadillo_proxy", "eye": [0, 0, 0],
            "frame_bytes": 5e8, "trace_ms": None, "gather_ms": None, "trace_ms_rank0": None}
    for tid, fb, text in (("rccl_lib", False, "RCCL send/recv inside libbeam_hip.so"),
                          ("torch_rccl", True, "torch.distributed gather over RCCL (the C-ABI communicator did not "
                                               "start: no librccl)"),
                          ("gloo_shared", False, "torch.distributed gather over gloo (shared-device rehearsal)")):
        out = bench.multi_record(a, dict(base, transport=text, transport_id=tid, fallback=fb), 2, _common(2))
        json.dumps(out, allow_nan=False)
        assert out["config"]["transport"] == tid and out["config"]["fallback"] is fb
        assert text in out["config"]["workload"]
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


def test_roofline_passes_its_own_cross_check():
    """on a realistic C3 record (round 5's numbers: 604 MB of §8(d) bytes per frame, the in-flight
    launch span 0.179 ms against a 0.0673 ms step, 66.5 MB of counted HBM bytes per frame; one frame at a time
    0.1316 ms per launch, 0.1411 ms per step, 64.4 MB) every roofline's time basis lies inside its step and its
    byte rate stays under the peak it is compared with: HBM bytes against the HBM peak, §8(d) bytes against L2."""
    src = "live"
    ks = bench.KIND_KERNELS["cull+quads"]
    infl = bench.roofline(604.0e6, 0.1794, 0.0673422, dict(_pmc_rec(), traffic=66.52e6), src, ks, overlapped=True)
    single = bench.roofline(604.0e6, 0.1316, 0.1411, dict(_pmc_rec(), traffic=64.4e6), src, (bench.TRACE_KERNEL,))
    for r, step in ((infl, 0.0673422), (single, 0.1411)):
        assert r["kernel_ms"] <= step + 1e-12
        assert r["traffic"] / (r["kernel_ms"] / 1e3) / 1e9 == r["achieved"] <= r["peak"] == bench.HBM_PEAK_GBS
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
        d = r["levels"]["data"]
        assert d["peak"] == bench.L2_PEAK_GBS and d["achieved"] <= d["peak"]
        assert abs(d["achieved"] - 604.0e6 / (r["kernel_ms"] / 1e3) / 1e9) < 1e-6
    assert infl["launch_ms"] == 0.1794 and infl["kernel_ms"] == 0.0673422 and infl["launch_overlapped"]
    assert abs(infl["frac"] - 66.52e6 / 0.0673422e-3 / 1e9 / 8000) < 1e-9  # ~0.12 of HBM per step
    assert abs(single["frac"] - 64.4e6 / 0.1316e-3 / 1e9 / 8000) < 1e-9
    # the compact line keeps the same numbers and says which time basis they use
    c = bench.compact_roofline(infl)
    assert c["kernel_ms"] <= 0.0673422 and c["step_ms"] == bench._r(0.0673422) and c["launch_overlapped"]
    assert c["achieved"] <= c["peak"] and "hbm" not in c["levels"]
    # without counters there is no HBM figure at all (no fallback to cache-served bytes against HBM)
    none = bench.roofline(604.0e6, 0.1316, 0.1411, None, "none", (bench.TRACE_KERNEL,))
    assert none["frac"] is None and none["achieved"] is None and none["levels"]["data"]["frac"] < 1


def test_build_required_bytes_per_kernel():
    """the build roofline's bytes are the per-kernel bytes the product needs (sorted triangle
    records and corner normals included), and each kernel's counted HBM bytes are reported against them."""
    n, V, R = 278520, 139262, 92000
    req = bench.build_required(n, V, R)
    assert set(req) == {"k_gather", "k_morton", "k_onesweep_wide", "k_bucket_sort", "k_span_chunk"}
    assert req["k_span_chunk"] == 4 * n + 4 * n + 12 * n + 12 * V + 48 * n + 128 * R
    lsd = bench.build_required(n, V, R, sort="lsd")
    assert "k_bucket_sort" not in lsd and lsd["k_onesweep_wide"] == 48 * n + 12 * n + 12 * V + 36 * n
    pk = {"k_gather": {"read_x2": 13.3e6, "write": 4.3e6}, "k_span_chunk": {"read_x2": 24.2e6, "write": 26.6e6},
          "k_chunk_table_lds": {"read_x2": 0.6e6, "write": 0.1e6}}
    r = bench.build_roofline(n, 0.0886, {"traffic": 117.8e6, "per_kernel": pk}, V, R)
    assert abs(r["bytes"] - sum(req.values())) < 1e-6 and r["model_bytes"] == n * bench.BUILD_BYTES_PER_TRI
    assert abs(r["per_kernel"]["k_span_chunk"]["counted_over_required"] - 50.8e6 / req["k_span_chunk"]) < 1e-9
    assert "counted_over_required" not in r["per_kernel"]["k_chunk_table_lds"]  # O(n / 512): no requirement
    c = bench.compact_build(r)
    assert set(c["counted_over_required"]) == {"k_gather", "k_span_chunk"}
    assert abs(c["traffic_over_bytes"] - 117.8e6 / sum(req.values())) < 1e-3


def _lim():
    return {"l2_hit": 0.919306938844901, "ta_busy": 0.5041896371732713, "wave_time_waiting_on_loads": 0.3796644903444764,
            "wave_time_issue_stalled": 0.31100200503550074, "wave_time_issuing": 0.3093018388114838}


def _pmc_rec():
    return {"traffic": 49573328.0, "read_bytes_counted": 7806368.0, "read_bytes_x2": 15612736.0,
            "write_bytes": 33960592.0, "l2_bytes": 612345678.0, "l2_read_bytes": 578000000.0,
            "l2_write_bytes": 34345678.0, "limiter": _lim(),
            "resources": {"k_trace_quad<false, 24, 1u, 0, false, 4>": {"scratch_size": 0, "lds_block_size": 13312},
                          "k_cull<false, 1>": {"scratch_size": 0, "lds_block_size": 512}}}


def _measured(name, light=False):
    """A side figure shaped like Workload.measure's, every key filled with realistic values."""
    src = "live rocprofv3 --pmc passes of this run (tools/pmc.py)"
    ks = bench.KIND_KERNELS["cull+quads"]
    out = {"scene": name, "tris": 1118136, "width": 1920, "height": 1080, "eye": [-0.34, 1.2, -3.5],
           "build_ms": 0.21856200695037842,
           "build_roofline": bench.build_roofline(1118136, 0.21856200695037842,
                                                  {"traffic": 275184896.0, "per_kernel": {
                                                      k: {"read_x2": 1.0e7, "write": 2.0e7} for k in (
                                                          "k_gather", "k_morton", "k_onesweep_wide", "k_bucket_sort",
                                                          "k_span_chunk", "k_pack4_table")}}),
           "frames_in_flight": 3, "mrays_s": 14716.29740882352, "ms_per_step": 0.1409050077199936,
           "trace_kernel_ms": 0.3616433024406433, "frame_hits": 151205, "frame_check": True,
           "trace_kind": "cull+quads",
           "roofline": bench.roofline(951902921, 0.3616433024406433, 0.1409050077199936, _pmc_rec(), src, ks, True),
           "single_frame": {"mrays_s": 8989.66061422273, "ms_per_step": 0.23066499270498753,
                            "trace_kernel_ms": 0.22170210182666777, "trace_kind": "quads",
                            "roofline": bench.roofline(951902921, 0.22170210182666777, 0.23066499270498753,
                                                       _pmc_rec(), src, (bench.TRACE_KERNEL,))},
           "per_ray": {"node_records": 2.3590123456790124, "tri_tests": 0.44990113811728394,
                       "hit_frac": 0.07291907793209877}}
    if light:
        out.update(light=[0.0, 10.0, -10.0], shadowed=16682, rays_incl_shadow_per_s_M=15789.396246449467)
        out["per_ray"].update(shadow_rays=151205, shadow_node_records_per_shadow_ray=15.57330776098674,
                              shadow_tri_tests_per_shadow_ray=6.6767104262425185)
    return out


def test_compact_line_fits_the_driver_tail():
    """the N = 1 line the driver parses stays far below 8 kB with every side figure filled
    (round 4's ~22-25 kB line was lost), is strict JSON, and keeps the contract fields; the full record
    goes to a file named in the line."""
    a = _args()
    bench.resolve_config(a, 1)
    head = _measured("armadillo_proxy")
    extra = {key: _measured(key, light=(cid == "c5")) for cid, key in bench.EXTRA_CONFIGS.items() if cid != "c3"}
    extra["reference_mode"] = {"build_ms": 0.4459240138530731, "trace_ms": 0.3830796003341675,
                               "mrays_s": 5412.974217867932, "frame_hits": 150985, "trace_kind": "kd march",
                               "in_flight": {"frames_in_flight": 3, "ms_per_frame": 0.1468, "mrays_s": 14116.27,
                                             "frame_check": True},
                               "kd_leaves": 16742, "face_refs": 184931, "config_id": "c2",
                               "roofline": bench.roofline(0, 0.383, 0.383, _pmc_rec(), "live", ("k_kd_march_coop<false",))}
    extra["aa_xml"] = {"scene": "f16", "width": 500, "height": 500, "eye": [0.0, 0.0, -2.1],
                       "closest_hit": {"build_ms": 0.0411, "trace_ms": 0.0201, "mrays_s": 12437.5,
                                       "in_flight_mrays_s": 20123.4, "frame_check": True,
                                       "in_flight_frame_check": True},
                       "reference_mode": {"build_ms": 0.1563, "trace_ms": 0.0412, "mrays_s": 6067.9,
                                          "frame_check": True, "in_flight_mrays_s": 9876.5},
                       "published": {"gpu": "GeForce GTX 660 Ti", "march_ms": 38.414, "build_ms": 56.476288,
                                     "source": "aa.xml"},
                       "speedup_vs_published_march": 932.4, "speedup_vs_published_build": 361.3}
    extra["hashed_grid"] = {"build_ms": 0.23, "trace_ms": 128.37, "mrays_s": 16.15, "frame_hits": 91589,
                            "trace_kind": "hash march", "cell_face_pairs": 254233, "buckets_used": 453,
                            "largest_bucket": 2187, "dropped_by_cap": 158647, "config_id": "c2"}
    cpu = {"value": 17.6, "unit": "Mrays/s", "cores": 16, "kind": "port", "algorithm": "reference",
           "algorithm_note": "x" * 300, "sample": "the reference's kd-tree march (oracle restatement of "
           "BuildTree.cu:367-499): 43 full 1920x1080 frames (89164800 rays, 5.1 s) on 16 threads (rows split 8 "
           "ranges/thread) + 4 frames on 1 thread (2.5 s); kd build 136 ms (1 thread)",
           "single_thread_mrays_s": 1.49, "build_ms": 136.2, "threads_note": "y" * 400,
           "all_affinity_linear_bound_mrays_s": 381.99, "affinity_cpus": 256, "cpu_model": "AMD EPYC 9575F 64-Core "
           "Processor", "host_threads": 256, "lbvh_port": {"mrays_s": 60.1, "threads": 16, "build_ms": 80.0, "note": "z"}}
    pmc = {"seconds": 13.3, "errors": None, "plan": {"segments": [{"label": f"s{i}"} for i in range(11)]}}
    full = bench.finite(bench.single_record(a, head, extra, cpu, pmc, "all passes ok", _common(1)))
    assert len(json.dumps(full)) > 15000  # the full record is the big one ...
    line = json.dumps(bench.compact_record(full, bench.FULL_RECORD), allow_nan=False)
    assert len(line) < 6000, len(line)  # ... the line fits the driver's ~8 kB tail with stderr beside it
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out
    assert out["config"]["config_id"] == "c3" and out["full_record"] == bench.FULL_RECORD
    r = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert set(r["levels"]) == {"data", "l2"}  # the HBM level is the contract fields themselves
    assert r["levels"]["l2"]["peak"] == bench.L2_PEAK_GBS and r["peak"] == bench.HBM_PEAK_GBS
    # frames in flight: counted HBM bytes of one frame over the step; §8(d) bytes over the step against L2
    assert abs(r["achieved"] - 49573328.0 / 0.1409050077199936e-3 / 1e9) < 1
    assert abs(r["levels"]["data"]["achieved"] - 951902921 / 0.1409050077199936e-3 / 1e9) < 1
    assert r["kernel_ms"] <= out["ms_per_step"]
    assert out["single_frame"]["roofline"]["levels"]["l2"]["bytes"] > 0
    assert set(out["side"]) == {"c2_bunny", "c4_armadillo_4k", "filled_view", "c5_merged_proxy_shadow", "aa_xml"}
    assert out["side"]["aa_xml"]["closest_hit"]["frame_check"] is True
    assert out["side"]["aa_xml"]["reference_mode"]["frame_check"] is True
    assert out["side"]["aa_xml"]["published_march_ms"] == 38.414
    assert out["side"]["c5_merged_proxy_shadow"]["rays_incl_shadow_per_s_M"] > 0
    assert out["cpu_baseline"]["kind"] == "port" and out["cpu_baseline"]["cores"] == 16
    assert out["reference_mode"]["in_flight_mrays_s"] > 0 and out["hashed_grid"]["mrays_s"] > 0


def test_nonfinite_values_become_null():
    assert bench.finite({"a": float("nan"), "b": [float("inf"), 1.0], "c": {"d": -float("inf")}}) == \
        {"a": None, "b": [None, 1.0], "c": {"d": None}}


def _run_bench(args, extra_env):
    import os
    import subprocess
    import sys
    env = dict(os.environ, **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, bench.__file__, *args], capture_output=True, text=True, env=env,
                          timeout=240, cwd=os.path.dirname(bench.__file__))


def test_gpus_n_self_launches_n_ranks():
    """`bench.py --gpus N` without a launcher starts torch.distributed.run with N ranks as a
    child process (dry run: the ranks meet over gloo, no GPU) and relays exactly one line with n_gpus == N."""
    p = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1"], {"BM_BENCH_DRY_RUN": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["dry_run"] and rec["steps"] == 3
    assert "launching 2 ranks" in p.stderr


def test_gpus_mismatch_prints_no_line():
    """A launcher whose WORLD_SIZE differs from --gpus must not yield a line labelled with the wrong N."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, BM_BENCH_DRY_RUN="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "8"], capture_output=True, text=True, env=env,
                       timeout=120, cwd=os.path.dirname(bench.__file__))
    assert p.returncode != 0 and p.stdout.strip() == ""
