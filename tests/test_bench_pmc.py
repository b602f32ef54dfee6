"""bench.py's live counter passes (tools/pmc.py), on synthetic rocprofv3 CSVs: the ordered dispatch
list of each pass is cut into the plan's segments, warm-up launches dropped, medians taken per
launch, builds grouped from their k_gather dispatch, and a dispatch list that does not match the plan
reports an error instead of figures."""
import csv
import os

import pytest

from tools import pmc

HDR = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size", "Kernel_Id",
       "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count",
       "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
NS = "void bm::(anonymous namespace)::"


def write_pass(d, dispatches, counter):
    """dispatches: [(kernel name, value)] in dispatch order; two rows per dispatch (split value)."""
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HDR)
        for i, (k, v) in enumerate(dispatches, 1):
            for ci, c in enumerate((counter,) if isinstance(counter, str) else counter):
                for half in (0.25 * v, 0.75 * v):  # per-dimension rows of one dispatch are summed
                    w.writerow([i, i, "Agent 2", 1, 1, 1, 64, 3, k, 256, 0, 0, 64, 0, 96, c, half * (ci + 1), 0, 1])


def build(k):
    return [(NS + "k_gather(bm::MeshDesc const*)", k), (NS + "k_morton(unsigned int)", k),
            (NS + "k_onesweep_wide<1>(unsigned int const*)", k), (NS + "k_pack4_span(unsigned int)", k)]


QUAD = NS + "k_trace_quad<false, 24, 1u, 0, false, 4>(bm::TraceParams)"
CULL = NS + "k_cull<false, 0>(bm::TraceParams)"
RAYS = NS + "k_trace_rays<false, 24, 1u, 0, false>(bm::TraceParams)"
COUNT = NS + "k_trace_quad<true, 24, 1u, 0, false, 4>(bm::TraceParams)"

PLAN = {"segments": [
    {"label": "c2/inflight", "kind": "cull+quads", "kernels": ["k_cull<false", "k_trace_rays<false"],
     "launches": 4, "warmup": 1},
    {"label": "c2/single", "kind": "quads", "kernels": ["k_trace_quad<false"], "launches": 3, "warmup": 1}],
    "builds": [["c2", 3]]}


def dispatches(scale):
    ds = []
    for b in range(3):
        ds += build(100 * scale + b)
    ds.append((NS + "k_gather(bm::MeshDesc const*)", 7))  # a reference-mode build: k_gather, then kd kernels
    ds.append((NS + "k_kd_top(bm::MeshDesc const*)", 7))
    ds.append((COUNT, 1e9))  # the counting trace is not a segment launch
    for i in range(4):
        ds += [(CULL, 10 * scale), (RAYS, (1000 + i) * scale)]
    ds.append(("__amd_rocclr_copyBuffer", 5))
    for i in range(3):
        ds.append((QUAD, (2000 + 10 * i) * scale))
    return ds


def test_segments_medians_and_builds(tmp_path):
    write_pass(str(tmp_path / "p0"), dispatches(1), "FETCH_SIZE")
    write_pass(str(tmp_path / "p1"), dispatches(2), "WRITE_SIZE")
    s = pmc.summarize({"p0": str(tmp_path / "p0"), "p1": str(tmp_path / "p1")}, PLAN)
    assert s["errors"] == {}
    inf, sing = s["segments"]["c2/inflight"], s["segments"]["c2/single"]
    assert inf["launches_counted"] == 3 and sing["launches_counted"] == 2
    # in flight: launches 2..4 sum cull + rays: 10 + 1001..1003 -> median 1012 KiB read
    assert inf["read_bytes_counted"] == 1012 * 1024
    assert inf["read_bytes_x2"] == 2 * 1012 * 1024
    assert inf["write_bytes"] == 2 * 1012 * 1024
    assert inf["traffic"] == 4 * 1012 * 1024
    assert sing["read_bytes_counted"] == 2015 * 1024  # median of 2010, 2020
    # builds: 3 builds of 4 launches each, the first two dropped -> the third (102 x 4)
    assert s["builds"]["c2"]["read_bytes_counted"] == 4 * 102 * 1024
    assert s["builds"]["c2"]["write_bytes"] == 4 * 202 * 1024


def test_mismatched_dispatch_list_reports_an_error(tmp_path):
    ds = [d for d in dispatches(1) if d[0] != CULL]  # a kind the plan does not describe
    write_pass(str(tmp_path / "p0"), ds, "FETCH_SIZE")
    s = pmc.summarize({"p0": str(tmp_path / "p0")}, PLAN)
    assert "p0" in s["errors"]
    assert s["segments"]["c2/inflight"]["traffic"] is None


@pytest.mark.parametrize("lim,hbm,want", [
    ({"wave_time_waiting_on_loads": 0.42, "wave_time_issue_stalled": 0.28, "wave_time_issuing": 0.30}, 0.07,
     "latency"),
    ({"wave_time_waiting_on_loads": 0.2, "wave_time_issue_stalled": 0.5, "wave_time_issuing": 0.3}, 0.07, "issue"),
    ({"wave_time_waiting_on_loads": 0.9}, 0.75, "hbm"),
    ({}, None, None)])
def test_bound_of(lim, hbm, want):
    assert pmc.bound_of(lim, hbm) == want


def test_bench_roofline_levels_each_against_its_own_peak():
    """Each byte count against the level that serves it: the contract fields are the
    counted HBM bytes vs 8 TB/s, the counted L2 request bytes and the §8(d) data bytes vs the aggregate L2
    peak (levels.l2, levels.data)."""
    import bench
    rec = {"traffic": 60e6, "read_bytes_counted": 6e6, "read_bytes_x2": 12e6, "write_bytes": 48e6,
           "l2_bytes": 700e6, "l2_read_bytes": 650e6, "l2_write_bytes": 50e6,
           "limiter": {"wave_time_waiting_on_loads": 0.41, "wave_time_issue_stalled": 0.3, "wave_time_issuing": 0.29}}
    # 4.7 GB of algorithmic bytes in 0.41 ms: 11 TB/s of data touched, above the HBM peak, below L2's
    r = bench.roofline(4.69e9, 0.41, 0.42, rec, "test", ("k_trace_quad<false",))
    assert r["traffic"] == 60e6 and r["bound"] == "latency" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - 60e6 / 0.41e-3 / 1e9) < 1e-6 and abs(r["frac"] - r["achieved"] / 8000) < 1e-12
    lv = r["levels"]
    assert abs(lv["data"]["achieved"] - 4.69e9 / 0.41e-3 / 1e9) < 1e-6
    assert abs(lv["hbm"]["achieved"] - 60e6 / 0.41e-3 / 1e9) < 1e-6 and lv["hbm"]["frac"] < 0.1
    assert abs(lv["l2"]["achieved"] - 700e6 / 0.41e-3 / 1e9) < 1e-6 and lv["l2"]["peak"] == bench.L2_PEAK_GBS
    assert lv["data"]["peak"] == bench.L2_PEAK_GBS and lv["data"]["frac"] < 1
    assert "algorithmic" not in r  # no cache-served bytes labelled against the HBM peak any more
    r2 = bench.roofline(4.69e9, 0.41, 0.42, None, "none", ("k_trace_quad<false",))
    assert r2["traffic"] is None and "hbm" not in r2["levels"] and r2["bound"] is None


def test_l2_pass_and_per_kernel_build_traffic(tmp_path):
    write_pass(str(tmp_path / "p0"), dispatches(1), "FETCH_SIZE")
    write_pass(str(tmp_path / "p1"), dispatches(2), "WRITE_SIZE")
    write_pass(str(tmp_path / "p4"), dispatches(3), ("TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum"))
    s = pmc.summarize({"p0": str(tmp_path / "p0"), "p1": str(tmp_path / "p1"), "p4": str(tmp_path / "p4")}, PLAN)
    sing = s["segments"]["c2/single"]
    assert sing["l2_read_bytes"] == 3 * 2015 * pmc.L2_READ_REQ_BYTES
    assert sing["l2_write_bytes"] == 2 * 3 * 2015 * pmc.L2_WRITE_REQ_BYTES
    pk = s["builds"]["c2"]["per_kernel"]
    assert pk["k_gather"]["read_x2"] == 2 * 102 * 1024 and pk["k_morton"]["write"] == 202 * 1024
