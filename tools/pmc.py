"""Live PMC counters for bench.py: HBM traffic and the limiter of the very kernels it times.

bench.py (N = 1, not already under a profiler) runs itself again as a child under
`rocprofv3 --pmc <group>` once per counter group (separate passes: FETCH_SIZE and WRITE_SIZE do not
fit one pass, MI355X_MICROARCH.md "Profiling"), with `--pmc-child PLAN`: the child builds and traces
the same workloads with nothing else launching a non-counting trace kernel, and writes the plan —
the ordered segments (config, mode, trace kind, launches) — so that the parent can cut the ordered
dispatch list of every pass into the same segments. Counters are read per dispatch (the rows of one
dispatch summed), a segment's figure is the median over its timed launches (warm-up launches
dropped), and the bytes follow the guide's HBM section: FETCH_SIZE and WRITE_SIZE are KiB; gfx950's
FETCH_SIZE counts half the bytes of wide coalesced reads, so the read side is reported as counted
and doubled, and `traffic` = doubled read + write (an upper estimate: Infinity-Cache hits are counted
as well). Builds are segmented the same way (a build starts at its k_gather dispatch).

Everything here is measurement infrastructure; no product path imports it.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import shutil
import statistics
import subprocess
import tempfile

# one counter group per rocprofv3 run (groups as tools/gpu_profile.sh has run them on the box)
GROUPS = (
    ("FETCH_SIZE",),
    ("WRITE_SIZE",),
    ("TCC_HIT_sum", "TCC_MISS_sum", "TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE"),
    ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"),
    ("TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCC_REQ_sum"),
)
# bytes per L1 -> L2 request, calibrated on gfx950 by tools/micro/l2_calib.hip (profiles/r05_l2_calib.md):
# a read request moves one 128-B line (16-B and 4-B coalesced reads and the trace's 7 x 16-B record reads
# alike: one request per 128-B line), a write request 64 B; requests x these = the bytes the L2 serves
L2_READ_REQ_BYTES = 128.0
L2_WRITE_REQ_BYTES = 64.0
# the non-counting launch kernels of every trace kind (bench.py KIND_KERNELS) and of reference mode
TRACE_PREFIXES = ("k_trace_quad<false", "k_cull<false", "k_trace_rays<false", "k_kd_march_coop<false",
                  "k_trace_persistent<false", "k_trace_pair<false", "k_trace_packet<0, false")
BUILD_FIRST = "k_gather"
BUILD_KERNELS = ("k_gather", "k_morton", "k_onesweep", "k_bucket_sort", "k_front", "k_span", "k_tree_chunk", "k_chunk_table", "k_pack",
                 "k_sort_tris", "k_emit", "k_digit_hist")


def under_profiler() -> bool:
    """True inside a rocprofv3 run (it exports ROCPROF_OUTPUT_PATH to the application)."""
    return "ROCPROF_OUTPUT_PATH" in os.environ


def short(name: str) -> str:
    n = name.replace("void ", "").replace("bm::(anonymous namespace)::", "")
    return n.split("(")[0]


def read_dispatches(pass_dir: str):
    """[(dispatch_id, short kernel name, {counter: value}, resources)] in dispatch order."""
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            e = per.get(d)
            if e is None:
                e = per[d] = (d, short(r["Kernel_Name"]), collections.defaultdict(float),
                              {"scratch_size": int(r.get("Scratch_Size") or 0),
                               "lds_block_size": int(r.get("LDS_Block_Size") or 0)})
            e[2][r["Counter_Name"]] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def segment(dispatches, plan):
    """Cut the trace dispatches into the plan's segments: {label: [[dispatch, ...] per launch]}.
    Raises ValueError when the dispatch sequence does not match the plan (then nothing is reported)."""
    seq = [d for d in dispatches if d[1].startswith(TRACE_PREFIXES)]
    out, i = {}, 0
    for s in plan:
        ks = s["kernels"]
        launches = []
        for _ in range(s["launches"]):
            grp = seq[i:i + len(ks)]
            if len(grp) != len(ks) or any(not g[1].startswith(k) for g, k in zip(grp, ks)):
                got = [g[1] for g in grp]
                raise ValueError(f"segment {s['label']}: expected {ks}, found {got}")
            launches.append(grp)
            i += len(ks)
        out[s["label"]] = launches[s.get("warmup", 0):]
    if i != len(seq):
        raise ValueError(f"{len(seq) - i} trace dispatches beyond the plan")
    return out


def builds(dispatches):
    """LBVH build launches grouped per build (a build starts at k_gather and sorts Morton keys), in
    order; reference-mode builds (k_gather, then kd kernels) are not LBVH builds and are left out."""
    groups, cur = [], None
    for d in dispatches:
        n = d[1]
        if n.startswith(BUILD_FIRST):
            cur = [d]
            groups.append(cur)
        elif cur is not None and n.startswith(BUILD_KERNELS):
            cur.append(d)
        else:
            cur = None
    return [g for g in groups if any(d[1].startswith("k_morton") for d in g)]


def _median_counter(launch_groups, counter, kernels=None):
    vals = []
    for grp in launch_groups:
        tot, seen = 0.0, False
        for d in grp:
            if kernels is not None and not d[1].startswith(kernels):
                continue
            if counter in d[2]:
                tot += d[2][counter]
                seen = True
        if seen:
            vals.append(tot)
    return statistics.median(vals) if vals else None


def limiter(launch_groups, kernel):
    """Wave-time split and cache figures of `kernel` (the longest of a launch) from the SQ/TCC/TA pass."""
    g = lambda c: _median_counter(launch_groups, c, (kernel,))  # noqa: E731
    lim = {}
    hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
    if hit is not None and miss is not None and hit + miss > 0:
        lim["l2_hit"] = hit / (hit + miss)
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for c, name in (("SQ_WAIT_ANY", "wave_time_waiting_on_loads"), ("SQ_WAIT_INST_ANY", "wave_time_issue_stalled"),
                        ("SQ_ACTIVE_INST_ANY", "wave_time_issuing")):
            if g(c) is not None:
                lim[name] = g(c) / wc
    ta, gui = g("TA_TA_BUSY_sum"), g("GRBM_GUI_ACTIVE")
    if ta is not None and gui:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; TA_TA_BUSY_sum the 256 CUs'
        lim["ta_busy"] = ta / (gui / 8 * 256)
    return lim


def bound_of(lim, hbm_frac, l2_frac=None):
    """The measured limiter, as a word: hbm (l2) when the counters put the kernel near the HBM (L2)
    roofline, otherwise the largest share of wave time: latency (parked on s_waitcnt) or issue (ready
    but stalled behind other waves' issue, or issuing)."""
    if hbm_frac is not None and hbm_frac >= 0.6:
        return "hbm"
    if l2_frac is not None and l2_frac >= 0.6:
        return "l2"
    w = lim.get("wave_time_waiting_on_loads")
    if w is None:
        return None
    other = max(lim.get("wave_time_issue_stalled", 0.0), lim.get("wave_time_issuing", 0.0))
    return "latency" if w >= other else "issue"


def summarize(pass_dirs, plan):
    """{label: record} for every plan segment plus {"builds": {config: record}} from the passes."""
    per_pass = {}
    for name, d in pass_dirs.items():
        try:
            per_pass[name] = read_dispatches(d)
        except (OSError, KeyError, ValueError) as e:
            per_pass[name] = e
    segs, errs = {}, {}
    for name, ds in per_pass.items():
        if isinstance(ds, Exception):
            errs[name] = f"{type(ds).__name__}: {ds}"
            continue
        try:
            segs[name] = segment(ds, plan["segments"])
        except ValueError as e:
            errs[name] = str(e)
    out = {"segments": {}, "builds": {}, "errors": errs}
    for s in plan["segments"]:
        lab, ks = s["label"], tuple(s["kernels"])
        rec = {"kernels": list(ks), "launches_counted": None}
        f = w = None
        if "p0" in segs:
            f = _median_counter(segs["p0"][lab], "FETCH_SIZE")
            rec["launches_counted"] = len(segs["p0"][lab])
        if "p1" in segs:
            w = _median_counter(segs["p1"][lab], "WRITE_SIZE")
        rec["read_bytes_counted"] = None if f is None else f * 1024
        rec["read_bytes_x2"] = None if f is None else 2 * f * 1024
        rec["write_bytes"] = None if w is None else w * 1024
        rec["traffic"] = None if f is None or w is None else 2 * f * 1024 + w * 1024
        lim = {}
        for pn in ("p2", "p3"):
            if pn in segs:
                lim.update(limiter(segs[pn][lab], ks[-1]))
        rec["limiter"] = lim
        if "p4" in segs:  # L1 -> L2 requests of every kernel of the launch
            rr = _median_counter(segs["p4"][lab], "TCP_TCC_READ_REQ_sum")
            wr = _median_counter(segs["p4"][lab], "TCP_TCC_WRITE_REQ_sum")
            if rr is not None and wr is not None:
                rec["l2_read_bytes"] = rr * L2_READ_REQ_BYTES
                rec["l2_write_bytes"] = wr * L2_WRITE_REQ_BYTES
                rec["l2_bytes"] = rec["l2_read_bytes"] + rec["l2_write_bytes"]
            acc = _median_counter(segs["p4"][lab], "TCP_TOTAL_CACHE_ACCESSES_sum")
            if acc is not None:
                rec["l1_tag_accesses"] = acc
        if "p0" in per_pass and not isinstance(per_pass["p0"], Exception) and "p0" in segs:
            last = segs["p0"][lab][-1] if segs["p0"][lab] else []
            rec["resources"] = {g[1]: g[3] for g in last}
        out["segments"][lab] = rec
    # builds: the plan's configs each ran `builds` builds before their traces, in plan order
    bl = {}
    for pn in ("p0", "p1"):
        ds = per_pass.get(pn)
        if ds is None or isinstance(ds, Exception):
            continue
        bl[pn] = builds(ds)
    if bl:
        k = 0
        for cfg, nb in plan.get("builds", []):
            rec = {}
            for pn, ctr, key in (("p0", "FETCH_SIZE", "read"), ("p1", "WRITE_SIZE", "write")):
                grp = bl.get(pn, [])[k:k + nb][2:]  # the first two builds allocate; the rest are steady
                v = _median_counter(grp, ctr) if grp else None
                rec[key] = v
            per_kernel = {}
            for pn, ctr, key, scale in (("p0", "FETCH_SIZE", "read_x2", 2048.0), ("p1", "WRITE_SIZE", "write", 1024.0)):
                for grp in bl.get(pn, [])[k:k + nb][2:]:
                    for d in grp:
                        if ctr in d[2]:
                            per_kernel.setdefault(d[1].split("<")[0], {}).setdefault(key, []).append(d[2][ctr] * scale)
            k += nb
            if rec.get("read") is not None and rec.get("write") is not None:
                out["builds"][cfg] = {"read_bytes_counted": rec["read"] * 1024, "read_bytes_x2": 2 * rec["read"] * 1024,
                                      "write_bytes": rec["write"] * 1024,
                                      "traffic": 2 * rec["read"] * 1024 + rec["write"] * 1024,
                                      # HBM bytes per build of each kernel (a kernel launched twice in a build
                                      # counts its launches' median twice over: medians of per-launch values)
                                      "per_kernel": {kn: {kk: statistics.median(v) * (len(v) // max(1, nb - 2))
                                                          for kk, v in kv.items()} for kn, kv in per_kernel.items()}}
    return out


def run_live(bench_py, child_args, timeout_s=150, keep_dir=None, log=None):
    """Run the counter passes of `bench.py <child_args> --pmc-child PLAN` and summarise them.
    Returns (summary or None, note). Each pass has its own time limit (SIGKILL); a failed pass only
    leaves its figures out."""
    work = tempfile.mkdtemp(prefix="bm_pmc_", dir="/tmp")
    plan_file = os.path.join(work, "plan.json")
    env = dict(os.environ, TMPDIR="/tmp")
    pass_dirs, notes = {}, []
    for i, grp in enumerate(GROUPS):
        d = os.path.join(work, f"p{i}")
        cmd = ["timeout", "-s", "KILL", str(int(timeout_s)), "rocprofv3", "--pmc", *grp, "--kernel-trace",
               "--output-format", "csv", "-d", d, "-o", "pmc", "--", "python3", bench_py, *child_args,
               "--pmc-child", plan_file]
        with open(os.path.join(work, f"p{i}.log"), "w") as lf:
            rc = subprocess.run(cmd, cwd="/tmp", env=env, stdout=lf, stderr=subprocess.STDOUT).returncode
        if log:
            log(f"pmc pass {i} ({' '.join(grp)}): rc={rc}")
        if rc != 0:
            notes.append(f"pass {' '.join(grp)} exited {rc}")
            if rc >= 124 or rc < 0:  # killed at its limit or by a signal: start no further GPU pass
                break
            continue
        pass_dirs[f"p{i}"] = d
    summary = None
    if pass_dirs and os.path.exists(plan_file):
        plan = json.load(open(plan_file))
        summary = summarize(pass_dirs, plan)
        summary["plan"] = plan
    if keep_dir:
        os.makedirs(keep_dir, exist_ok=True)
        for f in glob.glob(os.path.join(work, "*.log")) + [plan_file]:
            if os.path.exists(f):
                shutil.copy(f, keep_dir)
        for f in glob.glob(os.path.join(work, "p*", "**", "*counter_collection.csv"), recursive=True):
            shutil.copy(f, os.path.join(keep_dir, os.path.basename(os.path.dirname(f)) + "_" + os.path.basename(f)))
    shutil.rmtree(work, ignore_errors=True)
    return summary, "; ".join(notes)
