"""Build libbeam_hip.so (gfx950) in-tree with hipcc.

Floating-point flags are part of the parity contract: -ffp-contract=off (no FMA contraction: the
reference's CPU arithmetic has none), correctly rounded f32 division and sqrt, denormals kept.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libbeam_hip.so")
SOURCES = ["bm_api.cpp", "bm_obj.cpp", "bm_rccl.cpp", "bm_build.hip", "bm_trace.hip", "bm_trace_ab.hip", "bm_kd.hip",
           "bm_gather.hip"]  # bm_trace_ab.hip is empty unless an A/B build defines BM_TRACE_AB=1
HEADERS = ["bm_common.h", "bm_internal.h", "bm_trace_dev.h", os.path.join("..", "..", "include", "beam_c.h")]
ARCH = os.environ.get("BM_OFFLOAD_ARCH", "gfx950")

# Per-source flags. bm_kd.hip without the SLP vectorizer: it packed the kd walks' triangle/box arithmetic
# into v_pk_* pairs whose operand shuffles (v_mov) cost more than the pairing saved.
SOURCE_FLAGS = {"bm_kd.hip": ["-fno-slp-vectorize"]}

FP_FLAGS = [
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
    "-fno-fast-math",
]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def source_stamp() -> str:
    """Content hash of the library's sources, headers and compile flags: ties a committed profile
    (profiles/*_traffic.json) to the code revision it measured (bench.py refuses other stamps)."""
    import hashlib
    h = hashlib.sha256()
    for s in sorted(SOURCES + HEADERS):
        with open(os.path.join(CSRC, s), "rb") as f:
            h.update(s.encode() + b"\0" + f.read())
    h.update(" ".join(FP_FLAGS + [ARCH]).encode())
    h.update(repr(sorted(SOURCE_FLAGS.items())).encode())
    return h.hexdigest()[:16]


STAMP_FILE = LIB + ".stamp"  # source_stamp() of the sources the in-tree library was built from


def _stale() -> bool:
    """The in-tree library is missing or was built from other sources (content stamp, not mtimes:
    a copied tree keeps its stamp file, so a pushed build is reused only when it matches)."""
    if not os.path.exists(LIB) or not os.path.exists(STAMP_FILE):
        return True
    with open(STAMP_FILE) as f:
        return f.read().strip() != source_stamp()


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=(), extra_flags=()) -> str:
    """Compile the library; `out`/`defines`/`extra_flags` build an A/B variant elsewhere (tools/).
    One hipcc per source in parallel (objects in a scratch directory next to `out`), then one link."""
    if out == LIB and (defines or extra_flags):
        # the in-tree library is the product: an A/B variant there would inherit the stamp that
        # _lib.load() trusts, so variants go elsewhere (tools/build_ab.py)
        raise ValueError("A/B variant builds (defines / extra_flags) need their own output path")
    if out == LIB and not force and not _stale():
        return LIB
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *FP_FLAGS, "-Wall", "-Wno-unused-result",
             *[f"-D{d}" for d in defines], *extra_flags]
    with tempfile.TemporaryDirectory(dir=os.path.dirname(os.path.abspath(out))) as tmp:
        objs = [os.path.join(tmp, os.path.splitext(s)[0] + ".o") for s in SOURCES]
        cmds = [[hipcc(), *flags, *SOURCE_FLAGS.get(s, []), "-c", "-o", o, os.path.join(CSRC, s)]
                for s, o in zip(SOURCES, objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c), file=sys.stderr)
        workers = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
        with ThreadPoolExecutor(max_workers=workers) as pool:
            for c, r in zip(cmds, pool.map(lambda c: subprocess.run(c, cwd=CSRC, capture_output=True, text=True),
                                           cmds)):
                if r.returncode:
                    raise RuntimeError(f"{' '.join(c)}\n{r.stdout}{r.stderr}")
                if verbose and r.stderr:
                    print(r.stderr, file=sys.stderr)
        subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs, "-ldl"],
                       check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    if out == LIB:
        with open(STAMP_FILE, "w") as f:
            f.write(source_stamp() + "\n")
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
