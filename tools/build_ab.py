#!/usr/bin/env python3
"""Build an A/B variant of libbeam_hip.so with extra -D defines (time it with BEAM_HIP_LIB=...).

    python tools/build_ab.py raytracercuda_amd/libbeam_hip_w8.so BM_TRACE_WAVES_PER_EU=8
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracercuda_amd import build  # noqa: E402

if __name__ == "__main__":
    print(build.build(out=os.path.abspath(sys.argv[1]), defines=sys.argv[2:], verbose=True))
