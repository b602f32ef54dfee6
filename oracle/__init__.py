"""CPU oracle for the Beam primary-ray hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker (or the timed CPU baseline), never as the thing measured or shipped.
The product (raytracercuda_amd) never imports it and fails loudly without its HIP library.

See beam_oracle.h for what is restated (reference file:line) and the parity status.
"""
from .oracle import Oracle, OrcMeshes, load_oracle  # noqa: F401
