"""raytracercuda_amd — MI355X-native (gfx950) BVH build + primary-ray trace behind the reference's
Beam Scene/Mesh/Camera/RenderTarget API.

Native code: libbeam_hip.so (raytracercuda_amd/csrc: HIP kernels + the C ABI of include/beam_c.h).
Python: `beam` mirrors the reference's interface classes over that ABI; `scenes` holds the
synthetic workloads; `multigpu` the screen-band partition + RCCL gather.
"""
__all__ = ["beam", "scenes", "multigpu"]
