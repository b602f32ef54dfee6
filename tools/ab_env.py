"""A/B measurement tools only: tuning parameters from BM_* environment variables.

The library reads nothing from the environment (bm_context_set_param is the only way to change a
schedule); the A/B scripts under tools/ still select variants by environment variable, and this
module turns those into explicit parameters of the contexts the tools create."""
from __future__ import annotations

import os

from raytracercuda_amd import beam

ENV_PARAMS = {"BM_TRACE_VARIANT": "trace_variant", "BM_TRACE_SCHED": "trace_sched",
              "BM_TRACE_SCRAMBLE": "trace_scramble", "BM_TRACE_PRIO_AFTER": "trace_prio_after",
              "BM_TRACE_PRIO_LEVEL": "trace_prio_level", "BM_TRACE_REFILL_MIN": "trace_refill_min",
              "BM_CULL_TPR": "cull_tiles", "BM_TRACE_AUTO": "trace_auto_compact", "BM_TRACE_GRID": "trace_grid",
              "BM_READBACK_SYNC": "readback_sync", "BM_KD_QUEUE_CAP": "kd_queue_cap", "BM_KD_LQ_CAP": "kd_lq_cap",
              "BM_KD_SPLIT": "kd_split", "BM_KD_GRID": "kd_grid", "BM_KD_PAIR": "kd_pair", "BM_KD_TB": "kd_tb",
              "BM_KD_VARIANT": "kd_march", "BM_MSD_MAX_N": "msd_max_n", "BM_NRM_DEFER": "nrm_defer",
              "BM_BS_CAP": "bucket_lds_cap", "BM_MSD_WIDE_N": "msd_wide_n", "BM_FRONT_MAX_N": "front_max_n",
              "BM_KD_TOP_RANK": "kd_top_rank"}


def params(environ=None) -> dict:
    """{parameter name: value} of the BM_* variables set in `environ` (default os.environ)."""
    env = os.environ if environ is None else environ
    return {p: int(env[k]) for k, p in ENV_PARAMS.items() if env.get(k, "") != ""}


def Context(**kw):
    """beam.Context with the environment's A/B parameters (explicit params= entries win)."""
    return beam.Context(params={**params(), **(kw.pop("params", None) or {})}, **kw)
