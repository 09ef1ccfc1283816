"""Communication layer beyond RCCL: one-shot IPC exchange of BatchNorm statistics over xGMI
(``ipc.IpcStatsExchange``).  Bulk gradient all-reduce stays on RCCL (parallel/flat.py)."""
from .ipc import (IpcStatsExchange, fallback_if_failed, setup_stats_exchange,  # noqa: F401
                  site_key, tag_sites, IpcExchangeError, StepGuard, TUNING_STEPS)
