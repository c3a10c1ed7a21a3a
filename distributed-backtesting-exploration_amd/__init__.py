"""MI355X-native backtest engine for the worker job path of
brendisurfs/Distributed-Backtesting-Exploration.

The reference worker's job function `process_incoming_job`
(/root/reference/src/worker/process.rs:13-29) sleeps 1 s per job. Here it is a batch call into
libbt.so (include/bt.h): CSV bytes -> HBM-resident columns -> hand-written HIP kernels
(gfx950) -> one CompleteRequest.data string per job. See DESIGN.md.

Import as `dbx_amd` (the directory name has hyphens; /root/repo/dbx_amd.py is the shim).
"""
from .engine import (ABI_VERSION, PIPE_SLOTS, BT_BOLL, BT_DAILY, BT_EMA_OLS, BT_FLAG_PARITY, BT_FLAG_TIMING, BT_MINUTE,
                     BT_SMA_CROSS, SUMMARY_DTYPE, TOPK_DTYPE, TRADE_DTYPE, BtError, Engine, Grid,
                     build, config2_grid, config3_grid, config4_grid, config5_grid, lib,
                     merge_topk)

__all__ = [
    "ABI_VERSION", "PIPE_SLOTS", "BT_BOLL", "BT_DAILY", "BT_EMA_OLS", "BT_FLAG_PARITY", "BT_FLAG_TIMING", "BT_MINUTE",
    "BT_SMA_CROSS", "SUMMARY_DTYPE", "TOPK_DTYPE", "TRADE_DTYPE", "BtError", "Engine", "Grid",
    "build", "config2_grid", "config3_grid", "config4_grid", "config5_grid", "lib", "merge_topk",
]
