"""Record layouts of include/dmclock_gpu.h as numpy dtypes and ctypes structs.

These mirror the C-ABI byte for byte (tests/test_abi.py checks the sizes and
offsets against the compiled library).
"""
import ctypes

import numpy as np

# status codes
DMC_OK = 0
DMC_EAGAIN = 11
DMC_EINVAL = -1
DMC_ENOMEM = -2
DMC_EDEVICE = -3
DMC_EBADTAG = -1001
DMC_EBADPARAMS = -1002
DMC_EQUEUEFULL = -1004
DMC_ENOTREG = -1005
DMC_ENOTRUN = -1006  # pipelined: the previous call failed, this one was not executed
ABI_VERSION = 7  # include/dmclock_gpu.h DMC_ABI_VERSION

# AtLimit (dmclock_server.h:74-84)
AT_LIMIT_WAIT = 0
AT_LIMIT_ALLOW = 1
AT_LIMIT_REJECT = 2

# NextReqType (dmclock_server.h:506)
NEXT_RETURNING = 0
NEXT_FUTURE = 1
NEXT_NONE = 2

# engine options (dmc_queue_set_option)
OPT_SMALL_K = 1
OPT_FORCE_RADIX = 2
OPT_GRAPHS = 3
OPT_ACT_SPLIT = 4
OPT_SAMPLE = 5
OPT_SINGLE_OP = 6
OPT_FAIL_ALLOC = 7  # test hook: fail the next n device allocations
OPT_BREAK_ROUNDS = 8
OPT_FAULT = 13
OPT_HEAP_ORDER = 11
OPT_PIPELINE = 12
OPT_SERVE = 10

# PhaseType (dmclock_recs.h:33)
PHASE_RESERVATION = 0
PHASE_PRIORITY = 1

REQUEST_DTYPE = np.dtype(
    [("slot", "<u4"), ("cost", "<u4"), ("time", "<f8"), ("delta", "<u4"),
     ("rho", "<u4"), ("handle", "<u8")], align=True)
assert REQUEST_DTYPE.itemsize == 32

DECISION_DTYPE = np.dtype(
    [("handle", "<u8"), ("tag_r", "<f8"), ("tag_p", "<f8"), ("tag_l", "<f8"),
     ("slot", "<u4"), ("cost", "<u4"), ("phase", "<u4"), ("flags", "<u4")],
    align=True)
assert DECISION_DTYPE.itemsize == 48


class QueueParams(ctypes.Structure):
    _fields_ = [
        ("max_clients", ctypes.c_uint32),
        ("ring_capacity", ctypes.c_uint32),
        ("max_batch", ctypes.c_uint32),
        ("delayed", ctypes.c_int32),
        ("dynamic_info", ctypes.c_int32),
        ("at_limit", ctypes.c_int32),
        ("reject_threshold", ctypes.c_double),
        ("anticipation_timeout", ctypes.c_double),
        ("device", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class PullResult(ctypes.Structure):
    _fields_ = [
        ("n_decisions", ctypes.c_uint32),
        ("next_type", ctypes.c_uint32),
        ("when", ctypes.c_double),
        ("n_reservation", ctypes.c_uint32),
        ("n_priority", ctypes.c_uint32),
    ]


class ClientState(ctypes.Structure):
    _fields_ = [
        ("prev_r", ctypes.c_double), ("prev_p", ctypes.c_double),
        ("prev_l", ctypes.c_double), ("prev_arrival", ctypes.c_double),
        ("prop_delta", ctypes.c_double),
        ("front_r", ctypes.c_double), ("front_p", ctypes.c_double),
        ("front_l", ctypes.c_double), ("front_arrival", ctypes.c_double),
        ("r_inv", ctypes.c_double), ("w_inv", ctypes.c_double),
        ("l_inv", ctypes.c_double),
        ("last_tick", ctypes.c_uint64),
        ("count", ctypes.c_uint32),
        ("cur_delta", ctypes.c_uint32), ("cur_rho", ctypes.c_uint32),
        ("idle", ctypes.c_uint8), ("front_ready", ctypes.c_uint8),
        ("registered", ctypes.c_uint8), ("pad", ctypes.c_uint8),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_
                if name != "pad"}


class Stats(ctypes.Structure):
    _fields_ = [
        ("tick", ctypes.c_uint64),
        ("reserv_sched_count", ctypes.c_uint64),
        ("prop_sched_count", ctypes.c_uint64),
        ("limit_break_sched_count", ctypes.c_uint64),
        ("clients", ctypes.c_uint64),
        ("requests", ctypes.c_uint64),
    ]


class Counters(ctypes.Structure):
    """dmc_counters: engine path counters (dmc_queue_counters)."""
    _fields_ = [
        ("rounds", ctypes.c_uint64),
        ("radix_rounds", ctypes.c_uint64),
        ("bin_overflows", ctypes.c_uint64),
        ("dense_overflows", ctypes.c_uint64),
        ("single_steps", ctypes.c_uint64),
        ("candidates", ctypes.c_uint64),
        ("entries", ctypes.c_uint64),
        ("decisions", ctypes.c_uint64),
        ("graph_replays", ctypes.c_uint64),
        ("fused_calls", ctypes.c_uint64),
        ("sample_retries", ctypes.c_uint64),
        ("max_bin", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("bin_splits", ctypes.c_uint64),
        ("brk_rounds", ctypes.c_uint64),
        ("brk_fallbacks", ctypes.c_uint64),
        ("bad_rounds", ctypes.c_uint64),
        ("serve_yields", ctypes.c_uint64),
        ("serve_calls", ctypes.c_uint64),
        ("serve_launches", ctypes.c_uint64),
        ("act_batches", ctypes.c_uint64),
        ("act_seq_batches", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_
                if name != "reserved"}


def make_requests(slots, times, costs=1, deltas=1, rhos=1, handles=None):
    """Build a REQUEST_DTYPE array (broadcasting scalars)."""
    slots = np.asarray(slots, dtype=np.uint32)
    n = slots.shape[0]
    out = np.zeros(n, dtype=REQUEST_DTYPE)
    out["slot"] = slots
    out["time"] = np.broadcast_to(np.asarray(times, dtype=np.float64), (n,))
    out["cost"] = np.broadcast_to(np.asarray(costs, dtype=np.uint32), (n,))
    out["delta"] = np.broadcast_to(np.asarray(deltas, dtype=np.uint32), (n,))
    out["rho"] = np.broadcast_to(np.asarray(rhos, dtype=np.uint32), (n,))
    if handles is None:
        handles = np.arange(n, dtype=np.uint64)
    out["handle"] = np.broadcast_to(np.asarray(handles, dtype=np.uint64), (n,))
    return out


class GroupTracker(ctypes.Structure):
    """dmc_group_tracker: one server's device tracker state for a group step"""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "client_of_slot", "gdelta", "grho", "xd", "xr", "known", "first",
        "comp_delta", "comp_rho")]
