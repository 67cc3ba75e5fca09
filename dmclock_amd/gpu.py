"""ctypes binding of the HIP engine's C-ABI (include/dmclock_gpu.h).

`GpuQueue` exposes the same Python surface as the CPU restatement used by the
tests (set_info / add / pull / pull_batch / ...), so that one driver can run a
trace through both.  Like the C++ facade (dmclock_amd/include/dmclock_server.h)
it maps the reference's client ids to dense device slots and models
client_info_f: the ClientInfo a client maps to can be mutated in place (seen at
once, as through the reference's cached pointer) or replaced by a fresh object
(seen after update_client_info, or at every tag with dynamic_info / U1).

There is no CPU fallback: the engine library must be present and a HIP device
must exist, or construction fails loudly.
"""
import ctypes
import os

import numpy as np

from ._abi import (DECISION_DTYPE, REQUEST_DTYPE, ClientState, Counters,
                   PullResult, QueueParams, Stats, make_requests)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DMC_LIB: an alternative build of the same C-ABI (A/B runs of variants,
# scripts/gpu_ab_run.sh); default: the in-tree library
LIB_PATH = os.environ.get("DMC_LIB") or os.path.join(_HERE, "libdmclock_gpu.so")
_lib = None

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_i32 = ctypes.c_int
_f64 = ctypes.c_double

EXPORTS = {
    "dmc_queue_create": (_i32, [ctypes.POINTER(QueueParams), ctypes.POINTER(_vp)]),
    "dmc_queue_destroy": (_i32, [_vp]),
    "dmc_queue_stream": (_vp, [_vp]),
    "dmc_queue_sync": (_i32, [_vp]),
    "dmc_strerror": (ctypes.c_char_p, [_i32]),
    "dmc_client_register": (_i32, [_vp, _u32, _f64, _f64, _f64, _i32]),
    "dmc_client_register_batch": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _i32]),
    "dmc_client_update_info": (_i32, [_vp, _u32, _f64, _f64, _f64]),
    "dmc_client_bind_info_batch": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "dmc_queue_set_info_fn": (_i32, [_vp, _vp, _vp]),
    "dmc_client_mark_idle": (_i32, [_vp, _u32]),
    "dmc_client_mark_idle_batch": (_i32, [_vp, _u32, _vp]),
    "dmc_client_mark_idle_batch_device": (_i32, [_vp, _u32, _vp]),
    "dmc_client_erase": (_i32, [_vp, _u32, _vp, _u32, ctypes.POINTER(_u32)]),
    "dmc_client_get_state": (_i32, [_vp, _u32, ctypes.POINTER(ClientState)]),
    "dmc_client_last_ticks": (_i32, [_vp, _u32, _vp]),
    "dmc_add_batch": (_i32, [_vp, _u32, _vp, _vp]),
    "dmc_add_batch_device": (_i32, [_vp, _u32, _vp, _vp]),
    "dmc_pull_batch": (_i32, [_vp, _f64, _u32, _vp, ctypes.POINTER(PullResult)]),
    "dmc_pull_batch_device": (_i32, [_vp, _f64, _u32, _vp, _vp]),
    "dmc_add_pull_batch_device": (_i32, [_vp, _u32, _vp, _vp, _f64, _u32, _vp, _vp]),
    "dmc_remove_by_client": (_i32, [_vp, _u32, _i32, _vp, _u32,
                                    ctypes.POINTER(_u32)]),
    "dmc_client_requests": (_i32, [_vp, _u32, _vp, _u32, ctypes.POINTER(_u32)]),
    "dmc_client_filter": (_i32, [_vp, _u32, _u32, _vp]),
    "dmc_queue_requests": (_i32, [_vp, _vp, _vp, ctypes.c_uint64,
                                  ctypes.POINTER(ctypes.c_uint64)]),
    "dmc_queue_filter": (_i32, [_vp, _vp, ctypes.c_uint64, ctypes.POINTER(_i32)]),
    "dmc_client_erase_batch": (_i32, [_vp, _u32, _vp, _vp, _vp, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "dmc_stats_get": (_i32, [_vp, ctypes.POINTER(Stats)]),
    "dmc_queue_set_option": (_i32, [_vp, _i32, ctypes.c_int64]),
    "dmc_queue_counters": (_i32, [_vp, ctypes.POINTER(Counters), _i32]),
    "dmc_queue_counters_sized": (_i32, [_vp, _vp, ctypes.c_uint64, _i32]),
    "dmc_abi_version": (_i32, []),
    "dmc_queue_pipelined_error": (_i32, [_vp, _i32]),
    "dmc_tracker_tally": (_i32, [_vp, _vp, _vp, _u32, _vp, _vp]),
    "dmc_tracker_fill": (_i32, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp]),
    "dmc_tracker_collect": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dmc_tracker_advance": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "dmc_tracker_collect_sums": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "dmc_tracker_commit": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "dmc_group_create": (_i32, [_vp, _u32, ctypes.POINTER(_vp)]),
    "dmc_group_destroy": (_i32, [_vp]),
    "dmc_group_stream": (_vp, [_vp]),
    "dmc_group_tracker_collect_sums": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "dmc_group_tracker_join": (_i32, [_vp]),
    "dmc_group_side_stream": (_vp, [_vp]),
    "dmc_group_step_device": (_i32, [_vp, _u32, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    "dmc_group_profile_enable": (_i32, [_vp, _i32]),
    "dmc_group_profile_read": (_i32, [_vp, _u32, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(_f64)]),
    "dmc_profile_enable": (_i32, [_vp, _i32]),
    "dmc_profile_reset": (_i32, [_vp]),
    "dmc_profile_read": (_i32, [_vp, _u32, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(_f64)]),
    "dmc_profile_stage_name": (ctypes.c_char_p, [_u32]),
}
PROF_NSTAGES = 14

# dmc_info_fn: int (*)(void* ctx, uint32_t slot, double* r, double* w, double* l)
INFO_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _u32, ctypes.POINTER(_f64),
                           ctypes.POINTER(_f64), ctypes.POINTER(_f64))


class DmcError(RuntimeError):
    pass


def lib():
    """Load the engine library (no fallback: raises if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DmcError(
                f"{LIB_PATH} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            if os.environ.get("DMC_LIB") and not hasattr(L, name):
                continue  # (an A/B variant built before this entry point existed)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        msg = lib().dmc_strerror(rc).decode()
        raise DmcError(f"{what}: {msg} ({rc})")


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class GpuQueue:
    """One dmClock server queue on one HIP device."""

    def __init__(self, max_clients=1024, ring_capacity=64, max_batch=1 << 16,
                 delayed=False, dynamic_info=False, at_limit=0,
                 reject_threshold=0.0, anticipation=0.0, device=0,
                 branching=2, track_ties=True, info_callback=True, heap_order=False):
        """info_callback (U1 only): client_info_f through the engine's
        dmc_info_fn; False: the caller publishes changes with bind_info
        (explicit_bind), the device-API callers' contract.  heap_order:
        tie-exact dispatch (DMC_OPT_HEAP_ORDER, the reference's `branching`-ary
        heaps on the device); otherwise branching has no meaning (no heaps)."""
        del track_ties
        self.L = lib()
        p = QueueParams()
        p.max_clients = max_clients
        p.ring_capacity = ring_capacity
        p.max_batch = max_batch
        p.delayed = int(delayed)
        p.dynamic_info = int(dynamic_info)
        p.at_limit = at_limit
        p.reject_threshold = float(reject_threshold)
        p.anticipation_timeout = float(anticipation)
        p.device = device
        h = _vp()
        _check(self.L.dmc_queue_create(ctypes.byref(p), ctypes.byref(h)),
               "dmc_queue_create")
        self.h = h
        self.params = p
        if heap_order:
            from ._abi import OPT_HEAP_ORDER
            _check(self.L.dmc_queue_set_option(self.h, OPT_HEAP_ORDER, int(branching)),
                   "set_option(HEAP_ORDER)")
        self.dynamic = bool(dynamic_info)
        self.slot_of = {}      # client id -> slot
        self.client_of = []    # slot -> client id
        self.info_cur = {}     # client -> (r, w, l) client_info_f returns now
        self.info_dev = {}     # client -> (r, w, l) last pushed by update_info
        self._info_fn = None
        self.explicit_bind = self.dynamic and not info_callback
        if self.dynamic and info_callback:
            # U1: the engine asks for client_info_f(client) right before each
            # tag calculation of a host-API call (dmc_queue_set_info_fn)
            def info_fn(ctx, slot, r, w, l):
                try:
                    v = self.info_cur[self.client_of[slot]]
                except (KeyError, IndexError):
                    return 1
                r[0], w[0], l[0] = v
                return 0
            self._info_fn = INFO_FN(info_fn)  # keep the closure alive
            _check(self.L.dmc_queue_set_info_fn(self.h, ctypes.cast(self._info_fn, _vp),
                                                None), "set_info_fn")

    def close(self):
        if getattr(self, "h", None):
            self.L.dmc_queue_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- client_info_f model
    def set_info(self, client, r, w, l, fresh=False):
        self.info_cur[client] = (float(r), float(w), float(l))
        if not fresh and client in self.slot_of:
            self._push_info(client, force=self.dynamic)

    def bind_info(self, slots, r, w, l):
        """dmc_client_bind_info_batch: what client_info_f returns for these
        slots from now on (read at every tag calculation under U1)"""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        r = np.ascontiguousarray(r, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        l = np.ascontiguousarray(l, dtype=np.float64)
        _check(self.L.dmc_client_bind_info_batch(self.h, len(slots), _ptr(slots),
                                                 _ptr(r), _ptr(w), _ptr(l)),
               "bind_info_batch")

    def _push_info(self, client, force=False):
        # under U1 the device's cached info also changes at tag calculations,
        # so update_client_info always pushes
        v = self.info_cur[client]
        if force or self.info_dev.get(client) != v:
            _check(self.L.dmc_client_update_info(self.h, self.slot_of[client],
                                                 *v), "update_info")
            self.info_dev[client] = v

    def _slot(self, client):
        s = self.slot_of.get(client)
        if s is None:
            s = len(self.client_of)
            r, w, l = self.info_cur[client]
            _check(self.L.dmc_client_register(self.h, s, r, w, l, 0),
                   "register")
            self.slot_of[client] = s
            self.client_of.append(client)
            self.info_dev[client] = (r, w, l)
        return s

    def register_active(self, slots, r, w, l):
        """Bulk registration (deviation shared with the oracle): client id ==
        slot, idle=false, prop_delta=0."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        r = np.ascontiguousarray(r, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        l = np.ascontiguousarray(l, dtype=np.float64)
        _check(self.L.dmc_client_register_batch(self.h, len(slots), _ptr(slots),
                                                _ptr(r), _ptr(w), _ptr(l), 1),
               "register_batch")
        for i, s in enumerate(slots.tolist()):
            self.slot_of[s] = s
            self.info_cur[s] = self.info_dev[s] = (r[i], w[i], l[i])
        if len(self.client_of) < int(slots.max()) + 1:
            self.client_of.extend(range(len(self.client_of),
                                        int(slots.max()) + 1))

    def register(self, slots, r, w, l, active):
        """Register clients with client id == slot (trace drivers)."""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        r = np.ascontiguousarray(r, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        l = np.ascontiguousarray(l, dtype=np.float64)
        _check(self.L.dmc_client_register_batch(self.h, len(slots), _ptr(slots),
                                                _ptr(r), _ptr(w), _ptr(l),
                                                int(active)), "register_batch")
        top = int(slots.max()) + 1 if len(slots) else 0
        if len(self.client_of) < top:
            self.client_of.extend(range(len(self.client_of), top))
        for i, s in enumerate(slots.tolist()):
            self.slot_of[s] = s
            self.info_cur[s] = self.info_dev[s] = (r[i], w[i], l[i])

    # ---- hot path
    def add(self, client, time, delta=1, rho=1, cost=1, handle=0):
        s = self._slot(client)
        req = make_requests([s], [time], [cost], [delta], [rho], [handle])
        return int(self.add_batch(req)[0])

    def add_batch(self, reqs):
        """reqs: REQUEST_DTYPE array whose `slot` field holds device slots."""
        reqs = np.ascontiguousarray(reqs, dtype=REQUEST_DTYPE)
        rc = np.zeros(len(reqs), dtype=np.int32)
        _check(self.L.dmc_add_batch(self.h, len(reqs), _ptr(reqs), _ptr(rc)),
               "add_batch")
        return rc

    def pull(self, now):
        d, res = self.pull_batch(now, 1)
        if res.n_decisions:
            rec = d[0].copy()
            rec["slot"] = self.client_of[int(rec["slot"])]
            return 0, rec, 0.0
        return res.next_type, None, res.when

    def pull_batch(self, now, k):
        # a reused output buffer (first-touch page faults on a fresh 3 MB
        # array per call cost as much as the transfer); callers get a copy
        if getattr(self, "_out", None) is None or len(self._out) < max(k, 1):
            self._out = np.empty(max(k, 1), dtype=DECISION_DTYPE)
        out = self._out
        res = PullResult()
        _check(self.L.dmc_pull_batch(self.h, float(now), k, _ptr(out),
                                     ctypes.byref(res)), "pull_batch")
        return out[:res.n_decisions].copy(), res

    # ---- device-pointer variants (bench)
    def add_batch_device(self, d_reqs_ptr, n, d_rc_ptr):
        _check(self.L.dmc_add_batch_device(self.h, n, d_reqs_ptr, d_rc_ptr),
               "add_batch_device")

    def pull_batch_device(self, now, k, d_out_ptr, d_res_ptr=None):
        _check(self.L.dmc_pull_batch_device(self.h, float(now), k, d_out_ptr,
                                            d_res_ptr), "pull_batch_device")

    def add_pull_batch_device(self, d_reqs_ptr, n, d_rc_ptr, now, k, d_out_ptr,
                              d_res_ptr=None):
        """add_batch_device then pull_batch_device(now, k), fused into one
        graph launch when possible"""
        _check(self.L.dmc_add_pull_batch_device(self.h, n, d_reqs_ptr, d_rc_ptr,
                                                float(now), k, d_out_ptr, d_res_ptr),
               "add_pull_batch_device")

    def stream(self):
        return self.L.dmc_queue_stream(self.h)

    def sync(self):
        _check(self.L.dmc_queue_sync(self.h), "queue_sync")

    def set_option(self, option, value):
        _check(self.L.dmc_queue_set_option(self.h, option, int(value)),
               "set_option")

    def pipelined_error(self, clear=True):
        """DMC_OPT_PIPELINE: the error of the last pipelined call that a
        later call found failed (0: none) -- what a DMC_ENOTRUN stands for"""
        return self.L.dmc_queue_pipelined_error(self.h, int(clear))

    def counters(self, reset=False):
        """engine path counters (rounds, radix rounds, overflows, largest
        rank bin) since creation or the last reset"""
        c = Counters()
        _check(self.L.dmc_queue_counters(self.h, ctypes.byref(c), int(reset)),
               "queue_counters")
        return c.as_dict()

    # ---- stage timers (HIP events on the queue's stream)
    def profile(self, on=True):
        _check(self.L.dmc_profile_enable(self.h, int(on)), "profile_enable")

    def profile_reset(self):
        _check(self.L.dmc_profile_reset(self.h), "profile_reset")

    def profile_read(self):
        out = {}
        for st in range(PROF_NSTAGES):
            c, ms = ctypes.c_uint64(0), _f64(0.0)
            _check(self.L.dmc_profile_read(self.h, st, ctypes.byref(c),
                                           ctypes.byref(ms)), "profile_read")
            out[self.L.dmc_profile_stage_name(st).decode()] = (c.value, ms.value)
        return out

    # ---- maintenance
    def stats(self):
        st = Stats()
        _check(self.L.dmc_stats_get(self.h, ctypes.byref(st)), "stats")
        return st

    def request_count(self):
        return self.stats().requests

    def client_count(self):
        return self.stats().clients

    def sched_counts(self):
        st = self.stats()
        return st.reserv_sched_count, st.prop_sched_count

    def tick(self):
        return self.stats().tick

    def update_client_info(self, client):
        if client in self.slot_of:
            self._push_info(client, force=self.dynamic)

    def update_client_infos(self):
        for c in self.slot_of:
            self._push_info(c, force=self.dynamic)

    def remove_by_client(self, client, reverse=False):
        if client not in self.slot_of:
            return np.zeros(0, dtype=np.uint64)
        cap = self.params.ring_capacity
        out = np.zeros(cap, dtype=np.uint64)
        n = _u32(0)
        _check(self.L.dmc_remove_by_client(self.h, self.slot_of[client],
                                           int(reverse), _ptr(out), cap,
                                           ctypes.byref(n)), "remove_by_client")
        return out[:n.value].copy()

    def client_requests(self, client):
        cap = self.params.ring_capacity
        out = np.zeros(cap, dtype=np.uint64)
        n = _u32(0)
        _check(self.L.dmc_client_requests(self.h, self.slot_of[client],
                                          _ptr(out), cap, ctypes.byref(n)),
               "client_requests")
        return out[:n.value].copy()

    def queue_requests(self):
        """dmc_queue_requests: (counts per slot, every queued handle in slot
        order, FIFO per slot) in one device pass and one readback"""
        n = ctypes.c_uint64(0)
        counts = np.zeros(self.params.max_clients, dtype=np.uint32)
        _check(self.L.dmc_queue_requests(self.h, _ptr(counts), None, 0,
                                         ctypes.byref(n)), "queue_requests")
        hs = np.zeros(max(n.value, 1), dtype=np.uint64)
        _check(self.L.dmc_queue_requests(self.h, None, _ptr(hs), n.value,
                                         ctypes.byref(n)), "queue_requests")
        return counts, hs[:n.value]

    def remove_by_req_filter(self, fn, backwards=False):
        """remove_by_req_filter (dmclock_server.h:567-585): clients visited in
        ascending client-id order (std::map), each client's requests front to
        back, or back to front when `backwards`.  One readback of every queued
        handle, the filter on the host, one device compaction pass."""
        counts, hs = self.queue_requests()
        if not len(hs):
            return False
        offs = np.concatenate([[0], np.cumsum(counts, dtype=np.int64)]).astype(np.int64)
        keep = np.ones(len(hs), dtype=np.uint8)
        hl = hs.tolist()
        for c in sorted(self.slot_of):
            s = self.slot_of[c]
            a, b = int(offs[s]), int(offs[s + 1])
            order = range(b - 1, a - 1, -1) if backwards else range(a, b)
            for i in order:
                if fn(int(hl[i])):
                    keep[i] = 0
        if keep.all():
            return False
        anyr = _i32(0)
        _check(self.L.dmc_queue_filter(self.h, _ptr(keep), len(keep), ctypes.byref(anyr)),
               "queue_filter")
        return bool(anyr.value)

    def erase_batch(self, clients):
        """dmc_client_erase_batch: do_clean's erase of several clients in one
        pass; returns their queued handles (list order, FIFO per client)"""
        sl = np.ascontiguousarray([self.slot_of[c] for c in clients], dtype=np.uint32)
        n = ctypes.c_uint64(0)
        cap = len(sl) * self.params.ring_capacity
        hs = np.zeros(max(cap, 1), dtype=np.uint64)
        _check(self.L.dmc_client_erase_batch(self.h, len(sl), _ptr(sl), None, _ptr(hs),
                                             cap, ctypes.byref(n)), "erase_batch")
        return hs[:n.value].copy()

    def mark_idle_batch(self, slots):
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        _check(self.L.dmc_client_mark_idle_batch(self.h, len(slots), _ptr(slots)),
               "mark_idle_batch")

    def mark_idle_batch_device(self, d_slots_ptr, n):
        """dmc_client_mark_idle_batch_device: the slot list in HBM"""
        _check(self.L.dmc_client_mark_idle_batch_device(self.h, n, d_slots_ptr),
               "mark_idle_batch_device")

    def mark_idle(self, client):
        _check(self.L.dmc_client_mark_idle(self.h, self.slot_of[client]),
               "mark_idle")

    def erase(self, client):
        if client not in self.slot_of:
            return False
        n = _u32(0)
        _check(self.L.dmc_client_erase(self.h, self.slot_of[client], None, 0,
                                       ctypes.byref(n)), "erase")
        return True

    def client_state(self, client):
        s = ClientState()
        slot = self.slot_of.get(client, client)
        rc = self.L.dmc_client_get_state(self.h, slot, ctypes.byref(s))
        return s if rc == 0 else None

    def last_ticks(self, n):
        out = np.zeros(n, dtype=np.uint64)
        _check(self.L.dmc_client_last_ticks(self.h, n, _ptr(out)), "last_ticks")
        return out

