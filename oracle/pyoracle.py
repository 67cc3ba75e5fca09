"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement.

Loads oracle/libdmc_oracle.so (built by oracle/Makefile, see
__graft_entry__.build()).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product path never does.
"""
import ctypes
import os
import subprocess

import numpy as np

from dmclock_amd._abi import (DECISION_DTYPE, REQUEST_DTYPE, ClientState,
                              PullResult)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libdmc_oracle.so")
_lib = None

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int
_f64 = ctypes.c_double

FILTER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)


def build():
    """Compile the oracle library (make -C oracle)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sig = {
            "dmo_queue_create": (_vp, [_i32, _i32, _u32, _i32, _f64, _f64]),
            "dmo_queue_destroy": (None, [_vp]),
            "dmo_set_track_ties": (None, [_vp, _i32]),
            "dmo_info_set": (None, [_vp, _u32, _f64, _f64, _f64, _i32]),
            "dmo_register_active": (_i32, [_vp, _u32]),
            "dmo_register_active_batch": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp]),
            "dmo_add": (_i32, [_vp, _u64, _u32, _u32, _u32, _f64, _u32]),
            "dmo_add_batch": (_i32, [_vp, _u32, _vp, _vp]),
            "dmo_pull": (_i32, [_vp, _f64, _vp, ctypes.POINTER(_f64)]),
            "dmo_pull_batch": (_i32, [_vp, _f64, _u32, _vp,
                                      ctypes.POINTER(PullResult)]),
            "dmo_ties": (_u64, [_vp]),
            "dmo_tie_log_enable": (None, [_vp, _i32]),
            "dmo_tie_log_read": (_u64, [_vp, _vp, _u64]),
            "dmo_request_count": (_u64, [_vp]),
            "dmo_client_count": (_u64, [_vp]),
            "dmo_empty": (_i32, [_vp]),
            "dmo_tick": (_u64, [_vp]),
            "dmo_sched_counts": (None, [_vp, ctypes.POINTER(_u64),
                                        ctypes.POINTER(_u64)]),
            "dmo_remove_by_client": (_u32, [_vp, _u32, _i32, _vp, _u32]),
            "dmo_remove_by_req_filter": (_i32, [_vp, FILTER_FN, _vp, _i32]),
            "dmo_update_client_info": (None, [_vp, _u32]),
            "dmo_update_client_infos": (None, [_vp]),
            "dmo_clean": (_u64, [_vp, _u64, _u64, _u64]),
            "dmo_mark_idle": (None, [_vp, _u32]),
            "dmo_erase": (_i32, [_vp, _u32]),
            "dmo_client_state": (_i32, [_vp, _u32, ctypes.POINTER(ClientState)]),
            "dmo_client_tags": (_u32, [_vp, _u32, _vp, _u32]),
            "dmo_iheap_create": (_vp, [_u32, _i32, _i32]),
            "dmo_iheap_destroy": (None, [_vp]),
            "dmo_ielem_new": (_i32, [_vp, _i32]),
            "dmo_iheap_push": (None, [_vp, _vp, _i32]),
            "dmo_ielem_set": (None, [_vp, _i32, _i32]),
            "dmo_iheap_top": (_i32, [_vp]),
            "dmo_iheap_size": (_i32, [_vp]),
            "dmo_iheap_pop": (None, [_vp]),
            "dmo_iheap_promote": (None, [_vp, _vp, _i32]),
            "dmo_iheap_demote": (None, [_vp, _vp, _i32]),
            "dmo_iheap_adjust": (None, [_vp, _vp, _i32]),
            "dmo_iheap_remove_value": (_i32, [_vp, _i32]),
            "dmo_iheap_dump": (_i32, [_vp, _vp, _i32]),
            "dmo_tracker_create": (_vp, [_i32]),
            "dmo_tracker_destroy": (None, [_vp]),
            "dmo_tracker_track_resp": (None, [_vp, _u32, _i32, _u64]),
            "dmo_tracker_get_req_params": (None, [_vp, _u32,
                                                  ctypes.POINTER(_u32),
                                                  ctypes.POINTER(_u32)]),
            "dmo_now_seconds": (_f64, []),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleQueue:
    """PullPriorityQueue restated on the CPU (tie-exact, heap based)."""

    def __init__(self, delayed=False, dynamic_info=False, branching=2,
                 at_limit=0, reject_threshold=0.0, anticipation=0.0,
                 track_ties=True):
        self.L = lib()
        self.h = self.L.dmo_queue_create(int(delayed), int(dynamic_info),
                                         branching, at_limit,
                                         float(reject_threshold),
                                         float(anticipation))
        self.L.dmo_set_track_ties(self.h, int(track_ties))

    def close(self):
        if self.h:
            self.L.dmo_queue_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # client_info_f model
    def set_info(self, client, r, w, l, fresh=False):
        self.L.dmo_info_set(self.h, client, r, w, l, int(fresh))

    def register_active(self, clients, r, w, l):
        clients = np.ascontiguousarray(clients, dtype=np.uint32)
        r = np.ascontiguousarray(r, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        l = np.ascontiguousarray(l, dtype=np.float64)
        rc = self.L.dmo_register_active_batch(self.h, len(clients),
                                              _ptr(clients), _ptr(r), _ptr(w),
                                              _ptr(l))
        assert rc == 0, rc

    def register(self, clients, r, w, l, active):
        """Trace-driver registration: active -> bulk registration; inactive
        -> only client_info_f is defined (the record is created, idle, by the
        client's first add_request, dmclock_server.h:920-932)."""
        if active:
            self.register_active(clients, r, w, l)
        else:
            for c, a, b, d in zip(np.asarray(clients).tolist(), r, w, l):
                self.set_info(c, float(a), float(b), float(d))

    def add(self, client, time, delta=1, rho=1, cost=1, handle=0):
        return self.L.dmo_add(self.h, handle, client, delta, rho, time, cost)

    def add_batch(self, reqs):
        reqs = np.ascontiguousarray(reqs, dtype=REQUEST_DTYPE)
        rc = np.zeros(len(reqs), dtype=np.int32)
        self.L.dmo_add_batch(self.h, len(reqs), _ptr(reqs), _ptr(rc))
        return rc

    def pull(self, now):
        """One pull_request(now): (type, decision-record or None, when)."""
        d = np.zeros(1, dtype=DECISION_DTYPE)
        when = ctypes.c_double(0.0)
        t = self.L.dmo_pull(self.h, now, _ptr(d), ctypes.byref(when))
        return t, (d[0] if t == 0 else None), when.value

    def pull_batch(self, now, k):
        out = np.zeros(k, dtype=DECISION_DTYPE)
        res = PullResult()
        self.L.dmo_pull_batch(self.h, now, k, _ptr(out), ctypes.byref(res))
        return out[:res.n_decisions].copy(), res

    @property
    def ties(self):
        return self.L.dmo_ties(self.h)

    def tie_log(self, on=True):
        """tie study: log every tied decision's tied set"""
        self.L.dmo_tie_log_enable(self.h, int(on))

    def read_tie_log(self):
        """[(heap, chosen slot, [(slot, front arrival, front_since,
        last_tick), ...])] since the last read (the top first)"""
        n = self.L.dmo_tie_log_read(self.h, None, 0)
        buf = np.zeros(max(n, 1), np.uint64)
        self.L.dmo_tie_log_read(self.h, _ptr(buf), n)
        out, i = [], 0
        while i < n:
            heap, chosen, m = int(buf[i]), int(buf[i + 1]), int(buf[i + 2])
            i += 3
            mem = []
            for _ in range(m):
                mem.append((int(buf[i]), float(buf[i + 1:i + 2].view(np.float64)[0]),
                            int(buf[i + 2]), int(buf[i + 3])))
                i += 4
            out.append((heap, chosen, mem))
        return out

    def request_count(self):
        return self.L.dmo_request_count(self.h)

    def client_count(self):
        return self.L.dmo_client_count(self.h)

    def empty(self):
        return bool(self.L.dmo_empty(self.h))

    def tick(self):
        return self.L.dmo_tick(self.h)

    def sched_counts(self):
        a, b = _u64(0), _u64(0)
        self.L.dmo_sched_counts(self.h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def remove_by_client(self, client, reverse=False):
        cap = 1 << 16
        out = np.zeros(cap, dtype=np.uint64)
        n = self.L.dmo_remove_by_client(self.h, client, int(reverse),
                                        _ptr(out), cap)
        return out[:n].copy()

    def remove_by_req_filter(self, fn, backwards=False):
        cb = FILTER_FN(lambda h, ctx: 1 if fn(int(h)) else 0)
        return bool(self.L.dmo_remove_by_req_filter(self.h, cb, None,
                                                    int(backwards)))

    def update_client_info(self, client):
        self.L.dmo_update_client_info(self.h, client)

    def update_client_infos(self):
        self.L.dmo_update_client_infos(self.h)

    def clean(self, erase_point, idle_point, erase_max=2000):
        return self.L.dmo_clean(self.h, erase_point, idle_point, erase_max)

    def mark_idle(self, client):
        self.L.dmo_mark_idle(self.h, client)

    def erase(self, client):
        return bool(self.L.dmo_erase(self.h, client))

    def client_state(self, client):
        s = ClientState()
        rc = self.L.dmo_client_state(self.h, client, ctypes.byref(s))
        return s if rc == 0 else None

    def client_tags(self, client):
        cap = 4096
        out = np.zeros(3 * cap, dtype=np.float64)
        n = self.L.dmo_client_tags(self.h, client, _ptr(out), cap)
        return out[:3 * n].reshape(n, 3).copy()


class IntHeap:
    """IndIntruHeap over ints (support/src/indirect_intrusive_heap.h)."""

    def __init__(self, k=2, mode=0, alt_index=False):
        self.L = lib()
        self.h = self.L.dmo_iheap_create(k, mode, int(alt_index))

    def __del__(self):
        try:
            self.L.dmo_iheap_destroy(self.h)
        except Exception:
            pass

    def new(self, value):
        return self.L.dmo_ielem_new(self.h, value)

    def push_value(self, value):
        e = self.new(value)
        self.push(self, e)
        return e

    def push(self, src, eid):
        self.L.dmo_iheap_push(self.h, src.h, eid)

    def set(self, eid, value):
        self.L.dmo_ielem_set(self.h, eid, value)

    def top(self):
        return self.L.dmo_iheap_top(self.h)

    def __len__(self):
        return self.L.dmo_iheap_size(self.h)

    def pop(self):
        self.L.dmo_iheap_pop(self.h)

    def promote(self, src, eid):
        self.L.dmo_iheap_promote(self.h, src.h, eid)

    def demote(self, src, eid):
        self.L.dmo_iheap_demote(self.h, src.h, eid)

    def adjust(self, src, eid):
        self.L.dmo_iheap_adjust(self.h, src.h, eid)

    def remove_value(self, value):
        return bool(self.L.dmo_iheap_remove_value(self.h, value))

    def dump(self):
        out = np.zeros(len(self) + 1, dtype=np.int32)
        n = self.L.dmo_iheap_dump(self.h, _ptr(out), len(out))
        return out[:n].tolist()


class Tracker:
    """ServiceTracker<S, OrigTracker|BorrowingTracker> (dmclock_client.h)."""

    def __init__(self, kind="orig"):
        self.L = lib()
        self.h = self.L.dmo_tracker_create(0 if kind == "orig" else 1)

    def __del__(self):
        try:
            self.L.dmo_tracker_destroy(self.h)
        except Exception:
            pass

    def track_resp(self, server, phase, cost=1):
        self.L.dmo_tracker_track_resp(self.h, server, phase, cost)

    def get_req_params(self, server):
        d, r = _u32(0), _u32(0)
        self.L.dmo_tracker_get_req_params(self.h, server, ctypes.byref(d),
                                          ctypes.byref(r))
        return d.value, r.value
