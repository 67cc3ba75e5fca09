"""Multi-server dmClock on the device (BASELINE config 5).

dmClock servers are independent queues (sim/src/simulate.h:118-136; one queue
per server, sim/src/sim_server.h:84,123-130); the only coupling between them
is client side: every request carries delta/rho, the responses the client got
from the *other* servers since its previous request to this one
(ServiceTracker<S, OrigTracker>, dmclock_client.h:39-84, 163-287).

Here the clients' trackers live on the device next to the server queues
(dmclock_amd/csrc/dmc_tracker.h) and responses are delivered at epoch
boundaries: per epoch each server's decisions are tallied per client, the
per-client sums over all servers are combined across ranks with one
all-reduce (RCCL over xGMI for one process per GPU; gloo on CPU), and each
tracker advances by its own responses.  That all-reduce is the one exchange
step of the deployment; the dispatch path itself has no collective.

Arrays are torch tensors (device memory and the collective); every
computation on them is an engine kernel behind the C-ABI.
"""
import ctypes

import numpy as np

from .gpu import PROF_NSTAGES, GpuQueue, _check, lib

U32_NONE = -1  # 0xffffffff as int32


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class DeviceTrackers:
    """Client trackers for the S servers (queues) of one rank.

    Each server table has n_slots client slots; client_of_slot (S x n_slots,
    int32, optional; identity when None) names the global client of each
    slot, of n_clients global clients (default n_slots).  Per (server, slot):
    X_delta, X_rho, known; per global client: the delta/rho counters.

    lagged=False: deliver() hands each epoch's responses to the clients at
    that epoch's end (collect, all-reduce, advance, in sequence).
    lagged=True (the overlapped exchange): deliver()
    forms the epoch's per-client sums and starts their all-reduce, which runs
    while the next epoch's steps do; the responses reach the clients' counters
    at the next deliver() (finish() flushes the last one).  Per-slot tallies
    are double-buffered so that the next epoch tallies into the other half."""

    def __init__(self, queues, n_slots, device, n_clients=None, client_of_slot=None,
                 lagged=False):
        import torch
        self.torch = torch
        self.queues = list(queues)
        S, N = len(self.queues), n_slots
        G = n_clients if n_clients is not None else n_slots
        i32 = torch.int32
        self.N, self.G = N, G
        self.lagged = lagged
        if client_of_slot is not None:
            client_of_slot = torch.as_tensor(client_of_slot, dtype=i32).to(device)
            if tuple(client_of_slot.shape) != (S, N):
                raise ValueError("client_of_slot must be (servers, n_slots)")
            if int(client_of_slot.min()) < 0 or int(client_of_slot.max()) >= G:
                raise ValueError("client_of_slot out of range")
        self.cmap = client_of_slot
        self.gd = torch.ones(G, dtype=i32, device=device)
        self.gr = torch.ones(G, dtype=i32, device=device)
        # persistent all-reduce buffers: [half][delta, rho][client] (one
        # collective on a contiguous (2, G) block, no per-epoch stack)
        self.sums = torch.zeros((2, 2, G), dtype=i32, device=device)
        self.xd = torch.zeros((S, N), dtype=i32, device=device)
        self.xr = torch.zeros((S, N), dtype=i32, device=device)
        self.known = torch.zeros((S, N), dtype=torch.uint8, device=device)
        self.first = torch.full((S, N), U32_NONE, dtype=i32, device=device)
        self.comp = torch.zeros((2, 2, S, N), dtype=i32, device=device)
        self.cur = 0
        self.gg = None  # attach_group: the GpuGroup whose side stream collects
        self.pending = None  # lagged: (half, all-reduce work or None)
        self.allreduce_ms = []  # lagged: measured all-reduce time per epoch
        self.L = lib()
        self._gt = [None, None]
        torch.cuda.synchronize(device)

    @property
    def comp_d(self):
        return self.comp[self.cur, 0]

    @property
    def comp_r(self):
        return self.comp[self.cur, 1]

    @property
    def sum_d(self):
        return self.sums[0, 0]

    @property
    def sum_r(self):
        return self.sums[0, 1]

    def _map(self, s):
        return None if self.cmap is None else _p(self.cmap[s])

    def fill(self, s, d_reqs_ptr, n):
        """get_req_params for a batch of n requests to server s (device
        dmc_request array), on that queue's stream."""
        q = self.queues[s]
        _check(self.L.dmc_tracker_fill(q.h, ctypes.c_void_p(d_reqs_ptr), n,
                                       self._map(s), _p(self.gd), _p(self.gr),
                                       _p(self.xd[s]), _p(self.xr[s]),
                                       _p(self.known[s]), _p(self.first[s])),
               "dmc_tracker_fill")

    def tally(self, s, d_dec_ptr, d_res_ptr, cap):
        q = self.queues[s]
        _check(self.L.dmc_tracker_tally(q.h, ctypes.c_void_p(d_dec_ptr),
                                        ctypes.c_void_p(d_res_ptr), cap,
                                        _p(self.comp_d[s]), _p(self.comp_r[s])),
               "dmc_tracker_tally")

    def collect(self):
        """Epoch end, every server of the rank on its own stream: X += own
        responses, per-client sums += this server's responses."""
        for s, q in enumerate(self.queues):
            _check(self.L.dmc_tracker_collect(q.h, self.N, self._map(s),
                                              _p(self.xd[s]), _p(self.xr[s]),
                                              _p(self.comp_d[s]), _p(self.comp_r[s]),
                                              _p(self.sum_d), _p(self.sum_r)),
                   "dmc_tracker_collect")

    def _sync_queues(self):
        for q in self.queues:
            q.sync()

    def attach_group(self, group):
        """the GpuGroup the queues step in: the lagged delivery's per-client
        sums then run on the group's side stream beside its next steps
        (dmc_group_tracker_collect_sums), joined before the next commit"""
        self.gg = group

    def _collective(self, group):
        """the backend the delivery all-reduces over, None without one"""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return None
        return dist.get_backend(group)

    def _allreduce(self, buf, group, async_op):
        """the exchange step: RCCL on the device buffer (async: its work
        handle), gloo through host memory (blocking)"""
        torch = self.torch
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return None
        # (any initialized group: at world size 1 the all-reduce is the
        # identity, and RCCL still runs it on the device buffers)
        if dist.get_backend(group) == "gloo":
            host = buf.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(host)
            torch.cuda.synchronize(self.gd.device)
            return None
        if not async_op:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
            torch.cuda.synchronize(self.gd.device)
            return None
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group, async_op=True)
        work.wait()  # (the current stream waits for it; the host does not)
        ev1.record()
        return (work, ev0, ev1)

    def _advance(self, half):
        q0 = self.queues[0]
        _check(self.L.dmc_tracker_advance(q0.h, self.G, _p(self.gd), _p(self.gr),
                                          _p(self.sums[half, 0]), _p(self.sums[half, 1])),
               "dmc_tracker_advance")

    def deliver(self, group=None):
        """Epoch boundary.  Sequential: collect, one all-reduce of the
        per-client sums over the ranks (sum, modular int32), then the global
        counters advance.  Lagged: the previous epoch's delivery completes
        (commit + advance) and this epoch's sums start their all-reduce."""
        if self.lagged:
            return self._deliver_lagged(group)
        self.collect()
        self._sync_queues()
        self._allreduce(self.sums[0], group, async_op=False)
        self._advance(0)
        self.queues[0].sync()

    def _finish_pending(self):
        torch = self.torch
        half, work = self.pending
        if self.gg is not None:  # (the side stream's sums before commit and advance)
            _check(self.L.dmc_group_tracker_join(self.gg.h), "dmc_group_tracker_join")
        if work is not None:
            w, ev0, ev1 = work
            ev1.synchronize()
            self.allreduce_ms.append(ev0.elapsed_time(ev1))
        for s, q in enumerate(self.queues):
            _check(self.L.dmc_tracker_commit(q.h, self.N, _p(self.xd[s]), _p(self.xr[s]),
                                             _p(self.comp[half, 0, s]),
                                             _p(self.comp[half, 1, s])),
                   "dmc_tracker_commit")
        self._advance(half)
        self.pending = None
        del torch

    def _deliver_lagged(self, group):
        if self.pending is not None:
            self._finish_pending()
        h = self.cur
        if self.gg is not None:
            # the sums beside the next epoch's steps (they tally into the
            # other half); a collective on them waits for the side stream
            S = len(self.queues)
            vp = ctypes.c_void_p * S
            maps = vp(*[self.cmap[s].data_ptr() for s in range(S)]) \
                if self.cmap is not None else None
            _check(self.L.dmc_group_tracker_collect_sums(
                self.gg.h, self.N, maps, vp(*[self.comp[h, 0, s].data_ptr() for s in range(S)]),
                vp(*[self.comp[h, 1, s].data_ptr() for s in range(S)]),
                _p(self.sums[h, 0]), _p(self.sums[h, 1])), "dmc_group_tracker_collect_sums")
            if self._collective(group) == "nccl":
                torch = self.torch
                side = torch.cuda.ExternalStream(self.L.dmc_group_side_stream(self.gg.h),
                                                 device=self.gd.device)
                torch.cuda.current_stream(self.gd.device).wait_stream(side)
            elif self._collective(group) is not None:  # (gloo: staged through the host)
                _check(self.L.dmc_group_tracker_join(self.gg.h), "dmc_group_tracker_join")
                self._sync_queues()
        else:
            for s, q in enumerate(self.queues):
                _check(self.L.dmc_tracker_collect_sums(q.h, self.N, self._map(s),
                                                       _p(self.comp[h, 0, s]),
                                                       _p(self.comp[h, 1, s]),
                                                       _p(self.sums[h, 0]), _p(self.sums[h, 1])),
                       "dmc_tracker_collect_sums")
            self._sync_queues()
        self.pending = (h, self._allreduce(self.sums[h], group, async_op=True))
        self.cur = 1 - h  # the next epoch tallies into the other half

    def finish(self):
        """lagged: deliver the last epoch's pending responses"""
        if self.pending is not None:
            self._finish_pending()
            self._sync_queues()

    def group_trackers(self):
        """the dmc_group_tracker array (one per server) for GpuGroup.step,
        pointing at the current tally half"""
        from ._abi import GroupTracker
        if self._gt[self.cur] is None:
            arr = (GroupTracker * len(self.queues))()
            for s in range(len(self.queues)):
                m = self.cmap[s].data_ptr() if self.cmap is not None else None
                arr[s] = GroupTracker(m, self.gd.data_ptr(), self.gr.data_ptr(),
                                      self.xd[s].data_ptr(), self.xr[s].data_ptr(),
                                      self.known[s].data_ptr(), self.first[s].data_ptr(),
                                      self.comp[self.cur, 0, s].data_ptr(),
                                      self.comp[self.cur, 1, s].data_ptr())
            self._gt[self.cur] = arr
        return self._gt[self.cur]

    def state(self):
        """host copies (tests)"""
        f = lambda t: t.cpu().numpy().view(np.uint32)
        return {"gd": f(self.gd), "gr": f(self.gr), "xd": f(self.xd),
                "xr": f(self.xr), "known": self.known.cpu().numpy().astype(bool)}


class GpuGroup:
    """The S server queues of one device driven as one (dmc_group): a step is,
    for every member, the tracker fill (optional), n adds and k pulls --
    what fill + add_pull_batch_device + tally do on each queue alone, bit for
    bit -- as one launch per kernel over all members (blockIdx.y = member),
    one graph per step."""

    def __init__(self, queues):
        self.queues = list(queues)
        self.L = lib()
        arr = (ctypes.c_void_p * len(self.queues))(*[q.h for q in self.queues])
        h = ctypes.c_void_p()
        _check(self.L.dmc_group_create(arr, len(self.queues), ctypes.byref(h)),
               "dmc_group_create")
        self.h = h

    def step(self, n, d_reqs, d_rc, nows, k, d_out, d_res, trackers=None):
        """per-member device pointers (lists of ints), per-member `now`;
        trackers: DeviceTrackers.group_trackers() or None"""
        S = len(self.queues)
        vp = ctypes.c_void_p * S
        f = (ctypes.c_double * S)(*nows)
        _check(self.L.dmc_group_step_device(
            self.h, n, vp(*d_reqs), vp(*d_rc), f, k, vp(*d_out),
            vp(*d_res) if d_res is not None else None,
            ctypes.cast(trackers, ctypes.c_void_p) if trackers is not None else None),
            "dmc_group_step_device")

    def stream(self):
        return self.L.dmc_group_stream(self.h)

    def profile(self, on=True):
        """group stage timers on (reset) / off: profiled steps run eagerly,
        each multi-table kernel timed by its own dispatch"""
        _check(self.L.dmc_group_profile_enable(self.h, int(on)), "group_profile_enable")

    def profile_read(self):
        """{stage name: (launches, total ms)} over every kernel of the
        group's profiled steps (dmc_profile_stage_name's names)"""
        out = {}
        for st in range(PROF_NSTAGES):
            c, ms = ctypes.c_uint64(0), ctypes.c_double(0.0)
            _check(self.L.dmc_group_profile_read(self.h, st, ctypes.byref(c),
                                                 ctypes.byref(ms)), "group_profile_read")
            if c.value:
                out[self.L.dmc_profile_stage_name(st).decode()] = (c.value, ms.value)
        return out

    def close(self):
        if self.h:
            _check(self.L.dmc_group_destroy(self.h), "dmc_group_destroy")
            self.h = None


def make_queues(n_servers, n_clients, device=0, **kw):
    return [GpuQueue(max_clients=n_clients, device=device, **kw)
            for _ in range(n_servers)]
