"""Client-side delta/rho bookkeeping for Python callers: ServiceTracker with
OrigTracker or BorrowingTracker (/root/reference/src/dmclock_client.h).

The C++ callers use dmclock_amd/include/dmclock_client.h; the multi-GPU
deployment keeps the trackers on the device (multiserver.py).  This is the
host form the simulator driver (sim.py) uses: one instance per client,
requests and responses in event order.  Counters are unbounded Python ints
(the reference's uint64 Counter); the ReqParams values are cast to uint32
like the reference's `uint32_t(...)` (:65-66, :136-137).

The time-based server-map cleaning (do_clean, :263-286) is not modelled: a
simulation's trackers are short-lived.
"""

_U32 = 0xFFFFFFFF


class OrigTracker:
    """dmclock_client.h:39-84."""

    __slots__ = ("delta_prev_req", "rho_prev_req", "my_delta", "my_rho")

    def __init__(self, global_delta, global_rho):
        self.delta_prev_req = global_delta
        self.rho_prev_req = global_rho
        self.my_delta = 0
        self.my_rho = 0

    def prepare_req(self, the_delta, the_rho):  # :59-67
        d = the_delta - self.delta_prev_req - self.my_delta
        r = the_rho - self.rho_prev_req - self.my_rho
        self.delta_prev_req = the_delta
        self.rho_prev_req = the_rho
        self.my_delta = 0
        self.my_rho = 0
        return d & _U32, r & _U32

    def resp_update(self, phase, cost):  # :69-79 (counters updated by the caller)
        self.my_delta += cost
        if phase == 0:  # reservation
            self.my_rho += cost

    def last_delta(self):
        return self.delta_prev_req


class BorrowingTracker:
    """dmclock_client.h:90-154."""

    __slots__ = ("delta_prev_req", "rho_prev_req", "delta_borrow", "rho_borrow")

    def __init__(self, global_delta, global_rho):
        self.delta_prev_req = global_delta
        self.rho_prev_req = global_rho
        self.delta_borrow = 0
        self.rho_borrow = 0

    @staticmethod
    def _with_borrow(glob, previous, borrow):  # calc_with_borrow, :110-129
        result = glob - previous
        if result == 0:
            return 1, borrow + 1
        if result > borrow:
            return result - borrow, 0
        return 1, borrow - result + 1

    def prepare_req(self, the_delta, the_rho):  # :131-139
        d, self.delta_borrow = self._with_borrow(the_delta, self.delta_prev_req,
                                                 self.delta_borrow)
        r, self.rho_borrow = self._with_borrow(the_rho, self.rho_prev_req,
                                               self.rho_borrow)
        self.delta_prev_req = the_delta
        self.rho_prev_req = the_rho
        return d & _U32, r & _U32

    def resp_update(self, phase, cost):  # :141-149 (the counters only)
        pass

    def last_delta(self):
        return self.delta_prev_req


class ServiceTracker:
    """ServiceTracker<S, T> (dmclock_client.h:163-287): the delta / rho
    counters start at 1 (:186-187); a server seen for the first time gets
    ReqParams(1, 1) (:241-251)."""

    def __init__(self, kind="orig"):
        self.cls = OrigTracker if kind == "orig" else BorrowingTracker
        self.delta_counter = 1
        self.rho_counter = 1
        self.server_map = {}

    def track_resp(self, server, phase, cost=1):  # :221-236
        t = self.server_map.get(server)
        if t is None:
            t = self.server_map[server] = self.cls(self.delta_counter, self.rho_counter)
        self.delta_counter += cost
        if phase == 0:
            self.rho_counter += cost
        t.resp_update(phase, cost)

    def get_req_params(self, server):  # :241-251
        t = self.server_map.get(server)
        if t is None:
            self.server_map[server] = self.cls(self.delta_counter, self.rho_counter)
            return 1, 1
        return t.prepare_req(self.delta_counter, self.rho_counter)

    def server_count(self):
        return len(self.server_map)
