"""CPU restatement of the epoch-delivered client trackers (TEST
INFRASTRUCTURE: imported by tests/ only, as the checker of the device kernels
in dmclock_amd/csrc/dmc_tracker.h).

It follows ServiceTracker<S, OrigTracker> of the reference
(/root/reference/src/dmclock_client.h:39-84 OrigTracker::prepare_req and
resp_update, :221-251 track_resp / get_req_params) for many clients at once,
with responses delivered in bulk at epoch boundaries; tests pin it against the
sequential restatement of the tracker (oracle/pyoracle.Tracker).

State (uint32, modular like the reference's uint32 cast of Counter
differences): per global client the delta/rho counters (start at 1), per
(server, table slot) X = delta_prev_req + my_delta (and the rho analogue) and
a `known` flag (server in server_map); client_of_slot[s][slot] names the
global client of a server's table slot (identity when None).
"""
import numpy as np


class EpochTrackers:
    """lag=True: the overlapped exchange of dmclock_amd/multiserver.py
    (DeviceTrackers(lagged=True)): an epoch's responses are handed to the
    clients at the *next* epoch boundary (its sums all-reduced meanwhile);
    finish() flushes the last one."""

    def __init__(self, n_servers, n_slots, n_clients=None, client_of_slot=None, lag=False):
        G = n_slots if n_clients is None else n_clients
        self.S, self.N, self.G = n_servers, n_slots, G
        if client_of_slot is None:
            client_of_slot = np.tile(np.arange(n_slots, dtype=np.int64), (n_servers, 1))
        self.cmap = np.asarray(client_of_slot, np.int64)
        self.gd = np.ones(G, np.uint32)
        self.gr = np.ones(G, np.uint32)
        self.xd = np.zeros((n_servers, n_slots), np.uint32)
        self.xr = np.zeros((n_servers, n_slots), np.uint32)
        self.known = np.zeros((n_servers, n_slots), bool)
        self.comp_d = np.zeros((n_servers, n_slots), np.uint32)
        self.comp_r = np.zeros((n_servers, n_slots), np.uint32)
        self.lag = lag
        self.pend = None  # lag: (sum_d, sum_r, comp_d, comp_r) of the last epoch

    def fill(self, s, reqs):
        """get_req_params(s) for every request of `reqs` (batch order); sets
        reqs['delta'] / reqs['rho'] in place."""
        slots = reqs["slot"].astype(np.int64)
        delta = np.zeros(len(reqs), np.uint32)
        rho = np.zeros(len(reqs), np.uint32)
        _, first = np.unique(slots, return_index=True)
        c = slots[first]
        g = self.cmap[s, c]
        new = ~self.known[s, c]
        with np.errstate(over="ignore"):
            d = np.where(new, np.uint32(1), self.gd[g] - self.xd[s, c])
            r = np.where(new, np.uint32(1), self.gr[g] - self.xr[s, c])
        delta[first] = d
        rho[first] = r
        self.known[s, c] = True
        self.xd[s, c] = self.gd[g]
        self.xr[s, c] = self.gr[g]
        reqs["delta"] = delta
        reqs["rho"] = rho

    def tally(self, s, decisions):
        """track_resp's counting for one server's decisions."""
        slots = decisions["slot"].astype(np.int64)
        cost = decisions["cost"].astype(np.uint32)
        with np.errstate(over="ignore"):
            np.add.at(self.comp_d[s], slots, cost)
            res = decisions["phase"] == 0
            np.add.at(self.comp_r[s], slots[res], cost[res])

    def local_sums(self):
        """per global client: the responses of this object's servers"""
        sd = np.zeros(self.G, np.uint64)
        sr = np.zeros(self.G, np.uint64)
        np.add.at(sd, self.cmap.ravel(), self.comp_d.ravel().astype(np.uint64))
        np.add.at(sr, self.cmap.ravel(), self.comp_r.ravel().astype(np.uint64))
        return sd.astype(np.uint32), sr.astype(np.uint32)

    def deliver(self, sum_d=None, sum_r=None):
        """Epoch boundary: the global counters advance by every server's
        responses (sum_d/sum_r: the all-ranks sums; default: this object's
        servers), each server's X by its own (my_delta / my_rho).  lag: the
        previous epoch's responses are applied, this epoch's held back."""
        if sum_d is None:
            sum_d, sum_r = self.local_sums()
        if self.lag:
            prev = self.pend
            self.pend = (sum_d.copy(), sum_r.copy(), self.comp_d.copy(), self.comp_r.copy())
            self.comp_d[:] = 0
            self.comp_r[:] = 0
            if prev is not None:
                self._apply(*prev)
            return
        self._apply(sum_d, sum_r, self.comp_d, self.comp_r)
        self.comp_d[:] = 0
        self.comp_r[:] = 0

    def finish(self):
        """lag: apply the last epoch's held-back responses"""
        if self.lag and self.pend is not None:
            self._apply(*self.pend)
            self.pend = None

    def _apply(self, sum_d, sum_r, comp_d, comp_r):
        with np.errstate(over="ignore"):
            self.gd += sum_d
            self.gr += sum_r
            self.xd += comp_d
            self.xr += comp_r
