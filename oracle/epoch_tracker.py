"""CPU restatement of the epoch-delivered client trackers (TEST
INFRASTRUCTURE: imported by tests/ only, as the checker of the device kernels
in dmclock_amd/csrc/dmc_tracker.h).

It follows ServiceTracker<S, OrigTracker> of the reference
(/root/reference/src/dmclock_client.h:39-84 OrigTracker::prepare_req and
resp_update, :221-251 track_resp / get_req_params) for many clients at once,
with responses delivered in bulk at epoch boundaries; tests pin it against the
sequential restatement of the tracker (oracle/pyoracle.Tracker).

State (uint32, modular like the reference's uint32 cast of Counter
differences): per client the global delta/rho counters (start at 1), per
(server, client) X = delta_prev_req + my_delta (and the rho analogue) and a
`known` flag (server in server_map).
"""
import numpy as np


class EpochTrackers:
    def __init__(self, n_servers, n_clients):
        self.S, self.N = n_servers, n_clients
        self.gd = np.ones(n_clients, np.uint32)
        self.gr = np.ones(n_clients, np.uint32)
        self.xd = np.zeros((n_servers, n_clients), np.uint32)
        self.xr = np.zeros((n_servers, n_clients), np.uint32)
        self.known = np.zeros((n_servers, n_clients), bool)
        self.comp_d = np.zeros((n_servers, n_clients), np.uint32)
        self.comp_r = np.zeros((n_servers, n_clients), np.uint32)

    def fill(self, s, reqs):
        """get_req_params(s) for every request of `reqs` (batch order); sets
        reqs['delta'] / reqs['rho'] in place."""
        slots = reqs["slot"].astype(np.int64)
        delta = np.zeros(len(reqs), np.uint32)
        rho = np.zeros(len(reqs), np.uint32)
        _, first = np.unique(slots, return_index=True)
        c = slots[first]
        new = ~self.known[s, c]
        with np.errstate(over="ignore"):
            d = np.where(new, np.uint32(1), self.gd[c] - self.xd[s, c])
            r = np.where(new, np.uint32(1), self.gr[c] - self.xr[s, c])
        delta[first] = d
        rho[first] = r
        self.known[s, c] = True
        self.xd[s, c] = self.gd[c]
        self.xr[s, c] = self.gr[c]
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
        with np.errstate(over="ignore"):
            return (self.comp_d.sum(0, dtype=np.uint64).astype(np.uint32),
                    self.comp_r.sum(0, dtype=np.uint64).astype(np.uint32))

    def deliver(self, sum_d=None, sum_r=None):
        """Epoch boundary: the global counters advance by every server's
        responses (sum_d/sum_r: the all-ranks sums; default: this object's
        servers), each server's X by its own (my_delta / my_rho)."""
        if sum_d is None:
            sum_d, sum_r = self.local_sums()
        with np.errstate(over="ignore"):
            self.gd += sum_d
            self.gr += sum_r
            self.xd += self.comp_d
            self.xr += self.comp_r
        self.comp_d[:] = 0
        self.comp_r[:] = 0
