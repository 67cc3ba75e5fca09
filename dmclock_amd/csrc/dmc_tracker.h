// SPDX-License-Identifier: LGPL-2.1
//
// dmc_tracker.h -- the client side of multi-server dmClock on the device:
// ServiceTracker<S, OrigTracker> (/root/reference/src/dmclock_client.h:39-84,
// 163-287) for simulated clients whose responses are delivered in bulk at
// epoch boundaries (multi-GPU deployment).
//
// Per (server s, client c) the OrigTracker holds delta_prev_req, rho_prev_req
// and my_delta, my_rho; prepare_req returns delta = the_delta -
// delta_prev_req - my_delta.  Only the sum X = delta_prev_req + my_delta
// matters, so the state per (s, c) is X_delta, X_rho (uint32, modular like
// the reference's uint32 cast of the Counter difference) and a `known` byte
// (s is in the client's server_map).  Per client c: the global
// delta_counter / rho_counter (start at 1, ServiceTracker ctor :186-187).
//
//   get_req_params(s)  (:241-251)  unknown: known = 1, X = counters, (1, 1);
//                                  else (D - X_d, R - X_r), X = counters
//   track_resp(s, ph, cost) (:221-235), delivered per epoch:
//                                  D += cost, X_d(s) += cost (my_delta);
//                                  reservation: R += cost, X_r(s) += cost
// Requests of one client to one server inside a batch are served in batch
// order: the first gets the epoch's delta, later ones 0 (the counters did
// not move in between), exactly as the sequential reference would.
//
// A server's table slot s holds global client client_of_slot[s] (identity
// when the map is null): the per-(server, slot) state is slot-indexed, the
// global counters client-indexed (config 5: 16M clients, 2M per table).
#pragma once

#include "dmc_device.h"

namespace dmc {

// per-slot completion tallies of one server's decisions (track_resp's cost)
// (skip: the decisions a queue group's round already tallied where it wrote
// them, k_rrank_m / k_rapply_m)
__device__ inline void tally_body(const dmc_decision* dec, const dmc_pull_result* res,
                                  uint32_t cap, uint32_t* comp_d, uint32_t* comp_r,
                                  uint32_t skip = 0) {
  uint32_t n = res->n_decisions < cap ? res->n_decisions : cap;
  for (uint32_t i = skip + blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    const dmc_decision& d = dec[i];
    atomicAdd(&comp_d[d.slot], d.cost);
    if (d.phase == DMC_PHASE_RESERVATION) atomicAdd(&comp_r[d.slot], d.cost);
  }
}
__global__ void k_tally(const dmc_decision* dec, const dmc_pull_result* res,
                        uint32_t cap, uint32_t* comp_d, uint32_t* comp_r) {
  tally_body(dec, res, cap, comp_d, comp_r);
}

// first batch position of each (server, client) in the batch
__global__ void k_track_first(const dmc_request* reqs, uint32_t n, uint32_t nslots,
                              uint32_t* first) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = reqs[i].slot;
  if (s < nslots) atomicMin(&first[s], i);
}

// get_req_params for every request of the batch (one server)
__device__ inline void track_params_one(dmc_request* reqs, uint32_t n, uint32_t nslots,
                                        const uint32_t* client_of_slot,
                                        const uint32_t* gd, const uint32_t* gr,
                                        uint32_t* xd, uint32_t* xr, uint8_t* known,
                                        uint32_t* first, uint32_t i) {
  if (i >= n) return;
  uint32_t s = reqs[i].slot;
  if (s >= nslots) return;
  uint32_t delta = 0, rho = 0;  // a later request of the same client: no new responses
  if (first[s] == i) {
    uint32_t c = client_of_slot ? client_of_slot[s] : s;
    uint32_t D = gd[c], R = gr[c];
    if (!known[s]) {
      known[s] = 1;
      delta = 1;
      rho = 1;
    } else {
      delta = D - xd[s];
      rho = R - xr[s];
    }
    xd[s] = D;
    xr[s] = R;
    first[s] = 0xffffffffu;  // ready for the next batch
  }
  reqs[i].delta = delta;
  reqs[i].rho = rho;
}
__global__ void k_track_params(dmc_request* reqs, uint32_t n, uint32_t nslots,
                               const uint32_t* client_of_slot,
                               const uint32_t* gd, const uint32_t* gr,
                               uint32_t* xd, uint32_t* xr, uint8_t* known,
                               uint32_t* first) {
  track_params_one(reqs, n, nslots, client_of_slot, gd, gr, xd, xr, known, first,
                   blockIdx.x * blockDim.x + threadIdx.x);
}

// epoch end, per server: my_delta / my_rho of its responses (X += own) and
// the server's contribution to the per-client sums (atomics: the servers of
// a rank collect concurrently on their own streams)
__global__ void k_track_collect(uint32_t nslots, const uint32_t* client_of_slot,
                                uint32_t* xd, uint32_t* xr, uint32_t* comp_d,
                                uint32_t* comp_r, uint32_t* sum_d, uint32_t* sum_r) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    uint32_t cd = comp_d[s];
    if (!cd) continue;  // comp_r <= comp_d: nothing delivered to this slot
    uint32_t cr = comp_r[s];
    xd[s] += cd;
    xr[s] += cr;
    comp_d[s] = 0;
    comp_r[s] = 0;
    uint32_t c = client_of_slot ? client_of_slot[s] : s;
    atomicAdd(&sum_d[c], cd);
    if (cr) atomicAdd(&sum_r[c], cr);
  }
}

// Overlapped (lagged) delivery, split in two: at an epoch's end only the
// per-client sums of its responses are formed (the all-reduce of them runs
// during the next epoch); at the next epoch's end its own-response part
// commits (X += comp, comp cleared) together with the all-reduced sums
// (k_track_advance).
__global__ void k_track_sums(uint32_t nslots, const uint32_t* client_of_slot,
                             const uint32_t* comp_d, const uint32_t* comp_r,
                             uint32_t* sum_d, uint32_t* sum_r) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    const uint32_t cd = comp_d[s];
    if (!cd) continue;
    const uint32_t cr = comp_r[s];
    const uint32_t c = client_of_slot ? client_of_slot[s] : s;
    atomicAdd(&sum_d[c], cd);
    if (cr) atomicAdd(&sum_r[c], cr);
  }
}
__global__ void k_track_commit(uint32_t nslots, uint32_t* xd, uint32_t* xr, uint32_t* comp_d,
                               uint32_t* comp_r) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    const uint32_t cd = comp_d[s];
    if (!cd) continue;
    xd[s] += cd;
    xr[s] += comp_r[s];
    comp_d[s] = 0;
    comp_r[s] = 0;
  }
}

// after the all-reduce of the sums: the global counters advance (D += all
// servers' responses to the client), sums cleared for the next epoch
__global__ void k_track_advance(uint32_t nclients, uint32_t* gd, uint32_t* gr,
                                uint32_t* sum_d, uint32_t* sum_r) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nclients;
       c += gridDim.x * blockDim.x) {
    gd[c] += sum_d[c];
    gr[c] += sum_r[c];
    sum_d[c] = 0;
    sum_r[c] = 0;
  }
}

// multi-table forms (a queue group's step, dmc_group_step_device): the
// per-server arguments indexed by blockIdx.y, the bodies the same kernels'
struct TrackArgs {
  dmc_request* reqs;
  uint32_t n, nslots;
  const uint32_t *cmap, *gd, *gr;
  uint32_t *xd, *xr;
  uint8_t* known;
  uint32_t* first;
};
__global__ void k_track_first_m(const TrackArgs* a) {
  const TrackArgs& x = a[blockIdx.y];
  if (!x.reqs) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= x.n) return;
  const uint32_t s = x.reqs[i].slot;
  if (s < x.nslots) atomicMin(&x.first[s], i);
}
__global__ void k_track_params_m(const TrackArgs* a) {
  const TrackArgs& x = a[blockIdx.y];
  if (!x.reqs) return;
  track_params_one(x.reqs, x.n, x.nslots, x.cmap, x.gd, x.gr, x.xd, x.xr, x.known, x.first,
                   blockIdx.x * blockDim.x + threadIdx.x);
}
struct TallyArgs {
  const dmc_decision* dec;
  const dmc_pull_result* res;
  uint32_t cap;
  uint32_t *comp_d, *comp_r;
  uint32_t skip;  // decisions tallied by the round's own kernels
};
__global__ void k_tally_m(const TallyArgs* a) {
  const TallyArgs& x = a[blockIdx.y];
  if (x.dec) tally_body(x.dec, x.res, x.cap, x.comp_d, x.comp_r, x.skip);
}

}  // namespace dmc
