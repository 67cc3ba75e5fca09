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
__device__ inline void tally_body(const dmc_decision* dec, const dmc_pull_result* res,
                                  uint32_t cap, uint32_t* comp_d, uint32_t* comp_r) {
  uint32_t n = res->n_decisions < cap ? res->n_decisions : cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
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

// The epoch kernels below take 4 consecutive entries per thread, loaded at
// once (one level of loads: uint4 when the host found every array 16-byte
// aligned), over a grid that covers the arrays in one pass -- a grid-stride
// loop of single entries waited for each entry's load in turn (config 5's
// 2M-slot commit: 15 us, its 16M-client advance: 84 us).
__device__ inline uint4 ld4(const uint32_t* p, uint32_t s0, uint32_t n, bool vec) {
  if (vec && s0 + 4 <= n) return ld_as<uint4>(p + s0);
  uint4 v;
  v.x = s0 < n ? p[s0] : 0u;
  v.y = s0 + 1 < n ? p[s0 + 1] : 0u;
  v.z = s0 + 2 < n ? p[s0 + 2] : 0u;
  v.w = s0 + 3 < n ? p[s0 + 3] : 0u;
  return v;
}
__device__ inline uint32_t u4at(const uint4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
// X += (d, r) and (d, r) cleared, only at the entries with a count: the
// arrays are ~20 % dense per epoch at config 5, so writing whole groups of 4
// moved more bytes than the scattered entries (k_track_advance 102 vs 84 us)
__device__ inline void commit4(uint32_t s0, uint32_t n, const uint4& d, const uint4& r,
                               const uint4& a, const uint4& b, uint32_t* xd, uint32_t* xr,
                               uint32_t* cd, uint32_t* cr) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t dj = u4at(d, j), rj = u4at(r, j);
    if (s0 + j < n && (dj | rj)) {
      xd[s0 + j] = u4at(a, j) + dj;
      xr[s0 + j] = u4at(b, j) + rj;
      cd[s0 + j] = 0;
      cr[s0 + j] = 0;
    }
  }
}
// the per-client sums of 4 slots' responses (atomics: the servers of a rank
// collect concurrently on their own streams)
__device__ inline void sums4(uint32_t s0, uint32_t nslots, const uint32_t* client_of_slot,
                             const uint4& cd, const uint4& cr, bool vec, uint32_t* sum_d,
                             uint32_t* sum_r) {
  const uint4 cm = client_of_slot ? ld4(client_of_slot, s0, nslots, vec)
                                  : make_uint4(s0, s0 + 1, s0 + 2, s0 + 3);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t d = u4at(cd, j), r = u4at(cr, j), c = u4at(cm, j);
    if (d) atomicAdd(&sum_d[c], d);
    if (r) atomicAdd(&sum_r[c], r);
  }
}

// epoch end, per server: my_delta / my_rho of its responses (X += own) and
// the server's contribution to the per-client sums
// (a group of 4 entries with every count 0 is skipped; adding and clearing
// a zero entry is the identity)
__global__ void k_track_collect(uint32_t nslots, const uint32_t* client_of_slot,
                                uint32_t* xd, uint32_t* xr, uint32_t* comp_d,
                                uint32_t* comp_r, uint32_t* sum_d, uint32_t* sum_r, bool vec) {
  const uint32_t s0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (s0 >= nslots) return;
  const uint4 cd = ld4(comp_d, s0, nslots, vec), cr = ld4(comp_r, s0, nslots, vec);
  if (!(cd.x | cd.y | cd.z | cd.w | cr.x | cr.y | cr.z | cr.w)) return;
  const uint4 a = ld4(xd, s0, nslots, vec), b = ld4(xr, s0, nslots, vec);
  commit4(s0, nslots, cd, cr, a, b, xd, xr, comp_d, comp_r);
  sums4(s0, nslots, client_of_slot, cd, cr, vec, sum_d, sum_r);
}

// Overlapped (lagged) delivery, split in two: at an epoch's end only the
// per-client sums of its responses are formed (the all-reduce of them runs
// during the next epoch); at the next epoch's end its own-response part
// commits (X += comp, comp cleared) together with the all-reduced sums
// (k_track_advance).
__global__ void k_track_sums(uint32_t nslots, const uint32_t* client_of_slot,
                             const uint32_t* comp_d, const uint32_t* comp_r,
                             uint32_t* sum_d, uint32_t* sum_r, bool vec) {
  const uint32_t s0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (s0 >= nslots) return;
  const uint4 cd = ld4(comp_d, s0, nslots, vec), cr = ld4(comp_r, s0, nslots, vec);
  if (!(cd.x | cd.y | cd.z | cd.w | cr.x | cr.y | cr.z | cr.w)) return;
  sums4(s0, nslots, client_of_slot, cd, cr, vec, sum_d, sum_r);
}
__global__ void k_track_commit(uint32_t nslots, uint32_t* xd, uint32_t* xr, uint32_t* comp_d,
                               uint32_t* comp_r, bool vec) {
  const uint32_t s0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (s0 >= nslots) return;
  const uint4 cd = ld4(comp_d, s0, nslots, vec), cr = ld4(comp_r, s0, nslots, vec);
  if (!(cd.x | cd.y | cd.z | cd.w | cr.x | cr.y | cr.z | cr.w)) return;
  const uint4 a = ld4(xd, s0, nslots, vec), b = ld4(xr, s0, nslots, vec);
  commit4(s0, nslots, cd, cr, a, b, xd, xr, comp_d, comp_r);
}

// after the all-reduce of the sums: the global counters advance (D += all
// servers' responses to the client), sums cleared for the next epoch
__global__ void k_track_advance(uint32_t nclients, uint32_t* gd, uint32_t* gr,
                                uint32_t* sum_d, uint32_t* sum_r, bool vec) {
  const uint32_t c0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (c0 >= nclients) return;
  const uint4 sd = ld4(sum_d, c0, nclients, vec), sr = ld4(sum_r, c0, nclients, vec);
  if (!(sd.x | sd.y | sd.z | sd.w | sr.x | sr.y | sr.z | sr.w)) return;
  const uint4 a = ld4(gd, c0, nclients, vec), b = ld4(gr, c0, nclients, vec);
  commit4(c0, nclients, sd, sr, a, b, gd, gr, sum_d, sum_r);
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
};
__global__ void k_tally_m(const TallyArgs* a) {
  const TallyArgs& x = a[blockIdx.y];
  if (x.dec) tally_body(x.dec, x.res, x.cap, x.comp_d, x.comp_r);
}

}  // namespace dmc
