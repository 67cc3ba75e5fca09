/* SPDX-License-Identifier: LGPL-2.1
 *
 * dmclock_gpu.h -- C-ABI of the MI355X-native dmClock server queue.
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json's
 * north_star: the server-side dmClock priority queue of the reference
 * (crimson::dmclock::PullPriorityQueue / PushPriorityQueue,
 * /root/reference/src/dmclock_server.h).  The reference's boundary is a C++
 * template API, not an FFI; every entry point below names the reference member
 * it replaces (file:line).  The C++ facade in
 * dmclock_amd/include/dmclock_server.h re-exports the reference's template
 * names on top of these functions, so existing callers compile unchanged.
 *
 * Conventions
 *  - plain pointers and sizes only; no torch / HIP types in signatures.
 *  - a queue lives on one HIP device; every call on one queue handle must be
 *    serialised by the caller (the facade holds a mutex, mirroring the
 *    reference's data_mtx, dmclock_server.h:762).
 *  - clients are dense "slots" [0, max_clients); the facade maps the
 *    reference's client id type C to slots.
 *  - every function returns a status code (DMC_OK or a negative DMC_E*);
 *    nothing aborts.  Where the reference asserts, we return a code.
 *  - *_device variants take device pointers and run asynchronously on the
 *    queue's HIP stream (dmc_queue_stream); the others take host pointers and
 *    return when results are in host memory.
 */
#ifndef DMCLOCK_GPU_H
#define DMCLOCK_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ status codes */
#define DMC_OK 0
#define DMC_EAGAIN 11          /* AtLimit::Reject rejected the request (errno EAGAIN, dmclock_server.h:989-993) */
#define DMC_EINVAL (-1)        /* bad argument (unknown slot, bad params, ...) */
#define DMC_ENOMEM (-2)        /* device allocation failed */
#define DMC_EDEVICE (-3)       /* HIP runtime error */
#define DMC_EBADTAG (-1001)    /* cost==0 or r and w both 0 (reference asserts, dmclock_server.h:158,182) */
#define DMC_EBADPARAMS (-1002) /* rho > delta (reference asserts, dmclock_recs.h:51) */
#define DMC_EQUEUEFULL (-1004) /* the client's request ring is full (documented deviation: the
                                  reference's per-client std::deque is unbounded, :360) */
#define DMC_ENOTREG (-1005)    /* slot not registered */
#define DMC_ENOTRUN (-1006)    /* DMC_OPT_PIPELINE: the previous call on the queue failed and this
                                  call was not executed: none of its adds or pulls took effect and
                                  its outputs were not written; the previous call's own error is
                                  dmc_queue_pipelined_error()'s */

/* ------------------------------------------------------------ ABI version
 * Bumped at every incompatible change of this header (option ids, struct
 * layouts, status codes).  A caller compiled against one header checks
 * dmc_abi_version() == DMC_ABI_VERSION at start-up; dmc_counters is also
 * readable size-checked (dmc_queue_counters_sized).
 *   5: DMC_OPT_FAULT moved from 9 to 13 (9, round 3's DMC_OPT_PREDICT, is
 *      retired and returns DMC_EINVAL); DMC_ENOTRUN; dmc_counters gained
 *      act_batches / act_seq_batches (round 4) and renamed pred_* to
 *      bad_rounds / serve_yields. */
/*   6: dmc_queue_pipelined_error (the error a DMC_ENOTRUN stands for);
 *      dmc_group_profile_enable / dmc_group_profile_read.
 *   7: dmc_group_tracker_collect_sums / _join / dmc_group_side_stream. */
#define DMC_ABI_VERSION 7
int dmc_abi_version(void);

/* ------------------------------------------------------------ enums */
/* AtLimit, dmclock_server.h:74-84 */
#define DMC_AT_LIMIT_WAIT 0
#define DMC_AT_LIMIT_ALLOW 1
#define DMC_AT_LIMIT_REJECT 2

/* NextReqType, dmclock_server.h:506 */
#define DMC_NEXT_RETURNING 0
#define DMC_NEXT_FUTURE 1
#define DMC_NEXT_NONE 2

/* PhaseType, dmclock_recs.h:33 */
#define DMC_PHASE_RESERVATION 0
#define DMC_PHASE_PRIORITY 1

/* ------------------------------------------------------------ records */

/* Queue construction parameters.  Replaces the PullPriorityQueue /
 * PushPriorityQueue constructors (dmclock_server.h:1314-1341, 1545-1580) and
 * their template parameters IsDelayed and U1 (:1279, :1505).  The heap
 * branching factor B has no meaning on the device (there are no heaps). */
typedef struct dmc_queue_params {
  uint32_t max_clients;      /* slot capacity of the client table            */
  uint32_t ring_capacity;    /* per-client request ring, power of two        */
  uint32_t max_batch;        /* max requests per add batch and decisions per pull batch */
  int32_t delayed;           /* IsDelayed (DelayedTagCalc), :277-280          */
  int32_t dynamic_info;      /* U1: every tag calculation reads the bound
                                ClientInfo (dmc_client_bind_info_batch or the
                                dmc_info_fn) and caches it, :870-875          */
  int32_t at_limit;          /* DMC_AT_LIMIT_*                                */
  double reject_threshold;   /* RejectThreshold (AtLimitParam variant), :86-93 */
  double anticipation_timeout; /* :151-161                                    */
  int32_t device;            /* HIP device ordinal                            */
  int32_t reserved;
} dmc_queue_params;

/* One request of an add batch.  Replaces the arguments of
 * add_request(RequestRef&&, const C&, const ReqParams&, Time, Cost)
 * (dmclock_server.h:1398-1417; ReqParams dmclock_recs.h:40-72).  `handle`
 * stands for the RequestRef: the device never sees R, only this handle, which
 * comes back in the decision that dispatches the request. */
typedef struct dmc_request {
  uint32_t slot;   /* client slot                                           */
  uint32_t cost;   /* Cost, dmclock_recs.h:31                               */
  double time;     /* arrival Time, dmclock_util.h:33                       */
  uint32_t delta;  /* ReqParams::delta                                      */
  uint32_t rho;    /* ReqParams::rho                                        */
  uint64_t handle; /* opaque request handle                                 */
} dmc_request;     /* 32 bytes */

/* One dispatch decision of a pull batch.  Replaces PullReq::Retn
 * (dmclock_server.h:1287-1292): client, request, phase, cost; plus the tag
 * the request was dispatched with (before reduce_reservation_tags) so that
 * parity can be checked at the tag level. */
typedef struct dmc_decision {
  uint64_t handle;     /* the request's handle                                */
  double tag_r;        /* RequestTag::reservation at dispatch                 */
  double tag_p;        /* RequestTag::proportion                              */
  double tag_l;        /* RequestTag::limit                                   */
  uint32_t slot;       /* client slot                                         */
  uint32_t cost;       /* Cost                                                */
  uint32_t phase;      /* DMC_PHASE_*                                         */
  uint32_t flags;      /* bit0: the key tied with another client's (GPU: lowest slot won) */
} dmc_decision;        /* 48 bytes */

/* Outcome of a pull batch: how many decisions were returned and, when the
 * batch stopped early, what the stopping pull_request(now) returned
 * (PullReq::type and its Time, dmclock_server.h:1294-1305). */
typedef struct dmc_pull_result {
  uint32_t n_decisions; /* decisions written                                 */
  uint32_t next_type;   /* DMC_NEXT_RETURNING if k decisions were made, else
                           DMC_NEXT_FUTURE / DMC_NEXT_NONE of the stopping pull */
  double when;          /* future time when next_type == DMC_NEXT_FUTURE     */
  uint32_t n_reservation; /* decisions in the reservation phase              */
  uint32_t n_priority;    /* decisions in the priority phase                 */
} dmc_pull_result;

/* Per-client state snapshot for tests and debugging (ClientRec, :355-393). */
typedef struct dmc_client_state {
  double prev_r, prev_p, prev_l, prev_arrival; /* prev_tag                   */
  double prop_delta;
  double front_r, front_p, front_l, front_arrival; /* next_request().tag     */
  double r_inv, w_inv, l_inv;                  /* ClientInfo inverses        */
  uint64_t last_tick;
  uint32_t count;       /* queued requests                                   */
  uint32_t cur_delta, cur_rho;
  uint8_t idle, front_ready, registered, pad;
} dmc_client_state;

/* Queue counters, dmclock_server.h:806-812 */
typedef struct dmc_stats {
  uint64_t tick;
  uint64_t reserv_sched_count;
  uint64_t prop_sched_count;
  uint64_t limit_break_sched_count;
  uint64_t clients;   /* registered slots (client_count, :551-554)           */
  uint64_t requests;  /* queued requests (request_count, :557-564)           */
} dmc_stats;

typedef struct dmc_queue dmc_queue;

/* ------------------------------------------------------------ lifecycle */

/* Replaces PullPriorityQueue(ClientInfoFunc, AtLimitParam, double)
 * (dmclock_server.h:1314-1341).  Allocates the HBM client table and rings. */
int dmc_queue_create(const dmc_queue_params* params, dmc_queue** out);
int dmc_queue_destroy(dmc_queue* q);
/* The HIP stream (hipStream_t) every *_device call runs on (the serve
 * kernel, DMC_OPT_SERVE, is stopped first: work queued on the stream does
 * not wait behind it).  dmc_queue_sync waits for the stream. */
void* dmc_queue_stream(dmc_queue* q);
int dmc_queue_sync(dmc_queue* q);
const char* dmc_strerror(int code);

/* ------------------------------------------------------------ clients */

/* First sight of a client: do_add_request's client_map.emplace +
 * client_info_f + ClientRec(idle=true) (dmclock_server.h:920-932, 381-393).
 * active != 0 is the bulk-registration deviation used for 1M-client
 * populations (idle=false, prop_delta=0), applied identically to the oracle. */
int dmc_client_register(dmc_queue* q, uint32_t slot, double reservation,
                        double weight, double limit, int active);
int dmc_client_register_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                              const double* reservation, const double* weight,
                              const double* limit, int active);
/* update_client_info(s) after client_info_f returns new values
 * (dmclock_server.h:633-648; ClientInfo::update :111-118): the values become
 * both what client_info_f returns (the bound info) and the cached
 * client.info. */
int dmc_client_update_info(dmc_queue* q, uint32_t slot, double reservation,
                           double weight, double limit);

/* U1, get_cli_info (dmclock_server.h:870-875).  The engine models
 * client_info_f as a per-client "bound" ClientInfo: what client_info_f(c)
 * would return now.  With dynamic_info, every tag calculation (initial_tag
 * :878-907, update_next_tag :1021-1036) reads the bound info and stores it as
 * the client's cached info, which the reservation reductions use
 * (:1077-1111), exactly as the reference's `client.info = client_info_f(...)`.
 * Without dynamic_info the bound info is recorded and unused.
 *
 * dmc_client_bind_info_batch publishes new bound values (dirty pushes: only
 * the clients whose ClientInfo changed need one).  Unchanged values cost no
 * device work. */
int dmc_client_bind_info_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                               const double* reservation, const double* weight,
                               const double* limit);
/* A host client_info_f for callers that cannot push changes: with
 * dynamic_info the engine calls fn(ctx, slot, ...) on the calling thread
 * right before each tag calculation a host-API call may perform -- for every
 * request of dmc_add_batch, and in delayed mode for the client each
 * pull_request of dmc_pull_batch dispatches, between its selection and its
 * pop (such a dmc_pull_batch runs one pull at a time).  fn returns 0, or
 * non-zero to fail the call with DMC_EINVAL.  The *_device entry points never
 * call fn: their callers bind first.  fn == NULL removes it. */
typedef int (*dmc_info_fn)(void* ctx, uint32_t slot, double* reservation,
                           double* weight, double* limit);
int dmc_queue_set_info_fn(dmc_queue* q, dmc_info_fn fn, void* ctx);
/* do_clean's idle marking and erase, as explicit calls (dmclock_server.h
 * :1206-1255): mark_idle sets idle=true; erase drops the client and its
 * queued requests (their handles are written to handles_out, capacity cap). */
int dmc_client_mark_idle(dmc_queue* q, uint32_t slot);
/* The same for n registered clients (do_clean's idle pass over a client
 * set, :1230-1250); slots in host memory. */
int dmc_client_mark_idle_batch(dmc_queue* q, uint32_t n, const uint32_t* slots);
/* The same with the slot list in device memory, ordered on the queue's stream
 * (no host round trip; unregistered slots are ignored).  The engine's host
 * view of which clients are idle is re-read from the device when a later
 * host-API call needs it; device-API adds detect activations on the device. */
int dmc_client_mark_idle_batch_device(dmc_queue* q, uint32_t n, const uint32_t* d_slots);
int dmc_client_erase(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                     uint32_t cap, uint32_t* n_out);
int dmc_client_get_state(dmc_queue* q, uint32_t slot, dmc_client_state* out);
/* last_tick of every slot in [0, n) (for the facade's do_clean). */
int dmc_client_last_ticks(dmc_queue* q, uint32_t n, uint64_t* out);

/* ------------------------------------------------------------ hot path */

/* A batch of add_request_time calls in order (dmclock_server.h:1368-1417,
 * do_add_request :913-1018).  rc_out[i] gets 0, DMC_EAGAIN, or an error. */
int dmc_add_batch(dmc_queue* q, uint32_t n, const dmc_request* reqs,
                  int32_t* rc_out);
int dmc_add_batch_device(dmc_queue* q, uint32_t n, const dmc_request* d_reqs,
                         int32_t* d_rc_out);

/* Up to k successive pull_request(now) calls (dmclock_server.h:1425-1489),
 * stopping after the first that does not return a request. */
int dmc_pull_batch(dmc_queue* q, double now, uint32_t k, dmc_decision* out,
                   dmc_pull_result* result);
int dmc_pull_batch_device(dmc_queue* q, double now, uint32_t k,
                          dmc_decision* d_out, dmc_pull_result* d_result);
/* dmc_add_batch_device then dmc_pull_batch_device(now, k): the same results
 * as the two calls (the reference's add_request_time x n then
 * pull_request(now) x k, :1344-1489).  When no idle client must be
 * activated and the pull is one batched round, the add kernels and that round
 * run as one graph launch. */
int dmc_add_pull_batch_device(dmc_queue* q, uint32_t n, const dmc_request* d_reqs,
                              int32_t* d_rc, double now, uint32_t k,
                              dmc_decision* d_out, dmc_pull_result* d_result);

/* ------------------------------------------------------------ queue groups
 * S server queues of one device driven as one (BASELINE config 5's per-GPU
 * shape: dmClock servers are independent queues, sim/src/simulate.h:118-136,
 * one per server, sim/src/sim_server.h:84,123-130).  A group step does, for
 * every member s, exactly what dmc_tracker_fill (when trk is given) +
 * dmc_add_pull_batch_device + dmc_tracker_tally do on it alone -- the same
 * results, bit for bit -- with one launch per kernel over all members (one
 * graph per step).  Members must share device, max_clients and
 * ring_capacity; while in a group a member runs on the group's stream (its
 * other calls stay valid and are ordered with the group's steps).  A member
 * destroyed before its group leaves it. */
typedef struct dmc_group dmc_group;
typedef struct dmc_group_tracker {  /* one server's device tracker state (see dmc_tracker_*) */
  const uint32_t* client_of_slot;   /* NULL: identity */
  const uint32_t* gdelta;
  const uint32_t* grho;
  uint32_t* xd;
  uint32_t* xr;
  uint8_t* known;
  uint32_t* first;
  uint32_t* comp_delta;             /* tallied after the step (needs d_result) */
  uint32_t* comp_rho;
} dmc_group_tracker;
int dmc_group_create(dmc_queue* const* queues, uint32_t n, dmc_group** out);
int dmc_group_destroy(dmc_group* g);
void* dmc_group_stream(dmc_group* g);
/* Overlapped delivery for a queue group (no reference counterpart; the
 * values of dmc_tracker_collect_sums on every member): the members'
 * per-client sums, sum_*[client_of_slot[s][i]] += comp_*[s][i], run on a
 * stream of their own behind the group's work so far, beside the group's
 * next steps (which tally into the other half of the comp arrays).
 * dmc_group_tracker_join orders the group's stream behind them: call it
 * before anything on the group's stream reads the sums or clears those comp
 * arrays (the next epoch's commit and advance).  client_of_slot: NULL, or one
 * map per member (entries NULL: identity).  dmc_group_side_stream: that
 * stream (NULL before the first collection), for a collective on the sums. */
int dmc_group_tracker_collect_sums(dmc_group* g, uint32_t n_slots,
                                   const uint32_t* const* d_client_of_slot,
                                   const uint32_t* const* d_comp_delta,
                                   const uint32_t* const* d_comp_rho, uint32_t* d_sum_delta,
                                   uint32_t* d_sum_rho);
int dmc_group_tracker_join(dmc_group* g);
void* dmc_group_side_stream(dmc_group* g);
/* Per member s: requests d_reqs[s][0..n) (delta/rho filled first when trk),
 * statuses d_rc[s], pull time now[s], k pulls into d_out[s], result record
 * d_result[s]; trk: NULL or one entry per member. */
int dmc_group_step_device(dmc_group* g, uint32_t n, dmc_request* const* d_reqs,
                          int32_t* const* d_rc, const double* now, uint32_t k,
                          dmc_decision* const* d_out, dmc_pull_result* const* d_result,
                          const dmc_group_tracker* trk);
/* Group stage timers (an extension, like dmc_profile_*): while on, fused
 * group steps launch their multi-table kernels eagerly (no graph), each
 * timed by its own dispatch; dmc_group_profile_read returns, per
 * DMC_PROF_* stage (ADD_LINK, ADD_CHAIN, SCAN, SELECT = hist + pick, EMIT,
 * RANK, APPLY), the launches and their total milliseconds since the last
 * enable (which also resets them). */
int dmc_group_profile_enable(dmc_group* g, int on);
int dmc_group_profile_read(dmc_group* g, uint32_t stage, uint64_t* count, double* total_ms);

/* ------------------------------------------------------------ maintenance */

/* remove_by_client (dmclock_server.h:594-625): queued handles in FIFO order
 * (reverse != 0: LIFO) are written to handles_out; the queue is cleared. */
int dmc_remove_by_client(dmc_queue* q, uint32_t slot, int reverse,
                         uint64_t* handles_out, uint32_t cap, uint32_t* n_out);
/* Queued handles of one client, FIFO order (for remove_by_req_filter, :567-585). */
int dmc_client_requests(dmc_queue* q, uint32_t slot, uint64_t* handles_out,
                        uint32_t cap, uint32_t* n_out);
/* Keep only the requests whose keep[i] != 0 (i in FIFO order, n == count):
 * ClientRec::remove_by_req_filter's erase (:440-480). */
int dmc_client_filter(dmc_queue* q, uint32_t slot, uint32_t n,
                      const uint8_t* keep);
/* Whole-queue maintenance in a fixed number of device passes (no per-client
 * round trips).  remove_by_req_filter (dmclock_server.h:567-585) is
 *   dmc_queue_requests -> host filter over the handles -> dmc_queue_filter.
 * dmc_queue_requests: counts_out[s] (max_clients entries, may be NULL) = the
 * queued requests of slot s; handles_out = every queued handle, slots in
 * ascending order, each client's FIFO order; *n_out = their total.  With
 * handles_out NULL or cap < total only the counts and *n_out are written
 * (size the buffer and call again). */
int dmc_queue_requests(dmc_queue* q, uint32_t* counts_out, uint64_t* handles_out,
                       uint64_t cap, uint64_t* n_out);
/* ClientRec::remove_by_req_filter's erase for every client at once
 * (:440-480): keep[i] != 0 keeps the i-th handle of the last
 * dmc_queue_requests readback (n = its total); DMC_EINVAL if the queue
 * changed since.  *any_removed (may be NULL): whether a request was removed. */
int dmc_queue_filter(dmc_queue* q, const uint8_t* keep, uint64_t n, int* any_removed);
/* do_clean's erase (:1244-1255) of n distinct registered clients in one pass:
 * counts_out[i] (may be NULL) = slot i's queued requests, handles_out = their
 * handles (list order, FIFO per client; cap >= total or DMC_EINVAL), *n_out =
 * the total. */
int dmc_client_erase_batch(dmc_queue* q, uint32_t n, const uint32_t* slots,
                           uint32_t* counts_out, uint64_t* handles_out, uint64_t cap,
                           uint64_t* n_out);
int dmc_stats_get(dmc_queue* q, dmc_stats* out);

/* ------------------------------------------------------------ client side
 * Multi-server epochs: the reference's client-side
 * ServiceTracker<S, OrigTracker> (dmclock_client.h:39-84, 163-287) for
 * simulated clients, on the device, with responses delivered at epoch
 * boundaries.  All arrays are device memory indexed by client slot, owned by
 * the caller; they run on the queue's stream.  The caller sums the per-server
 * tallies over all servers of all ranks (an all-reduce) between tally and
 * deliver. */
/* track_resp's counting: comp_delta[slot] += cost for each of the
 * d_result->n_decisions (<= cap) decisions, comp_rho[slot] += cost for the
 * reservation-phase ones. */
int dmc_tracker_tally(dmc_queue* q, const dmc_decision* d_dec,
                      const dmc_pull_result* d_result, uint32_t cap,
                      uint32_t* d_comp_delta, uint32_t* d_comp_rho);
/* get_req_params (dmclock_client.h:241-251) for every request of a batch to
 * this queue's server, in batch order: writes d_reqs[i].delta / .rho.
 * client_of_slot: the global client of each table slot (NULL: identity);
 * xd/xr/known: this server's per-slot tracker state; gdelta/grho: the
 * clients' global counters (start at 1); first: per-slot scratch, all
 * 0xffffffff initially (left so). */
int dmc_tracker_fill(dmc_queue* q, dmc_request* d_reqs, uint32_t n,
                     const uint32_t* d_client_of_slot, const uint32_t* d_gdelta,
                     const uint32_t* d_grho, uint32_t* d_xd, uint32_t* d_xr,
                     uint8_t* d_known, uint32_t* d_first);
/* Overlapped delivery, the two halves of
 * dmc_tracker_collect: at an epoch's end sum_*[client_of_slot[s]] += comp_*
 * only (the all-reduce of the sums then runs during the next epoch); at the
 * next epoch's end dmc_tracker_commit moves that epoch's own responses into
 * the server's tracker state (xd += comp_delta, xr += comp_rho, comp_* = 0)
 * beside dmc_tracker_advance of the all-reduced sums. */
int dmc_tracker_collect_sums(dmc_queue* q, uint32_t n_slots, const uint32_t* d_client_of_slot,
                             const uint32_t* d_comp_delta, const uint32_t* d_comp_rho,
                             uint32_t* d_sum_delta, uint32_t* d_sum_rho);
int dmc_tracker_commit(dmc_queue* q, uint32_t n_slots, uint32_t* d_xd, uint32_t* d_xr,
                       uint32_t* d_comp_delta, uint32_t* d_comp_rho);
/* Epoch end for one server (track_resp, :221-235): xd += comp_delta, xr +=
 * comp_rho (my_delta / my_rho), sum_*[client_of_slot[s]] += comp_* (atomic;
 * the servers of a rank may collect concurrently), comp_* = 0. */
int dmc_tracker_collect(dmc_queue* q, uint32_t n_slots,
                        const uint32_t* d_client_of_slot, uint32_t* d_xd,
                        uint32_t* d_xr, uint32_t* d_comp_delta, uint32_t* d_comp_rho,
                        uint32_t* d_sum_delta, uint32_t* d_sum_rho);
/* After the sums are all-reduced over the ranks: gdelta += sum_delta, grho
 * += sum_rho (the_delta / the_rho of track_resp), sums cleared. */
int dmc_tracker_advance(dmc_queue* q, uint32_t n_clients, uint32_t* d_gdelta,
                        uint32_t* d_grho, uint32_t* d_sum_delta, uint32_t* d_sum_rho);

/* ------------------------------------------------------------ tuning
 * Engine options (no reference counterpart): pulls with k <= SMALL_K run one
 * general do_next_request at a time (default 8); FORCE_RADIX ranks batched
 * pulls with a radix sort instead of the bin-rank pass (both exact). */
#define DMC_OPT_SMALL_K 1
#define DMC_OPT_FORCE_RADIX 2
#define DMC_OPT_GRAPHS 3       /* 0: launch every kernel eagerly (default 1: replay captured hipGraphs) */
#define DMC_OPT_ACT_SPLIT 4    /* 1: resolve each activation's idle reset by splitting the batch on the
                                  host (default 0: all of a batch's activations on the device) */
#define DMC_OPT_SAMPLE 5       /* pull-round thresholds for tables of >= 65,536 slots: 1 (default) from
                                  a 1/8 sample of the first keys, validated exactly (a failing round is
                                  re-run exactly); 0 always exact; 2 a test mode with no sampling margin */
#define DMC_OPT_SINGLE_OP 6    /* 1 (default): host-API adds of one request of a non-idle client and
                                  pulls with k <= SMALL_K run the single-op path (one kernel per add,
                                  two per pull, results in host-mapped memory, one round trip);
                                  0: the general launch sequence */
#define DMC_OPT_FAULT 13        /* test hook: 1 = the next rounds' pick leaves phase 1's selection
                                  unset (each such round must fail its outcome check: DMC_EDEVICE,
                                  never a short dispatch); 0 (default): off.  (Option 9, the
                                  retired DMC_OPT_PREDICT, returns DMC_EINVAL.) */
#define DMC_OPT_SERVE 10        /* 1: single-op adds and pulls (as DMC_OPT_SINGLE_OP) are served by a
                                  persistent one-workgroup kernel polling host-mapped commands: no
                                  launch per call; the pull reduces per-group summaries of the
                                  fronts instead of scanning every client.  Any other call stops
                                  it; it exits by itself after 2 ms without a command.
                                  0 (default): the single-op kernels */
#define DMC_OPT_BREAK_ROUNDS 8  /* 1 (default): AtLimit::Allow's limit breaks (dmclock_server.h:1157-1165)
                                  run as batched rounds after the eligible work ran out (immediate
                                  mode); 0: one general pull_request step each */
#define DMC_OPT_HEAP_ORDER 11   /* K >= 2: tie-exact dispatch -- the reference's three indirect
                                  K-ary heaps (IndIntruHeap, dmclock_server.h:768-797) kept on the
                                  device and driven in the reference's order; among equal keys the
                                  reference's heap top wins (default: lowest slot, flagged).  Every
                                  add and pull then runs in call order on one workgroup (exact, not
                                  fast).  Set before the first client is registered; clients may
                                  be registered once; queue groups do not take such queues.
                                  0: off (default) */
#define DMC_OPT_PIPELINE 12     /* 1: dmc_add_pull_batch_device calls are pipelined -- a call queues its
                                  graph behind the previous call's and returns; the previous call is
                                  finished (its round's outcome read, re-runs if it needed any) after
                                  that launch, so the device runs the calls back to back.  A call's
                                  results are complete once the next call on the queue, or any other
                                  call such as dmc_queue_sync, has returned; an error of a call is
                                  reported by that next call, which then was not executed itself
                                  (DMC_ENOTRUN when the error is the previous call's alone; the
                                  queue stays usable).  A round that needs the host shuts a
                                  device-side gate and the next call's queued graph does nothing (it
                                  is launched again).  0 (default): each call waits for its round */
#define DMC_OPT_FAIL_ALLOC 7    /* test hook: the queue's next `value` device buffer allocations
                                  (growth of its batch, decision, radix and activation buffers)
                                  fail; the call returns DMC_ENOMEM, the queue stays usable */
int dmc_queue_set_option(dmc_queue* q, int option, int64_t value);

/* DMC_OPT_PIPELINE: the status of the last pipelined call that failed when a
 * later call finished it -- the error that later call reported as
 * DMC_ENOTRUN (or returned itself) -- 0 if none; clear != 0 resets it.  A
 * failure whose call's successor had already run (the device failed: the
 * queue's state is unknown) also marks the queue failed: every later call
 * returns DMC_EDEVICE. */
int dmc_queue_pipelined_error(dmc_queue* q, int clear);

/* Engine path counters since creation (or the last reset): which ranking
 * path the batched pull rounds took and how often a round was re-run.  No
 * reference counterpart; for tests and the benchmark's records. */
typedef struct dmc_counters {
  uint64_t rounds;          /* batched pull rounds run (re-runs included)          */
  uint64_t radix_rounds;    /* of which ranked by the radix path                    */
  uint64_t bin_overflows;   /* rounds aborted by a rank-bin overflow (re-run with fewer pulls,
                               bin_splits, or on the radix path)                    */
  uint64_t dense_overflows; /* radix rounds re-run with a larger dense buffer       */
  uint64_t single_steps;    /* general single pull_request steps                    */
  uint64_t candidates;      /* candidate clients visited by completed rounds         */
  uint64_t entries;         /* rank records (bin path) / dense entries (radix path) they emitted */
  uint64_t decisions;       /* decisions of completed rounds                         */
  uint64_t graph_replays;   /* captured hipGraphs replayed (add segments, rounds, fused calls) */
  uint64_t fused_calls;     /* dmc_add_pull_batch_device calls run as one add + round launch */
  uint64_t sample_retries;  /* rounds re-run because a sampled threshold admitted too few keys */
  uint32_t max_bin;         /* largest rank bin of a bin-ranked round (records)     */
  uint32_t reserved;
  uint64_t bin_splits;      /* of the overflowed rounds: re-run as a smaller round   */
  uint64_t brk_rounds;      /* limit-break rounds started (AtLimit::Allow)           */
  uint64_t brk_fallbacks;   /* limit-break rounds whose state was not break-ready    */
  uint64_t bad_rounds;      /* rounds that failed their outcome check (DMC_EDEVICE returned) */
  uint64_t serve_yields;    /* times this queue's idle k_serve was stopped so that another
                               queue's call need not wait behind it (DMC_OPT_SERVE) */
  uint64_t serve_calls;     /* single adds / pulls answered by the serve kernel (DMC_OPT_SERVE) */
  uint64_t serve_launches;  /* serve kernel launches (first call, after another call or idling) */
  uint64_t act_batches;     /* add batches whose activations were resolved on the device */
  uint64_t act_seq_batches; /* of those, resolved in order by one wave (k_act_hard: an
                               activated client left empty -- AtLimit::Reject rejected its
                               request -- whose basis later requests of the batch moved) */
} dmc_counters;
int dmc_queue_counters(dmc_queue* q, dmc_counters* out, int reset);
/* The same, copying min(size, sizeof(dmc_counters)) bytes: a caller built
 * against an older, smaller dmc_counters passes its own sizeof. */
int dmc_queue_counters_sized(dmc_queue* q, void* out, uint64_t size, int reset);

/* ------------------------------------------------------------ profiling
 * Stage timers: HIP events recorded on the queue's stream around each stage
 * of the add and pull pipelines (an extension of this library; the reference
 * has compile-time PROFILE timers around add/pull instead,
 * dmclock_server.h:1309-1312, support/src/profile.h). */
#define DMC_PROF_ADD_LINK 0
#define DMC_PROF_ADD_CHAIN 1
#define DMC_PROF_ACTIVATE 2
#define DMC_PROF_SCAN 3     /* pull round: k_rscan */
#define DMC_PROF_SELECT 4   /* k_rhist + k_rpick */
#define DMC_PROF_EMIT 5     /* k_remit */
#define DMC_PROF_SORT 6     /* radix path: key32 + sort + fix-up */
#define DMC_PROF_RANK 7     /* k_rrank (radix path: sizes + scans + decide) */
#define DMC_PROF_APPLY 8    /* k_rapply */
#define DMC_PROF_STEP 9     /* one general pull_request */
#define DMC_PROF_FUTURE 10  /* a round's terminal pull */
#define DMC_PROF_CAND 11    /* k_rcand */
#define DMC_PROF_CHAIN_SCAN 12 /* k_chain_scan: a fused call's add chain beside the round's scan */
#define DMC_PROF_APPLY_LINK 13 /* k_apply_link: a pipelined call's filing beside the previous
                                  call's deferred apply */
#define DMC_PROF_NSTAGES 14

int dmc_profile_enable(dmc_queue* q, int on);
int dmc_profile_reset(dmc_queue* q);
int dmc_profile_read(dmc_queue* q, uint32_t stage, uint64_t* count,
                     double* total_ms);
const char* dmc_profile_stage_name(uint32_t stage);

#ifdef __cplusplus
}
#endif

#endif /* DMCLOCK_GPU_H */
