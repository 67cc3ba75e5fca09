// The serve path: one-at-a-time add_request / pull_request (the drop-in
// caller's calling convention, dmclock_server.h:1425-1489 pull_request and
// :1627-1660 add_request of a Pull queue) without a kernel launch per call.
//
// A persistent single-workgroup kernel (k_serve) polls a host-mapped command
// block; the host writes a command and its sequence number and polls for the
// matching completion.  The pull decision needs the three heap tops
// (reservation, ready proportion, limit) over every client; instead of the
// single-op path's scan of all N fronts, the table is cut into G <= 1024
// groups of 2^gshift slots and each group's StepRed summary (the same
// reduction step_scan_body computes, with readiness taken from the F_READY
// flag alone) is kept in LDS.  A decision reduces the G summaries; an add or
// a pop changes one client, whose group is re-summarised (2^gshift fronts);
// the limit scan's ready marks (:1131-1143, committed when the reservation
// phase did not dispatch, exactly as k_fast_apply commits them) re-summarise
// only the groups whose earliest not-ready limit has passed.  The decision is
// step_decision's, the pop step_apply_body's, the add add_chain_slot's: the
// same arithmetic as every other path.
//
// Exit conditions every wave reaches: a stop command, no command for
// `idle_ticks` of the 100 MHz wall clock, or, after an answer, a lifetime of
// 5 x `idle_ticks` (the host relaunches on demand).  The lifetime bounds how
// long a queue's k_serve can hold a hardware queue that another queue's
// k_serve waits behind (more queues than hardware queues in a process).
// The summaries are written back to HBM at exit (valid until any other call
// changes the table; the host then rebuilds them with k_gsum_build).
#pragma once

constexpr int kServeThreads = 256;
constexpr uint32_t kServeMaxG = 1024;
enum : uint32_t { kServeNone = 0, kServeAdd = 1, kServePull = 2, kServeStop = 3 };
enum : uint32_t { kServeRunning = 1, kServeExited = 2 };

// Host-mapped command block.  The command is words 0-6 of one 64-byte line:
// the sequence number, op | k << 8 | check << 16, now, the request.  The
// host writes words 1-6, then the sequence number (release); k_serve reads
// all seven words with one load per poll (a lane each) and takes a new
// sequence number only with a matching check, a 48-bit hash of the other
// words (a read torn by the host's stores fails it and is polled again).
// The answer is in the second line, then done_seq (system-scope release).
// The tick (:918) is k_serve's own: the launch's, plus one per add.
struct alignas(64) ServeIO {
  uint64_t req_seq;
  uint64_t cmd;
  double now;
  dmc_request req;
  uint64_t pad0;
  // device -> host
  alignas(64) uint64_t done_seq;
  uint32_t state;
  int32_t rc;
  uint32_t n, n_res, n_prio;
  int32_t type;
  double when;
  uint64_t clk[4];  // wall clock: command seen, command read, answered, published
  uint64_t phase[3];  // wall clock inside the first step: add/total, pop, summary
  uint64_t cyc[2];    // shader clock at command read and at answer (the clock rate)
  dmc_decision dec[kFastK];
};
static_assert(offsetof(ServeIO, done_seq) == 64, "the command is one 64-byte line");
static_assert(sizeof(dmc_request) == 32, "the request is words 3-6");
constexpr int kServeCmdWords = 7;

// the command's check: a hash of its sequence number, op, k, now and request
__host__ __device__ inline uint64_t serve_check(uint64_t seq, uint64_t opk, uint64_t now,
                                                uint64_t r0, uint64_t r1, uint64_t r2,
                                                uint64_t r3) {
  uint64_t h = seq * 0x9E3779B97F4A7C15ull;
  const uint64_t w[6] = {opk & 0xffffull, now, r0, r1, r2, r3};
  for (int i = 0; i < 6; ++i) {
    h ^= w[i];
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  return h >> 16;  // 48 bits
}

__device__ inline uint64_t sys_load_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline uint32_t sys_load_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __attribute__((always_inline)) inline void stepred_clear(StepRed& a) {
  a.r = ArgMin{kMaxKey, kNone, 0};
  a.p = a.r;
  a.pnr = a.r;
  a.lmin_nr = kMaxKey;
  a.lmin_rd = kMaxKey;
  a.n_any = a.n_ready = a.n_notready = 0;
  a.pad = 0;
}

// Wave reductions on the DPP network (row shifts within 16-lane rows, then
// the row broadcasts of lane 15 and lane 31): a few ALU cycles a step, where
// a shuffle is an LDS round trip.  Every lane starts with its own value; the
// wave's result is in lane 63.  Lanes a step has no source for receive the
// identity.
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline uint32_t dpp32(uint32_t v, uint32_t idn) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)idn, (int)v, CTRL, ROWS, 0xf, false);
}
template <int C, int R>
struct DppStep {
  static constexpr int ctrl = C, rows = R;
};
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline void stepred_dpp_step(StepRed& a) {
  auto k64 = [](uint64_t v) {
    return ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32), 0xffffffffu) << 32) |
           dpp32<CTRL, ROWS>((uint32_t)v, 0xffffffffu);
  };
  auto am = [&](const ArgMin& x) {
    return ArgMin{k64(x.key), dpp32<CTRL, ROWS>(x.slot, kNone), dpp32<CTRL, ROWS>(x.cnt, 0u)};
  };
  StepRed b;
  b.r = am(a.r);
  b.p = am(a.p);
  b.pnr = am(a.pnr);
  b.lmin_nr = k64(a.lmin_nr);
  b.lmin_rd = k64(a.lmin_rd);
  b.n_any = dpp32<CTRL, ROWS>(a.n_any, 0u);
  b.n_ready = dpp32<CTRL, ROWS>(a.n_ready, 0u);
  b.n_notready = dpp32<CTRL, ROWS>(a.n_notready, 0u);
  stepred_combine(a, b);
}
__device__ __attribute__((always_inline)) inline void wave_stepred(StepRed& a) {
  stepred_dpp_step<0x111, 0xf>(a);  // row_shr:1
  stepred_dpp_step<0x112, 0xf>(a);  // row_shr:2
  stepred_dpp_step<0x114, 0xf>(a);  // row_shr:4
  stepred_dpp_step<0x118, 0xf>(a);  // row_shr:8 (lane 15 of a row: the row's)
  stepred_dpp_step<0x142, 0xa>(a);  // row_bcast:15 into rows 1 and 3
  stepred_dpp_step<0x143, 0xc>(a);  // row_bcast:31 into rows 2 and 3
}

template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline uint64_t dpp64(uint64_t v, uint64_t idn) {
  return ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32), (uint32_t)(idn >> 32)) << 32) |
         dpp32<CTRL, ROWS>((uint32_t)v, (uint32_t)idn);
}
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline void argmin_dpp_step(ArgMin& a) {
  const ArgMin b{dpp64<CTRL, ROWS>(a.key, kMaxKey), dpp32<CTRL, ROWS>(a.slot, kNone),
                 dpp32<CTRL, ROWS>(a.cnt, 0u)};
  a = argmin_combine(a, b);
}
__device__ __attribute__((always_inline)) inline void wave_argmin_dpp(ArgMin& a) {
  argmin_dpp_step<0x111, 0xf>(a);
  argmin_dpp_step<0x112, 0xf>(a);
  argmin_dpp_step<0x114, 0xf>(a);
  argmin_dpp_step<0x118, 0xf>(a);
  argmin_dpp_step<0x142, 0xa>(a);
  argmin_dpp_step<0x143, 0xc>(a);
}
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline void minsum_dpp_step(uint64_t& m0, uint64_t& m1,
                                                                       uint32_t& c0, uint32_t& c1,
                                                                       uint32_t& c2) {
  const uint64_t b0 = dpp64<CTRL, ROWS>(m0, kMaxKey), b1 = dpp64<CTRL, ROWS>(m1, kMaxKey);
  m0 = b0 < m0 ? b0 : m0;
  m1 = b1 < m1 ? b1 : m1;
  c0 += dpp32<CTRL, ROWS>(c0, 0u);
  c1 += dpp32<CTRL, ROWS>(c1, 0u);
  c2 += dpp32<CTRL, ROWS>(c2, 0u);
}

// Block-wide combine of per-thread StepReds into *out (visible to every
// thread on return): the 256 partials go to LDS and each wave reduces one
// part of the record over all of them -- wave 0 the r argmin, wave 1 p,
// wave 2 pnr, wave 3 the limit minima and the counts -- four short
// reductions side by side instead of one long one per wave.
constexpr int kServeRes = kServeThreads;  // the result's index in the LDS array
__device__ __attribute__((always_inline)) inline void serve_block_reduce(const StepRed& a,
                                                                         StepRed* part) {
  StepRed* out = part + kServeRes;
  static_assert(kServeThreads == 256, "one wave per part of the record");
  __syncthreads();  // (the previous result has been read)
  part[threadIdx.x] = a;
  __syncthreads();
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 3) {
    auto f = [&](const StepRed& x) { return w == 0 ? x.r : w == 1 ? x.p : x.pnr; };
    ArgMin m = f(part[lane]);
#pragma unroll
    for (int j = 1; j < 4; ++j) m = argmin_combine(m, f(part[lane + 64 * j]));
    wave_argmin_dpp(m);
    if (lane == 63) {
      if (w == 0) out->r = m;
      else if (w == 1) out->p = m;
      else out->pnr = m;
    }
  } else {
    uint64_t m0 = kMaxKey, m1 = kMaxKey;
    uint32_t c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const StepRed& x = part[lane + 64 * j];
      m0 = x.lmin_nr < m0 ? x.lmin_nr : m0;
      m1 = x.lmin_rd < m1 ? x.lmin_rd : m1;
      c0 += x.n_any;
      c1 += x.n_ready;
      c2 += x.n_notready;
    }
    minsum_dpp_step<0x111, 0xf>(m0, m1, c0, c1, c2);
    minsum_dpp_step<0x112, 0xf>(m0, m1, c0, c1, c2);
    minsum_dpp_step<0x114, 0xf>(m0, m1, c0, c1, c2);
    minsum_dpp_step<0x118, 0xf>(m0, m1, c0, c1, c2);
    minsum_dpp_step<0x142, 0xa>(m0, m1, c0, c1, c2);
    minsum_dpp_step<0x143, 0xc>(m0, m1, c0, c1, c2);
    if (lane == 63) {
      out->lmin_nr = m0;
      out->lmin_rd = m1;
      out->n_any = c0;
      out->n_ready = c1;
      out->n_notready = c2;
      out->pad = 0;
    }
  }
  __syncthreads();
}

// block-wide argmin into sha[0] (visible to every thread on return)
__device__ __attribute__((always_inline)) inline void serve_block_argmin(ArgMin a, ArgMin* sha) {
  auto step = [&](auto ctrl_rows) {
    constexpr int CTRL = decltype(ctrl_rows)::ctrl, ROWS = decltype(ctrl_rows)::rows;
    ArgMin b;
    b.key = ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(a.key >> 32), 0xffffffffu) << 32) |
            dpp32<CTRL, ROWS>((uint32_t)a.key, 0xffffffffu);
    b.slot = dpp32<CTRL, ROWS>(a.slot, kNone);
    b.cnt = dpp32<CTRL, ROWS>(a.cnt, 0u);
    a = argmin_combine(a, b);
  };
  step(DppStep<0x111, 0xf>{});
  step(DppStep<0x112, 0xf>{});
  step(DppStep<0x114, 0xf>{});
  step(DppStep<0x118, 0xf>{});
  step(DppStep<0x142, 0xa>{});
  step(DppStep<0x143, 0xc>{});
  __syncthreads();  // (the previous result has been read)
  if ((threadIdx.x & 63) == 63) sha[1 + (threadIdx.x >> 6)] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgMin o = sha[1];
    for (int i = 2; i <= kServeThreads / 64; ++i) o = argmin_combine(o, sha[i]);
    sha[0] = o;
  }
  __syncthreads();
}

// one front's contribution to a summary (step_scan_body's classification)
__device__ __attribute__((always_inline)) inline void summary_add(StepRed& a, const ScanRec& sr,
                                                                  uint32_t s, bool rdy) {
  ++a.n_any;
  a.r = argmin_combine(a.r, ArgMin{okey(sr.r), s, 1});
  const uint64_t kp = okey(sr.pk), kl = okey(sr.l);
  if (rdy) {
    ++a.n_ready;
    a.lmin_rd = kl < a.lmin_rd ? kl : a.lmin_rd;
    if (sr.pk < kInf) a.p = argmin_combine(a.p, ArgMin{kp, s, 1});
  } else {
    ++a.n_notready;
    a.lmin_nr = kl < a.lmin_nr ? kl : a.lmin_nr;
    a.pnr = argmin_combine(a.pnr, ArgMin{kp, s, 1});
  }
}

// One group's summary (step_scan_body's reduction over slots
// [g << gshift, (g + 1) << gshift)), into sh[kServeRes].  MARK: the limit
// scan's ready marks for fronts with l <= now are committed first;
// otherwise readiness is the flag alone.  The fronts are loaded kSumBatch
// per lane before the first is used (one memory latency per batch).
constexpr int kSumBatch = 4;  // (1024-slot groups: one batch)
template <bool MARK>
__device__ __attribute__((always_inline)) inline void group_summary(const Table& tb, uint32_t g,
                                                                    uint32_t gshift, double now,
                                                                    StepRed* sh) {
  StepRed a;
  stepred_clear(a);
  const uint32_t s0 = g << gshift;
  const uint32_t s1 = min(tb.n, s0 + (1u << gshift));
  for (uint32_t b = s0 + threadIdx.x; b < s1; b += kSumBatch * kServeThreads) {
    ScanRec rs[kSumBatch];
#pragma unroll
    for (int u = 0; u < kSumBatch; ++u) {
      const uint32_t s = b + u * kServeThreads;
      if (s < s1) rs[u] = tb.sc[s];
      else rs[u].count = 0;
    }
#pragma unroll
    for (int u = 0; u < kSumBatch; ++u) {
      const ScanRec& sr = rs[u];
      if (!sr.count) continue;
      const uint32_t s = b + u * kServeThreads;
      bool rdy = (sr.flags & F_READY) != 0;
      if (MARK && !rdy && sr.l <= now) {  // k_step_mark
        tb.sc[s].flags = sr.flags | F_READY;
        rdy = true;
      }
      summary_add(a, sr, s, rdy);
    }
  }
  serve_block_reduce(a, sh);
}

// every group's summary, one workgroup per group
__global__ void __launch_bounds__(kServeThreads)
k_gsum_build(Table tb, StepRed* gs, uint32_t gshift) {
  __shared__ StepRed sh[kServeRes + 1];
  group_summary<false>(tb, blockIdx.x, gshift, 0.0, sh);
  if (threadIdx.x == 0) gs[blockIdx.x] = sh[kServeRes];
}

// the summaries' combine (into sh[kServeRes])
__device__ __attribute__((always_inline)) inline void serve_total(const StepRed* sg, uint32_t G, StepRed* sh) {
  StepRed a;
  stepred_clear(a);
  for (uint32_t i = threadIdx.x; i < G; i += kServeThreads) stepred_combine(a, sg[i]);
  serve_block_reduce(a, sh);
}

// The answer: the command's sequence number after a release fence (the
// decisions and counts in host-mapped memory before it); thread 0.
__device__ __attribute__((always_inline)) inline void serve_publish(ServeIO* io, uint64_t seen,
                                                                    uint64_t c_seen,
                                                                    uint64_t c_read, bool trace) {
  if (trace) {
    io->clk[0] = c_seen;
    io->clk[1] = c_read;
    io->clk[2] = wall_clock64();
    io->cyc[1] = __builtin_amdgcn_s_memtime();
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (trace) io->clk[3] = wall_clock64();
  __hip_atomic_store(&io->done_seq, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One group's summary by waves 1-3 (192 lanes, their fronts kWaveSumBatch
// per lane in flight): each wave reduces its share on the DPP network, the
// last one to finish (an LDS ticket) combines the three into *sg_out and
// sets *done -- no block barrier, so that wave 0 keeps polling and serving
// adds meanwhile (a pull's deferred re-summary).
constexpr int kWaveSumBatch = 6;  // (1024-slot groups: one batch)
__device__ __attribute__((always_inline)) inline void waves_group_summary(
    const Table& tb, uint32_t g, uint32_t gshift, StepRed* sg_out, StepRed* part,
    uint32_t* ticket, uint32_t* done) {
  constexpr uint32_t NL = kServeThreads - 64;
  const uint32_t li = threadIdx.x - 64, lane = threadIdx.x & 63;
  StepRed a;
  stepred_clear(a);
  const uint32_t s0 = g << gshift;
  const uint32_t s1 = min(tb.n, s0 + (1u << gshift));
  for (uint32_t b = s0 + li; b < s1; b += kWaveSumBatch * NL) {
    ScanRec rs[kWaveSumBatch];
#pragma unroll
    for (int u = 0; u < kWaveSumBatch; ++u) {
      const uint32_t s = b + u * NL;
      if (s < s1) rs[u] = tb.sc[s];
      else rs[u].count = 0;
    }
#pragma unroll
    for (int u = 0; u < kWaveSumBatch; ++u) {
      const ScanRec& sr = rs[u];
      if (!sr.count) continue;
      summary_add(a, sr, b + u * NL, (sr.flags & F_READY) != 0);
    }
  }
  wave_stepred(a);
  if (lane == 63) {
    part[li >> 6] = a;
    if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) ==
        NL / 64 - 1) {
      StepRed t = part[0];
      for (uint32_t w = 1; w < NL / 64; ++w) stepred_combine(t, part[w]);
      *sg_out = t;
      *ticket = 0;
      __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

__global__ void __launch_bounds__(kServeThreads)
k_serve(Table tb, StepRed* gs, uint32_t G, uint32_t gshift, ServeIO* io, int at_limit,
        uint32_t nregistered, unsigned long long* sched, uint64_t seq0,
        uint64_t idle_ticks, uint64_t tick, bool trace) {
  __shared__ StepRed sg[kServeMaxG];
  __shared__ StepRed sh[kServeRes + 1];
  __shared__ ArgMin sha[kServeThreads / 64 + 1];
  __shared__ uint32_t s_nst;
  __shared__ uint16_t s_stale[kServeMaxG];
  __shared__ uint64_t s_cmd[8];  // the command line's words (op 0: exit)
  // an add's request (words 3-6 of the line), stored into a dmc_request
  // object byte-wise (st_as): read as its own type, never through s_cmd
  __shared__ dmc_request s_req;
  __shared__ uint32_t s_life;
  __shared__ int32_t s_rc;
  __shared__ StepCtl s_c;
  // a pull's last pop leaves its group's re-summary owed (s_pend): waves
  // 1-3 run it while wave 0 polls and serves adds, which need no other group's
  // summary; an add to that group waits for it (s_pdone), a pull for the
  // block barrier
  __shared__ uint32_t s_pend;
  __shared__ uint32_t s_pdone;
  __shared__ StepRed s_rpart[kServeThreads / 64 - 1];
  __shared__ uint32_t s_rticket;
  for (uint32_t i = threadIdx.x; i < G; i += kServeThreads) sg[i] = gs[i];
  if (threadIdx.x == 0) {
    s_pend = kNone;
    s_pdone = 1;
    s_rticket = 0;
    s_life = 0;
  }
  uint64_t seen = seq0;  // (wave 0's)
  const uint64_t born = wall_clock64();
  uint64_t c_seen = 0, c_read = 0;
  bool published = false;  // this command's answer is out (a pull's last decision)
  uint32_t owed = kNone;   // (every thread's copy of the group this iteration left owed)
  __syncthreads();
  for (;;) {
    const uint32_t pend = s_pend;
    if (threadIdx.x < 64) {
      // wave 0 polls: the command line, one load per poll; adds are served
      // here, one after another, until a pull (or the end) comes
      const uint32_t lane = threadIdx.x;
      // (the command words -- seq, op, now, the request -- are written by
      // the host and only ever read here, as whole words through system-
      // scope atomic loads, never as their declared members: no access of
      // another type for alias analysis to order them against)
      const uint64_t* line = reinterpret_cast<const uint64_t*>(io);
      for (;;) {
        const uint64_t t0 = wall_clock64();
        bool got = false;
        uint64_t w = 0;
        for (;;) {
          w = lane < kServeCmdWords ? sys_load_u64(line + lane) : 0;
          const uint64_t sq = shfl_u64(w, 0);
          if (sq != seen) {
            const uint64_t opk = shfl_u64(w, 1);
            if ((opk >> 16) == serve_check(sq, opk, shfl_u64(w, 2), shfl_u64(w, 3),
                                           shfl_u64(w, 4), shfl_u64(w, 5), shfl_u64(w, 6))) {
              seen = sq;
              got = true;
              break;
            }
          }
          if (wall_clock64() - t0 > idle_ticks) break;
          __builtin_amdgcn_s_sleep(1);
        }
        c_seen = wall_clock64();
        if (got) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (lane < kServeCmdWords) s_cmd[lane] = got ? w : 0;
        if (lane >= 3 && lane < 7)
          st_as<uint64_t>(reinterpret_cast<char*>(&s_req) + 8 * (lane - 3), got ? w : 0);
        c_read = c_seen;
        if (trace && lane == 0) io->cyc[0] = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t op = (uint32_t)(s_cmd[1] & 0xff);
        if (op != kServeAdd) break;  // a pull, a stop or the idle end: the block's
        // k_add_one: a request for a client with no request is its new
        // front, inserted into the group's summary (exact: nothing leaves
        // it); otherwise the fronts, and the summary, are unchanged
        const uint64_t s_tick = tick++;  // (++tick, :918: the host's count follows)
        uint32_t life = 0;
        if (lane == 0) {
          const dmc_request* s_reqp = &s_req;
          const uint32_t s = s_reqp->slot;
          if (s >= tb.n || !(tb.sc[s].flags & F_REG)) {
            s_rc = DMC_ENOTREG;
          } else {
            if (pend != kNone && (s >> gshift) == pend) {
              // (its group's owed re-summary reads the fronts: first)
              while (!__hip_atomic_load(&s_pdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
                __builtin_amdgcn_s_sleep(1);
            }
            AddParams p{s_reqp, &s_rc, s_tick, 1, 0};
            AddState st;
            add_chain_slot(tb, p, s, 1, 0, nullptr, nullptr, ActBuf{}, &st);
            if (st.front_set) {
              const ScanRec sr = tb.sc[s];
              summary_add(sg[s >> gshift], sr, s, (sr.flags & F_READY) != 0);
            }
          }
          if (trace) {
            io->phase[0] = wall_clock64();
            io->phase[2] = io->phase[0];
          }
          io->rc = s_rc;
          serve_publish(io, seen, c_seen, c_read, trace);
          life = wall_clock64() - born > 5 * idle_ticks ? 1u : 0u;
        }
        if (__builtin_amdgcn_readfirstlane(life)) {  // lifetime over
          if (lane < kServeCmdWords) s_cmd[lane] = 0;
          break;
        }
      }
    } else if (pend != kNone) {
      waves_group_summary(tb, pend, gshift, &sg[pend], s_rpart, &s_rticket, &s_pdone);
    }
    __syncthreads();  // (the owed re-summary is in)
    if (threadIdx.x == 0) s_pend = kNone;  // (read again only after the next barriers)
    owed = kNone;
    const uint32_t op = (uint32_t)(s_cmd[1] & 0xff);
    if (op != kServePull) break;
    const uint32_t s_k = (uint32_t)((s_cmd[1] >> 8) & 0xff);
    const double s_now = __builtin_bit_cast(double, s_cmd[2]);
    const uint64_t s_tick = tick;
    const double now = s_now;
    published = false;
    {
      uint32_t n = 0, nres = 0, nprio = 0;
      int32_t type = DMC_NEXT_RETURNING;
      double when = 0.0;
      published = false;
      while (n < s_k) {
        // the reservation heap's top: the group argmin of the groups' r
        // minima (lowest group on equal keys is the lowest slot; the tied
        // fronts' count is the sum)
        ArgMin ar{kMaxKey, kNone, 0};
        for (uint32_t i = threadIdx.x; i < G; i += kServeThreads)
          ar = argmin_combine(ar, ArgMin{sg[i].r.key, i, sg[i].r.cnt});
        serve_block_argmin(ar, sha);
        if (trace && threadIdx.x == 0 && n == 0) io->phase[0] = wall_clock64();
        StepCtl c{};
        c.type = -1;
        if (sha[0].key != kMaxKey && from_okey(sha[0].key) <= now) {
          c.type = DMC_NEXT_RETURNING;  // :1124-1128
          c.prio = 0;
          c.slot = sg[sha[0].slot].r.slot;
          c.tie = sha[0].cnt > 1;
        } else if (nregistered) {
          // the limit scan: re-summarise the groups holding a not-ready
          // front whose limit has passed, committing its ready mark
          if (threadIdx.x == 0) s_nst = 0;
          __syncthreads();  // (and every thread has read the r top)
          for (uint32_t i = threadIdx.x; i < G; i += kServeThreads)
            if (sg[i].n_notready && from_okey(sg[i].lmin_nr) <= now)
              s_stale[atomicAdd(&s_nst, 1u)] = (uint16_t)i;
          __syncthreads();
          const uint32_t nst = s_nst;
          for (uint32_t j = 0; j < nst; ++j) {
            const uint32_t g = s_stale[j];
            group_summary<true>(tb, g, gshift, now, sh);
            if (threadIdx.x == 0) sg[g] = sh[kServeRes];
          }
          __syncthreads();
          // the ready heap's top (:1146-1151)
          ArgMin ap{kMaxKey, kNone, 0};
          for (uint32_t i = threadIdx.x; i < G; i += kServeThreads)
            ap = argmin_combine(ap, ArgMin{sg[i].p.key, i, sg[i].p.cnt});
          serve_block_argmin(ap, sha);
          if (sha[0].key != kMaxKey) {
            c.type = DMC_NEXT_RETURNING;
            c.prio = 1;
            c.mark = 1;
            c.slot = sg[sha[0].slot].p.slot;
            c.tie = sha[0].cnt > 1;
          }
        }
        if (c.type < 0) {  // no work now: the full reduction decides
          serve_total(sg, G, sh);
          c = step_decision(sh[kServeRes], now, at_limit, nregistered);
        }
        if (c.type != DMC_NEXT_RETURNING) {
          type = c.type;
          when = c.when;
          break;
        }
        ++n;
        (c.prio ? nprio : nres)++;
        if (threadIdx.x == 0) {
          s_c = c;
          step_apply_body(tb, s_tick, &s_c, io->dec, n - 1, sched);
          if (trace && n == 1) io->phase[1] = wall_clock64();
          if (n == s_k) {
            // the call's last decision: answer first, re-summarise after
            io->n = n;
            io->n_res = nres;
            io->n_prio = nprio;
            io->type = type;
            io->when = when;
            serve_publish(io, seen, c_seen, c_read, trace);
          }
        }
        published = n == s_k;
        __syncthreads();
        const uint32_t g = c.slot >> gshift;
        if (published) {
          // the call's last pop: its group's re-summary is owed (waves
          // 1-3, beside the next commands' polling)
          owed = g;
          if (threadIdx.x == 0) {
            s_pend = g;
            s_pdone = 0;
          }
        } else {
          group_summary<false>(tb, g, gshift, now, sh);
          if (threadIdx.x == 0) sg[g] = sh[kServeRes];
        }
        if (trace && threadIdx.x == 0 && n == 1) io->phase[2] = wall_clock64();
        __syncthreads();
      }
      if (threadIdx.x == 0 && !published) {
        io->n = n;
        io->n_res = nres;
        io->n_prio = nprio;
        io->type = type;
        io->when = when;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!published) serve_publish(io, seen, c_seen, c_read, trace);
      s_life = wall_clock64() - born > 5 * idle_ticks;
    }
    __syncthreads();
    if (s_life) break;  // lifetime over
  }
  // (a re-summary still owed: the lifetime ended right after a pull)
  if (owed != kNone) {
    const uint32_t g = owed;
    group_summary<false>(tb, g, gshift, 0.0, sh);
    if (threadIdx.x == 0) sg[g] = sh[kServeRes];
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < G; i += kServeThreads) gs[i] = sg[i];
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(&io->state, (uint32_t)kServeExited, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
