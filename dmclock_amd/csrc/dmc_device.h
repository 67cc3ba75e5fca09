// SPDX-License-Identifier: LGPL-2.1
//
// dmc_device.h -- device-side data layout and per-client arithmetic of the
// MI355X dmClock engine.  Everything here is exact IEEE-754 double arithmetic
// in the reference's order (no FMA contraction: explicit __d*_rn intrinsics,
// and the library is built with -ffp-contract=off).
//
// Layout (per queue, N client slots, ring capacity Q):
//   ScanRec (32 B per slot, struct of arrays): the front request's heap keys
//     -- reservation r, proportion key pk = p + prop_delta, limit l -- the
//     ring cursor and the flags: everything a pass over the whole table
//     reads, one coalesced 32-byte record per slot;
//   ClientRec (64 B, random access): prev tag, inverses, prop_delta;
//   ClientAux (16 B, random access): cur_delta / cur_rho, last_tick;
//   request rings: ring[slot * Q + i], one 64-byte ReqEntry per request.
// A client a walker or the add path visits costs its ClientRec line, its
// ScanRec line and the ring lines it uses.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// k_chain_scan's batch stamp in ScanRec::stamp (1), or a separate 32-bit
// touch array (0, rounds 4's layout, for A/B)
#ifndef DMC_STAMP_SC
#define DMC_STAMP_SC 1
#endif

// Kernels request their first data with the gate / skip word they check
// (one level of loads instead of two; 0: the check first, round 4's form)
#ifndef DMC_EARLY_LOADS
#define DMC_EARLY_LOADS 1
#endif

namespace dmc {

constexpr double kInf = __builtin_huge_val();
constexpr uint64_t kMaxKey = ~0ull;
// ReqEntry::dec of a request no pull round has dispatched (set at add)
constexpr uint32_t kNoDec = 0xffffffffu;

enum : uint8_t { F_IDLE = 1, F_READY = 2, F_REG = 4 };

// One queued request: its tag (RequestTag, dmclock_server.h:135-143) plus the
// opaque handle that stands for the RequestRef.
struct alignas(16) ReqEntry {
  double r, p, l, arrival;
  uint64_t handle;
  uint32_t cost, delta, rho;
  uint32_t dec;  // pull round stamp: decision offset of this pop (kNoDec: none)
  uint32_t tie;  // pull round scratch: tie flag of this pop
  uint32_t pad;
};
static_assert(sizeof(ReqEntry) == 64, "ReqEntry must be 64 bytes");

// Per-client state the add, emit and apply kernels reach at random: one
// line (the scanned columns are ScanRec's).
struct alignas(64) ClientRec {
  double prev_r, prev_p, prev_l, prev_arr;  // ClientRec::prev_tag
  double r_inv, w_inv, l_inv;                // ClientInfo inverses
  double pd;                                 // ClientRec::prop_delta
};
static_assert(sizeof(ClientRec) == 64, "ClientRec must be 64 bytes");

// Per-client state only the add path (and delayed pops) touch.
struct alignas(16) ClientAux {
  uint32_t cur_delta, cur_rho;  // last ReqParams
  uint64_t last_tick;
};
static_assert(sizeof(ClientAux) == 16, "ClientAux must be 16 bytes");

// The front request's heap keys (the reference's three heaps order clients
// by these, dmclock_server.h:722-757), the ring cursor and the flags.  pk is
// the ready heap's key p + prop_delta (:734-735), cached: it changes with
// the front and with prop_delta (activations), and its writers compute it
// with the reference's arithmetic (__dadd_rn).
struct alignas(32) ScanRec {
  double r, pk, l;
  uint8_t head, count;  // request ring cursor (ring capacity <= 64)
  uint8_t flags;        // F_*
  uint8_t stamp;        // the low byte of the epoch of the last add batch that
                        // filed the slot with the scan running beside the add
                        // chain (k_chain_scan's scan leaves such slots to the
                        // chain); cleared for every slot when the epoch wraps
  uint32_t nadd;        // the add batch in flight: the client's requests in it
                        // (k_add_link's atomic; k_add_chain resets it; 0
                        // outside a batch)
};
static_assert(sizeof(ScanRec) == 32, "ScanRec must be 32 bytes");
static_assert(offsetof(ScanRec, head) == 24 && offsetof(ScanRec, count) == 25 &&
                  offsetof(ScanRec, flags) == 26 && offsetof(ScanRec, stamp) == 27 &&
                  offsetof(ScanRec, nadd) == 28,
              "ScanRec cursor layout");

// The ClientInfo client_info_f returns for a client now (its inverses): the
// caller publishes it with dmc_client_bind_info_batch.  With dynamic_info
// (U1) every tag calculation reads it and makes it the client's cached info
// (get_cli_info, dmclock_server.h:870-875); the reductions use the cached
// info (:1083-1109), as the reference's client.info.
struct alignas(32) BoundInfo {
  double r_inv, w_inv, l_inv, pad;
};
static_assert(sizeof(BoundInfo) == 32, "BoundInfo must be 32 bytes");

// Client table pointers (passed by value to kernels).
struct Table {
  uint32_t n;      // slots
  uint32_t q;      // ring capacity (power of two, <= 64)
  uint32_t qmask;
  int32_t delayed;
  int32_t at_limit;
  double reject_thr;
  double antic;
  ClientRec* rec;  // N
  ScanRec* sc;     // N
  ClientAux* aux;  // N
  ReqEntry* ring;
  const BoundInfo* binfo;  // U1 (dynamic_info): read at every tag; else null
  // DMC_OPT_PIPELINE: the gate word a pipelined round's end sets when the
  // host must finish its call first; the next call's graph, already queued,
  // then does nothing (every kernel of it checks); else null
  const uint32_t* gate;
  // per slot: the epoch of the last add batch that filed it with the scan
  // running beside the add chain (AddParams::epoch, k_chain_scan)
  uint32_t* touch;
  // DMC_OPT_HEAP_ORDER: per position of the running add batch, the heap calls
  // the reference makes for it (k_add_chain writes, k_heap_events replays:
  // 0 none, 1 a key changed with no heap call, 2 adjust x 3, 3 adjust x 3
  // twice); else null
  uint8_t* hev;
};

__host__ __device__ inline uint64_t dbits(double x) {
  uint64_t u;
  __builtin_memcpy(&u, &x, 8);
  return u;
}
__host__ __device__ inline double bitsd(uint64_t u) {
  double x;
  __builtin_memcpy(&x, &u, 8);
  return x;
}
// Whole-word access to memory declared with other types (a vector load of a
// scalar column, a record's words, the ScanRec cursor): through
// __builtin_memcpy, whose byte access may alias any type, so type-based
// alias analysis can never move it across the members' own loads and stores
// (an access through a reinterpret_cast pointer of another type could be,
// and once was: DESIGN.md section 10).  p must be aligned for T; the copy
// compiles to one access of sizeof(T) bytes.
template <typename T>
__device__ inline T ld_as(const void* p) {
  T v;
  __builtin_memcpy(&v, __builtin_assume_aligned(p, alignof(T)), sizeof(T));
  return v;
}
template <typename T>
__device__ inline void st_as(void* p, const T& v) {
  __builtin_memcpy(__builtin_assume_aligned(p, alignof(T)), &v, sizeof(T));
}

// The same, through an explicit address space: ld_lds (p in LDS: ds_read)
// and ld_glb (p in device memory: global_load).  Where one value comes from
// either an LDS stage or memory, one generic pointer compiles to a flat
// access, which counts against both of the wave's memory counters (a wait
// for an LDS read then also waits for it) and which the compiler orders
// behind pending flat stores.  The words are may_alias (any type, as
// ld_as's byte copy).
typedef uint32_t __attribute__((may_alias, address_space(3))) lds_w32;
typedef unsigned long long __attribute__((may_alias, address_space(3))) lds_w64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((may_alias, address_space(3))) lds_w128;
typedef uint32_t __attribute__((may_alias, address_space(1))) glb_w32;
typedef unsigned long long __attribute__((may_alias, address_space(1))) glb_w64;
typedef u32x4 __attribute__((may_alias, address_space(1))) glb_w128;
template <typename T, typename W128, typename W64, typename W32>
__device__ __forceinline__ T ld_words(const void* p) {
  T v;
  if constexpr (sizeof(T) % 16 == 0 && alignof(T) >= 16) {
    u32x4 t[sizeof(T) / 16];
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 16); ++k) t[k] = ((const W128*)p)[k];
    __builtin_memcpy(&v, t, sizeof(T));
  } else if constexpr (sizeof(T) % 8 == 0 && alignof(T) >= 8) {
    unsigned long long t[sizeof(T) / 8];
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 8); ++k) t[k] = ((const W64*)p)[k];
    __builtin_memcpy(&v, t, sizeof(T));
  } else {
    static_assert(sizeof(T) % 4 == 0 && alignof(T) >= 4, "whole 4-byte words");
    uint32_t t[sizeof(T) / 4];
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) t[k] = ((const W32*)p)[k];
    __builtin_memcpy(&v, t, sizeof(T));
  }
  return v;
}
template <typename T, typename W128, typename W64, typename W32, size_t A = alignof(T)>
__device__ __forceinline__ void st_words(void* p, const T& v) {
  if constexpr (sizeof(T) % 16 == 0 && A >= 16) {
    u32x4 t[sizeof(T) / 16];
    __builtin_memcpy(t, &v, sizeof(T));
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 16); ++k) ((W128*)p)[k] = t[k];
  } else if constexpr (sizeof(T) % 8 == 0 && A >= 8) {
    unsigned long long t[sizeof(T) / 8];
    __builtin_memcpy(t, &v, sizeof(T));
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 8); ++k) ((W64*)p)[k] = t[k];
  } else {
    static_assert(sizeof(T) % 4 == 0 && alignof(T) >= 4, "whole 4-byte words");
    uint32_t t[sizeof(T) / 4];
    __builtin_memcpy(t, &v, sizeof(T));
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) ((W32*)p)[k] = t[k];
  }
}
template <typename T, size_t A = alignof(T)>
__device__ __forceinline__ void st_lds(void* p, const T& v) {
  st_words<T, lds_w128, lds_w64, lds_w32, A>(p, v);
}
// (A: the alignment p has, when more than T's)
template <typename T, size_t A = alignof(T)>
__device__ __forceinline__ void st_glb(void* p, const T& v) {
  st_words<T, glb_w128, glb_w64, glb_w32, A>(p, v);
}
template <typename T>
__device__ __forceinline__ T ld_lds(const void* p) {
  return ld_words<T, lds_w128, lds_w64, lds_w32>(p);
}
template <typename T>
__device__ __forceinline__ T ld_glb(const void* p) {
  return ld_words<T, glb_w128, glb_w64, glb_w32>(p);
}

// The ScanRec cursor word -- head | count << 8 | flags << 16 | stamp << 24 |
// nadd << 32 -- read and written whole (8-aligned at offset 24).
__device__ inline uint64_t cursor_load(const ScanRec* r) {
  return ld_as<uint64_t>(reinterpret_cast<const char*>(r) + offsetof(ScanRec, head));
}
__device__ inline void cursor_store(ScanRec* r, uint64_t w) {
  st_as<uint64_t>(reinterpret_cast<char*>(r) + offsetof(ScanRec, head), w);
}
static_assert(offsetof(ScanRec, head) == 24 && offsetof(ScanRec, nadd) == 28,
              "the cursor word is ScanRec's last 8 bytes");

// order-preserving map double -> u64 (ascending)
__host__ __device__ inline uint64_t okey(double x) {
  uint64_t u = dbits(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ inline double from_okey(uint64_t k) {
  return bitsd((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// tag_calc, dmclock_server.h:246-259
__device__ inline double tag_step(double time, double prev, double inc,
                                  uint32_t dist, bool high, uint32_t cost) {
  if (inc == 0.0) return high ? kInf : -kInf;
  double units = (double)((uint64_t)dist + (uint64_t)cost);
  double cand = __dadd_rn(prev, __dmul_rn(inc, units));
  return (time < cand) ? cand : time;
}

struct Tag3 {
  double r, p, l, arrival;
};

// RequestTag(prev, info, delta, rho, time, cost, antic), :145-183.
// Returns false where the reference asserts.
__device__ inline bool make_tag(const Tag3& prev, double rinv, double winv,
                                double linv, uint32_t delta, uint32_t rho,
                                double time, uint32_t cost, double antic,
                                Tag3* out) {
  if (cost == 0) return false;
  double max_time = time;
  if (__dsub_rn(time, antic) < prev.arrival) max_time = __dsub_rn(max_time, antic);
  Tag3 t;
  t.r = tag_step(max_time, prev.r, rinv, rho, true, cost);
  t.p = tag_step(max_time, prev.p, winv, delta, true, cost);
  t.l = tag_step(max_time, prev.l, linv, delta, false, cost);
  t.arrival = time;
  if (!(t.r < kInf || t.p < kInf)) return false;
  *out = t;
  return true;
}

// assign_unpinned_tag / update_req_tag, :399-412 (prev in registers)
__device__ inline void assign_unpinned(double& lhs, double rhs) {
  if (rhs != kInf && rhs != -kInf) lhs = rhs;
}

// reduce_reservation_tags offset, :1090-1091: uint32 (cost + rho) first
__device__ inline double resv_offset(double rinv, uint32_t cost,
                                     uint32_t rho) {
  return __dmul_rn(rinv, (double)(uint32_t)(cost + rho));
}

// Per-client sequence of pops inside one pull batch at fixed `now` is a pure
// function of that client's own state (see dmc_round.h).  The walkers below
// enumerate it; the kernels that call them (scan, emit, apply) run the same
// arithmetic, so what is applied is exactly what was ranked.

// A client's queue state as the walkers need it, loaded once by the caller
// (all loads issued together, before the first ring access).
struct CView {
  uint32_t h, c;          // ring head, queued requests
  uint32_t cd, cr;        // cur_delta, cur_rho (delayed mode)
  double rinv, winv, linv;  // the cached ClientInfo (client.info)
  double pd;              // prop_delta
  double tr, tw, tl;      // the info a delayed tag calculation reads (U1: bound)
  // reduce_reservation_tags' inverse after a pop at queue position i of a
  // batch (delayed mode): the pop fetched the info if an entry follows it,
  // and so did every earlier pop of the batch (:1021-1036, 1077-1111)
  __device__ double red_rinv(uint32_t i) const {
    return (i > 0 || i + 1 < c) ? tr : rinv;
  }
};

// the tag-calculation info of a view: U1 reads the bound info
__device__ inline void view_tag_info(const Table& tb, uint32_t s, CView& v) {
  if (tb.delayed && tb.binfo) {
    const BoundInfo b = tb.binfo[s];
    v.tr = b.r_inv;
    v.tw = b.w_inv;
    v.tl = b.l_inv;
  } else {
    v.tr = v.rinv;
    v.tw = v.winv;
    v.tl = v.linv;
  }
}

__device__ inline CView load_view(const Table& tb, uint32_t s) {
  CView v;
  v.h = tb.sc[s].head;
  v.c = tb.sc[s].count;
  v.cd = tb.aux[s].cur_delta;
  v.cr = tb.aux[s].cur_rho;
  v.rinv = tb.rec[s].r_inv;
  v.winv = tb.rec[s].w_inv;
  v.linv = tb.rec[s].l_inv;
  v.pd = tb.rec[s].pd;
  view_tag_info(tb, s, v);
  return v;
}

// A client's queue as the walkers read it: queue position i (0 = front) is
// ring entry (h + i) & qmask.  The first `ns` positions may be staged (LDS)
// by the caller: one burst of wide loads before the walk instead of one
// dependent 64-byte read per visit (on gfx950 every wait for a load also
// waits for the wave's earlier stores, so interleaved entry reads and
// decision stores serialise).
struct RingView {
  const ReqEntry* g;   // the client's ring
  const ReqEntry* st;  // staged positions [0, ns) (LDS)
  uint32_t h, qmask, ns;
  // (each side through its own address space: ld_lds / ld_glb)
  __device__ ReqEntry at(uint32_t i) const {
    if (i < ns) return ld_lds<ReqEntry>(st + i);
    return ld_glb<ReqEntry>(g + ((h + i) & qmask));
  }
  __device__ double r_at(uint32_t i) const {
    if (i < ns) return ld_lds<double>(&st[i].r);
    return ld_glb<double>(&g[(h + i) & qmask].r);
  }
  // reduce_reservation_tags' offset of position i (:1090-1091)
  __device__ double offset_at(uint32_t i, double rinv) const {
    uint32_t cost, rho;
    if (i < ns) {
      cost = ld_lds<uint32_t>(&st[i].cost);
      rho = ld_lds<uint32_t>(&st[i].rho);
    } else {
      cost = ld_glb<uint32_t>(&g[(h + i) & qmask].cost);
      rho = ld_glb<uint32_t>(&g[(h + i) & qmask].rho);
    }
    return resv_offset(rinv, cost, rho);
  }
};

__device__ inline RingView ring_view(const Table& tb, uint32_t s, uint32_t h) {
  return RingView{tb.ring + (size_t)s * tb.q, nullptr, h, tb.qmask, 0};
}

// Stage the first min(c, K) queue positions of slot s into st (this
// thread's LDS slice): all loads issued before the first store.  In two
// halves (StageLoads: the burst in registers; stage_put: its LDS stores) so
// that a caller can issue its other loads of the same level in between.
template <int K>
struct StageLoads {
  uint4 x[K][4];  // 16-byte chunks (registers, never a private array)
  uint32_t ns;
};
// ALL: all K positions, queued or not (every index is masked into the
// slot's ring: in bounds; positions past the count are staged and never
// read): no value-or-zero per load, whose merge the compiler resolves with
// a copy -- and a wait -- right after each load (k_remit's walkers); else
// only the queued ones (k_rapply)
template <int K, bool ALL = false>
__device__ __attribute__((always_inline)) inline StageLoads<K> stage_load(
    const Table& tb, uint32_t s, uint32_t h, uint32_t c, const ReqEntry* st) {
  StageLoads<K> L;
  L.ns = st ? (c < (uint32_t)K ? c : (uint32_t)K) : 0;
  const ReqEntry* g = tb.ring + (size_t)s * tb.q;
  if (ALL) {
    if (st) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const char* src = reinterpret_cast<const char*>(g + ((h + j) & tb.qmask));
#pragma unroll
        for (int k = 0; k < 4; ++k) L.x[j][k] = ld_as<uint4>(src + 16 * k);
      }
    }
    return L;
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const char* src = reinterpret_cast<const char*>(g + ((h + j) & tb.qmask));
#pragma unroll
    for (int k = 0; k < 4; ++k)
      L.x[j][k] = (uint32_t)j < L.ns ? ld_as<uint4>(src + 16 * k) : make_uint4(0, 0, 0, 0);
  }
  return L;
}
template <int K>
__device__ __attribute__((always_inline)) inline RingView stage_put(
    const Table& tb, uint32_t s, uint32_t h, const StageLoads<K>& L, ReqEntry* st) {
  RingView v = ring_view(tb, s, h);
  if (!st) return v;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    char* dst = reinterpret_cast<char*>(st + j);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((uint32_t)j < L.ns) st_as<uint4>(dst + 16 * k, L.x[j][k]);
  }
  v.st = st;
  v.ns = L.ns;
  return v;
}
template <int K>
__device__ inline RingView stage_ring(const Table& tb, uint32_t s, uint32_t h,
                                      uint32_t c, ReqEntry* st) {
  if (!st) return ring_view(tb, s, h);
  const StageLoads<K> L = stage_load<K>(tb, s, h, c, st);
  return stage_put<K>(tb, s, h, L, st);
}

__device__ inline void keep(double v) { asm volatile("" ::"v"(v)); }

// Visitor callbacks: pop(i, tag, cost, handle, kind, dec, tie) for each pop
// (i = queue position, dec/tie = the ring entry's round scratch; kind: a
// PopKind), and group(key, run) after each priority group.
enum PopKind : uint32_t {
  kPopR = 0,      // reservation pop
  kPopHead = 1,   // priority pop opening a group (the group's key)
  kPopChain = 2,  // priority pop inside a limit-break group's run (walk_p, brk)
};
struct NullVisit {
  __device__ void pop(uint32_t, const Tag3&, uint32_t, uint64_t, uint32_t, uint32_t,
                      uint32_t) {}
  __device__ void group(uint64_t, uint32_t) {}
};

// Reservation phase walk (R-prefix): entries whose reservation tag is
// <= min(now, thr) and whose ordered key <= T, popped without reductions.
// Immediate mode reads stored tags; Delayed mode recomputes each new front
// with update_next_tag (:1021-1036).  `limit` bounds the pops (apply mode).
// Returns the number of pops; leaves the final prev tag in *prev (delayed).
// `stamped` (apply): walk exactly the entries the ranking stamped.
template <typename V>
__device__ inline uint32_t walk_r(const Table& tb, const RingView& rv, const CView& cv,
                                  double now, uint64_t T, uint32_t limit, V& vis,
                                  Tag3* prev_io, Tag3* front_out,
                                  uint32_t* front_cost, bool stamped = false) {
  const uint32_t c = cv.c;
  uint32_t n = 0;
  if (c == 0) return 0;
  if (!tb.delayed) {
    ReqEntry e = rv.at(0);
    while (n < c && n < limit) {
      if (!(e.r <= now) || okey(e.r) > T || (stamped && e.dec == kNoDec)) break;
      vis.pop(n, Tag3{e.r, e.p, e.l, e.arrival}, e.cost, e.handle, kPopR, e.dec,
              e.tie);
      ++n;
      if (n < c) e = rv.at(n);
    }
    if (front_out && n < c) {
      *front_out = Tag3{e.r, e.p, e.l, e.arrival};
      *front_cost = e.cost;
    }
    return n;
  }
  // delayed: front tag is stored; later tags are computed at pop time
  ReqEntry e0 = rv.at(0);
  Tag3 cur{e0.r, e0.p, e0.l, e0.arrival};
  uint32_t cur_cost = e0.cost, cur_dec = e0.dec, cur_tie = e0.tie;
  uint64_t cur_h = e0.handle;
  while (n < c && n < limit) {
    if (!(cur.r <= now) || okey(cur.r) > T || (stamped && cur_dec == kNoDec)) break;
    vis.pop(n, cur, cur_cost, cur_h, kPopR, cur_dec, cur_tie);
    ++n;
    if (n < c) {
      const ReqEntry e = rv.at(n);
      Tag3 nt;
      if (!make_tag(cur, cv.tr, cv.tw, cv.tl, cv.cd, cv.cr, e.arrival,
                    e.cost, tb.antic, &nt))
        nt = Tag3{e.r, e.p, e.l, e.arrival};
      if (prev_io) {
        assign_unpinned(prev_io->r, nt.r);
        assign_unpinned(prev_io->l, nt.l);
        assign_unpinned(prev_io->p, nt.p);
        prev_io->arrival = nt.arrival;
      }
      cur = nt;
      cur_cost = e.cost;
      cur_h = e.handle;
      cur_dec = e.dec;
      cur_tie = e.tie;
    }
  }
  if (front_out && n < c) {
    *front_out = cur;
    *front_cost = cur_cost;
  }
  return n;
}

// Priority phase walk: a sequence of groups, each a priority pop of the
// front (eligible if ready and proportion < inf; the first front's ready
// flag comes from the table, later fronts become ready at the next limit
// scan iff limit <= now) with key p + prop_delta <= T, followed by the
// reservation pops its reduce_reservation_tags exposes (r <= now).
// `limit` bounds the total pops (apply mode).  On return *pmask has bit i set
// for every entry popped by priority (immediate mode), used to recompute the
// reduced reservation tags of the entries behind them.
// brk (limit-break rounds, AtLimit::Allow, immediate mode): the pulls after
// the eligible work ran out (no front with r <= now, none ready) pop the
// ready-heap top regardless of its limit (:1157-1165); each such group's
// run then takes the pops its reduction exposes to the next pulls: a front
// with r <= now (reservation) or with l <= now (readied by the next limit
// scan and popped as the only ready front, kPopChain), until the front has
// neither.
struct WalkP {
  uint32_t pops;
  uint32_t groups;
  uint64_t pmask;
};

// immediate-mode reservation tag of entry i after the reductions of the
// priority pops before it, applied in order (:1088-1095)
__device__ inline double reduced_r(const RingView& rv, uint32_t i, uint64_t pmask,
                                   double rinv) {
  double r = rv.r_at(i);
  // the priority pops before i, ascending (i <= 63: queue capacity <= 64)
  for (uint64_t m = pmask & ((1ull << i) - 1ull); m; m &= m - 1ull)
    r = __dsub_rn(r, rv.offset_at((uint32_t)__ffsll((unsigned long long)m) - 1u, rinv));
  return r;
}

// The walk starts at queue position `start` (the front left after the
// round's reservation pops); `start_tag` is that entry's tag in delayed mode
// (the walk_r front, used iff use_start_tag), `ready0` its ready flag (only
// the untouched front can carry one: a front exposed by a reservation pop is
// ready iff limit <= now).
// `kstamp` != 0 (apply, kstamp = the round's k): walk exactly the groups the
// ranking stamped; a group stamped at decision offset o keeps at most
// kstamp - o pops (the round's last group can be cut inside its run).
template <typename V>
__device__ inline WalkP walk_p(const Table& tb, const RingView& rv, const CView& cv,
                               double now, uint64_t T, uint32_t limit, V& vis,
                               Tag3* prev_io, Tag3* front_out,
                               uint32_t* front_cost, uint32_t start,
                               Tag3 start_tag, bool use_start_tag, bool ready0,
                               uint32_t kstamp = 0, bool brk = false) {
  WalkP w{0, 0, 0};
  const uint32_t c = cv.c;
  if (start >= c) return w;
  const double pdv = cv.pd, rinv = cv.rinv;
  if (!tb.delayed) {
    uint32_t i = start;
    while (i < c && w.pops < limit) {
      const ReqEntry e = rv.at(i);
      // (a limit-break group's head needs no readiness: brk)
      bool rdy = brk || ((i == start) ? (ready0 || e.l <= now) : (e.l <= now));
      if (!rdy || !(e.p < kInf)) break;
      uint64_t key = okey(__dadd_rn(e.p, pdv));
      if (key > T || (kstamp && e.dec == kNoDec)) break;
      const uint32_t glim = kstamp ? kstamp - e.dec : 0xffffffffu;  // pops in group
      double r_now = reduced_r(rv, i, w.pmask, rinv);
      vis.pop(i, Tag3{r_now, e.p, e.l, e.arrival}, e.cost, e.handle, kPopHead, e.dec,
              e.tie);
      w.pmask |= 1ull << i;
      ++i;
      ++w.pops;
      uint32_t run = 0;
      while (i < c && w.pops < limit && run + 1 < glim) {
        double ri = reduced_r(rv, i, w.pmask, rinv);
        const ReqEntry er = rv.at(i);
        if (ri <= now) {  // the next pull's reservation pop
          vis.pop(i, Tag3{ri, er.p, er.l, er.arrival}, er.cost, er.handle, kPopR,
                  er.dec, er.tie);
        } else if (brk && er.l <= now && er.p < kInf) {
          // limit breaks: the next pull's limit scan readies this front and
          // pops it (the only ready front, :1135-1151), with its reduction
          vis.pop(i, Tag3{ri, er.p, er.l, er.arrival}, er.cost, er.handle, kPopChain,
                  er.dec, er.tie);
          w.pmask |= 1ull << i;
        } else {
          break;
        }
        ++i;
        ++w.pops;
        ++run;
      }
      vis.group(key, run);
      ++w.groups;
    }
    if (front_out && i < c) {
      const ReqEntry e = rv.at(i);
      *front_out = Tag3{reduced_r(rv, i, w.pmask, rinv), e.p, e.l, e.arrival};
      *front_cost = e.cost;
    }
    return w;
  }
  // delayed mode
  const ReqEntry e0 = rv.at(start);
  Tag3 cur = use_start_tag ? start_tag : Tag3{e0.r, e0.p, e0.l, e0.arrival};
  uint32_t cur_cost = e0.cost, cur_dec = e0.dec, cur_tie = e0.tie;
  uint32_t cur_rho = start ? cv.cr : e0.rho;  // a recomputed front carries cur_rho
  uint64_t cur_h = e0.handle;
  uint32_t i = start;
  auto advance = [&](bool prio) {
    // pop entry i (tag `cur`), compute the next front by update_next_tag and,
    // after a priority pop, reduce it and prev (:1021-1036, :1077-1085)
    double off = prio ? resv_offset(cv.red_rinv(i), cur_cost, cur_rho) : 0.0;
    ++i;
    if (i < c) {
      const ReqEntry e = rv.at(i);
      Tag3 nt;
      if (!make_tag(cur, cv.tr, cv.tw, cv.tl, cv.cd, cv.cr, e.arrival, e.cost,
                    tb.antic, &nt))
        nt = Tag3{e.r, e.p, e.l, e.arrival};
      if (prev_io) {
        assign_unpinned(prev_io->r, nt.r);
        assign_unpinned(prev_io->l, nt.l);
        assign_unpinned(prev_io->p, nt.p);
        prev_io->arrival = nt.arrival;
      }
      if (prio) nt.r = __dsub_rn(nt.r, off);
      cur = nt;
      cur_cost = e.cost;
      cur_rho = cv.cr;
      cur_h = e.handle;
      cur_dec = e.dec;
      cur_tie = e.tie;
    }
    if (prio && prev_io) prev_io->r = __dsub_rn(prev_io->r, off);
  };
  while (i < c && w.pops < limit) {
    bool rdy = (i == start) ? (ready0 || cur.l <= now) : (cur.l <= now);
    if (!rdy || !(cur.p < kInf)) break;
    uint64_t key = okey(__dadd_rn(cur.p, pdv));
    if (key > T || (kstamp && cur_dec == kNoDec)) break;
    const uint32_t glim = kstamp ? kstamp - cur_dec : 0xffffffffu;  // pops in group
    vis.pop(i, cur, cur_cost, cur_h, kPopHead, cur_dec, cur_tie);
    advance(true);
    ++w.pops;
    uint32_t run = 0;
    while (i < c && w.pops < limit && run + 1 < glim) {
      if (!(cur.r <= now)) break;
      vis.pop(i, cur, cur_cost, cur_h, kPopR, cur_dec, cur_tie);
      advance(false);
      ++w.pops;
      ++run;
    }
    vis.group(key, run);
    ++w.groups;
  }
  if (front_out && i < c) {
    *front_out = cur;
    *front_cost = cur_cost;
  }
  return w;
}

}  // namespace dmc
