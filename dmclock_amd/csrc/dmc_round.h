// SPDX-License-Identifier: LGPL-2.1
//
// dmc_round.h -- one batched pull round: k successive pull_request(now)
// (dmclock_server.h:1420-1489, do_next_request :1115-1186) as six
// data-parallel kernels over the client table.
//
// Why one round covers both heaps.  Within a batch of pulls at one `now`:
//  * while some front has r <= now the pulls are reservation pops in
//    ascending r (:1124-1128), with no reductions: each client contributes a
//    prefix of its queue ("R prefix": the entries with r <= now);
//  * once none is left, every pull runs the limit scan (:1135-1144) and pops
//    the ready front with the smallest p + prop_delta (:1146-1151); its
//    reduce_reservation_tags (:1077-1111) can expose reservation pops of that
//    client only, taken by the very next pulls.  Each client contributes a
//    sequence of *groups* (a priority pop + the reservation run it exposes)
//    with non-decreasing keys, starting from its state after its R prefix.
// So the first k pulls are: if the R prefixes hold n_R >= k entries, the k
// smallest of them; otherwise all n_R of them followed by the P groups in key
// order up to k - n_R pops.  Each client's R prefix and group sequence is a
// pure function of its own state, enumerated by one thread (walk_r / walk_p),
// and the global order comes from ranking (phase, key, slot, ring position).
//
// Kernels (one thread per client slot unless noted):
//   k_rscan   R prefix length + first R key, first P key of the post-R front,
//             pending limit-scan mark; per-block counts and key ranges
//             (the graph's parameter node: publishes the call's parameters)
//   k_rhist   the round's totals; key histograms of both phases (2048 bins
//             each, over the exact key ranges, flushed into kShards shards);
//             its last block: thresholds T_R / T_P (every key <= T is a
//             candidate, at least the needed number of keys are <= T) and the
//             rank-bin tables (R bins [0, kNBPhase), P bins [kNBPhase, kNBR))
//   k_remit   candidates (first key <= T) selected and compacted per wave,
//             the others' pending marks settled; candidates enumerate their
//             entries into rank bins; its last block: the bins' prefix sums,
//             the decision count
//   k_rrank   one block per rank bin: rank in LDS, decide, stamp the ring entries
//   k_rapply  replays each candidate's dispatched pops with the same
//             arithmetic, writes the decision records and the new state
//   k_rfinish round summary to host-mapped memory (AtLimit::Allow; under
//             Wait / Reject k_round_future ends the round, running the
//             terminal pull first when the round ran out of work)
// A rank bin that outgrows kBinCap (massively tied keys) aborts the round
// (overflow = 2): the host replays it on the radix path (dense entries,
// 32-bit radix sort + exact fix-up).
#pragma once

#include <type_traits>

#include "dmc_device.h"

namespace dmc {

constexpr int kBlockR = 256;
// k_rrank's block (one rank bin each): 128 threads, so that all 4096 bins'
// blocks are resident at once (16 per CU; r04e: 12.6 vs 14.7 us at 256)
#ifndef DMC_RANK_THREADS
#define DMC_RANK_THREADS 128
#endif
constexpr int kRankThreads = DMC_RANK_THREADS;
constexpr int kHistBinsR = 2048;        // per phase
constexpr int kNBR = 4096;              // rank bins: R [0, 2048), P [2048, 4096)
constexpr int kNBPhase = kNBR / 2;
// super-bins of 64 rank bins: k_remit's blocks sum their records per
// super-bin in LDS and flush the sums, so that each k_rrank block finds its
// bin's offsets from 64 super-bin sums and the <= 63 bins before it in its
// super-bin (no prefix pass over all 4096 bins)
constexpr int kSupBins = 64;
constexpr int kNSup = kNBR / kSupBins;
// The histogram's shards (block % kShards): one, measured fastest (select
// 15.9 -> 13.4 us against 8 XCD shards): the pick's loads of every shard
// cost more than the same-address flush atomics of k_rhist's 32 blocks.
#ifndef DMC_HIST_SHARDS
#define DMC_HIST_SHARDS 1
#endif
constexpr int kShards = DMC_HIST_SHARDS;
// k_remit's sampled-threshold counts: one per XCD (256 blocks' same-address
// atomics would serialise)
constexpr int kCntShards = 8;
constexpr uint32_t kBinCapR = 512;      // entries per rank bin (2 per thread of k_rrank)
constexpr uint32_t kNoneR = 0xffffffffu;
constexpr uint8_t F_PMARK = 8;          // pending limit-scan mark (this round)

// Per-phase selection state.
struct PhaseSel {
  uint64_t kmin, kmax;  // ordered-key range of the first keys
  uint64_t T;           // candidates: first key <= T (0: none)
  uint32_t n_elig;      // clients with an eligible first key
  uint32_t hshift;      // histogram bin of key k: hist_bin(k, hmin, hshift)
  uint32_t tbin;        // histogram bin holding T (last bin of the table)
  uint32_t valid;       // kSelValid once the pick wrote it (k_rscan zeroes it)
  uint64_t hmin;        // histogram base (histogram coordinates, KeyMap)
  uint64_t lo0, hitop;  // coordinate span of the open-ended first / last bin
  double vmin, scale;   // the phase's KeyMap (with kmin)
  double inv_w, inv_last;  // rank_bin_r's split scales (interior / last bin)
};

// Histogram range of a phase: base key and bin shift (bins 0 and
// kHistBinsR - 1 are open-ended).
struct HistRange {
  uint64_t hmin;
  uint32_t shift;
  uint32_t pad;
};

struct RoundPart {  // per-block partials of k_rscan
  uint32_t cnt[2];
  uint64_t n_r;
  uint64_t mn[2], mx[2];
};

// Round state (device resident).
struct Round {
  PhaseSel ph[2];
  uint64_t n_r;          // entries in all R prefixes
  uint32_t k_total;      // pulls requested
  uint32_t p_runs;       // the R prefixes hold fewer than k_total entries
  uint32_t bin_ovf;      // a rank bin outgrew kBinCapR
  uint32_t dense_n;      // radix path: dense entries emitted
  uint32_t n_dec;        // decisions of the round
  uint32_t n_prio;       // priority pops (= applied P groups)
  uint32_t g_last;       // decision index of the last applied P group's pop
  uint32_t terminal;     // eligible work ran out before k_total
  uint32_t overflow;     // 1: dense capacity, 2: rank bin (retry on radix)
  uint32_t next_type;    // DMC_NEXT_* of the stopping pull (terminal)
  double when;
  unsigned long long rsv0[2];  // (unused)
  uint32_t n_cand;       // candidate clients (k_rcand)
  uint32_t n_pgroups;    // P groups emitted (k_rbscan)
  uint32_t n_emit;       // rank records emitted (k_rbscan)
  uint32_t sampled;      // the thresholds came from a 1/8 sample of the first keys
  uint32_t brk;          // a limit-break round (AtLimit::Allow after the eligible
                         // work ran out: walk_p's brk groups)
  uint32_t brk_bad;      // ... whose state was not break-ready (overflow = 5)
  uint32_t brk_prio;     // ... its priority pops (counted by k_rapply)
  uint32_t brk_done;     // ... k_rapply's block ticket (the summary goes last)
  uint32_t ccnt[2 * kCntShards];  // sampled rounds: first keys at or below T, per
                               // phase, in XCD shards (k_remit)
  uint32_t bin_max[2];   // diagnostics: largest rank bin per phase
  uint32_t ecnt[4];      // diagnostics: candidates fast / several records /
                         // one P group with a run / other slow (k_remit)
  unsigned long long bin_sq;  // diagnostics: sum of squared bin counts
  RoundPart tot;         // reduced scan partials (k_rreduce)
  // diagnostics (DMC_TAIL_TIMING builds): wall clocks of the kernels with a
  // last-block tail: [0] first k_rhist block start, [1] its last block's
  // ticket, [2] pick done; [3] first k_remit block start, [4] its last
  // block's ticket, [5] bin prefixes done
  unsigned long long tdbg[12];  // [6..8] pick steps, [9..11] bin_prefix steps
  // per-call parameters, published by k_rscan (the graph's parameter node)
  double now;
  dmc_decision* out;
  uint64_t tick;
  dmc_pull_result* res;  // device-API result record (null: the host writes it)
  uint64_t seq;          // round sequence number, published to the host
  uint32_t fault;        // test hook (CallParams::fault)
  uint32_t skip;         // this round's kernels do nothing (its k_rscan found the gate shut)
  uint32_t* gate;        // a pipelined round: its end sets the gate (CallParams::gate)
};

// A pipelined round ends its call (the host has nothing left to do for
// it): the gate stays open and the next call's queued kernels run.  One
// formula for its three readers -- the round's last block, which sets the
// gate (rfinish_body); a filing merged beside the round's apply, which
// cannot read the gate that launch writes (add_link_body); and the host's
// settle_pending -- so that they never disagree.  (A skipped round's apply
// never reaches rfinish_body: its gate stays shut.)
__host__ __device__ inline bool round_ends_call(const Round& r) {
  return !r.skip && !r.overflow && r.n_dec >= r.k_total;
}

struct CallParams {
  uint32_t k_total;
  uint32_t brk;  // a limit-break round
  double now;
  dmc_decision* out;
  uint64_t tick;
  dmc_pull_result* res;
  uint64_t seq;
  uint32_t fault;  // test hook (DMC_OPT_FAULT): 1 = phase 1's selection left unset
  uint32_t epoch;  // k_chain_scan: the slots stamped with it are the add chain's to scan
  uint32_t* gate;  // DMC_OPT_PIPELINE: a pipelined call's round (its end sets the gate)
};

// Host-mapped (fine-grained pinned) round summary: the round's last kernel
// copies Round here and then publishes seq, so the host learns the outcome
// by polling host memory instead of a device-to-host copy and a stream
// synchronisation (two command-processor round trips per call).  Two of
// them, by seq parity: with DMC_OPT_PIPELINE the next round may end while
// the host reads this one's.
struct HostRound {
  Round r;
  uint64_t seq;
};

__device__ inline uint64_t shfl_down_u64r(uint64_t v, int d) {
  uint32_t lo = __shfl_down((uint32_t)v, d), hi = __shfl_down((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t wmin64(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1) {
    uint64_t o = shfl_down_u64r(v, d);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline uint64_t wmax64(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1) {
    uint64_t o = shfl_down_u64r(v, d);
    v = o > v ? o : v;
  }
  return v;
}
__device__ inline uint64_t wsum64(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1) v += shfl_down_u64r(v, d);
  return v;
}
__device__ inline uint32_t wsum32(uint32_t v) {
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
  return v;
}

struct CountV {
  uint32_t pops = 0, groups = 0;
  __device__ void pop(uint32_t, const Tag3&, uint32_t, uint64_t, uint32_t, uint32_t,
                      uint32_t) {
    ++pops;
  }
  __device__ void group(uint64_t, uint32_t) { ++groups; }
};

// ---------------------------------------------------------------- k_rscan
// Per slot: R key = front r if r <= now (its R prefix is walked for its
// length and, in delayed mode, the post-R front tag); P key = p + prop_delta of
// the post-R front if it is ready (flag, or limit <= now: the first priority
// pull's limit scan) and p < inf.  An untouched front that this scan would
// mark gets F_PMARK; k_rapply turns it into F_READY iff the priority pulls ran.
// Each thread takes kScanSlots slots and issues all their column loads before
// any walk; blocks of kScanBlock threads, so that the per-block partials
// (counts, key ranges) stay few.
// (build-time overridable for launch-shape sweeps: results do not depend on them)
#ifndef DMC_SCAN_SLOTS
#define DMC_SCAN_SLOTS 1
#endif
#ifndef DMC_SCAN_BLOCK
#define DMC_SCAN_BLOCK 1024
#endif
constexpr int kScanSlots = DMC_SCAN_SLOTS;
constexpr int kScanBlock = DMC_SCAN_BLOCK;

// Sampled thresholds: for large tables the round's threshold histogram is
// built from every kSample-th slot's first keys (k_rscan writes them
// compactly), with a margin on the needed count; k_remit counts the exact
// first keys at or below each threshold and a round whose sampled threshold
// admits too few is re-run with the exact histogram (overflow = 3).
#ifndef DMC_SAMPLE
#define DMC_SAMPLE 8
#endif
constexpr uint32_t kSample = DMC_SAMPLE;  // (a power of two)
static_assert((kSample & (kSample - 1)) == 0, "kSample: a power of two");
constexpr uint32_t kSampleMinN = 1u << 16;

// k_remit's candidate test streams a 32-bit quantized first key per phase
// (the ordered key's top half, capped at 0xfffffffe; 0xffffffff: no key) and
// compares it with the threshold's; the pick rounds every finite threshold up
// to the end of its quantum (T | 0xffffffff: any T at or above the needed key
// is exact), so that key <= T  <=>  key32 <= T32 exactly.  (Finite and
// infinite keys have top halves <= 0xfff00000.)
__device__ inline uint32_t key32(uint64_t k) {
  if (k == kMaxKey) return 0xffffffffu;
  const uint32_t h = (uint32_t)(k >> 32);
  return h > 0xfffffffeu ? 0xfffffffeu : h;
}

struct ScanCols {
  uint32_t c, h;
  double fr, pk, fl;  // the front's heap keys (ScanRec)
  uint8_t f;
};

// A slot's first R prefix step, requested for all of a thread's slots
// before any of them is walked (immediate mode, front r <= now): queue
// position 1's tag and the client's prop_delta, one level of loads.
struct ScanPre {
  double r1, p1, l1, pd;
};

struct ScanOut {
  uint64_t kr, kp;
  uint32_t m;
  uint8_t f;
  bool mark;  // a pending limit-scan mark to store
};

// The slot's keys from its ScanRec columns (and, for an R prefix, its ring):
// no stores (scan_store makes them after every slot of the thread is done,
// since a load's wait also waits for the wave's earlier stores).
__device__ inline ScanOut scan_compute(const Table& tb, uint32_t s, const ScanCols& x,
                                       const ScanPre& pre, double now, bool brk = false,
                                       bool* bad = nullptr) {
  ScanOut o{kMaxKey, kMaxKey, 0, x.f, false};
  if (!x.c) return o;
  if (brk) {
    // a limit-break round: every front's key is its p + prop_delta (the
    // ready-heap order of not-ready fronts); the state must be the one the
    // eligible work left: no front with r <= now, none ready or with
    // l <= now, every p finite (else the host runs general pulls)
    if (x.fr <= now || x.fl <= now || (x.f & F_READY) || !(x.pk < kInf)) *bad = true;
    else o.kp = okey(x.pk);
    return o;
  }
  Tag3 pf;
  bool have_pf = true, ready;
  double pkv = kInf;
  if (x.fr <= now) {
    o.kr = okey(x.fr);
    double pd;
    uint32_t m;
    if (!tb.delayed) {
      // the front (r == fr) is in the prefix; position 1 was requested up
      // front, a longer prefix walks on from position 2
      pd = pre.pd;
      m = 1;
      if (m < x.c) {
        if (!(pre.r1 <= now)) {
          pf = Tag3{pre.r1, pre.p1, pre.l1, 0.0};
        } else {
          const ReqEntry* ring = tb.ring + (size_t)s * tb.q;
          m = 2;
          while (m < x.c) {
            const ReqEntry& e = ring[(x.h + m) & tb.qmask];
            if (!(e.r <= now)) {
              pf = Tag3{e.r, e.p, e.l, e.arrival};
              break;
            }
            ++m;
          }
        }
      }
    } else {
      CountV v;
      uint32_t fc;
      const CView cvx = load_view(tb, s);
      pd = cvx.pd;
      m = walk_r(tb, ring_view(tb, s, cvx.h), cvx, now, kMaxKey, 0xffffffffu, v,
                 nullptr, &pf, &fc);
    }
    o.m = m;
    have_pf = m < x.c;
    ready = pf.l <= now;
    // the post-R front's key, with the client's prop_delta
    if (have_pf && ready) pkv = __dadd_rn(pf.p, pd);
  } else {
    pkv = x.pk;
    ready = (x.f & F_READY) || x.fl <= now;
    if (!(x.f & F_READY) && x.fl <= now) {
      o.f = x.f | F_PMARK;
      o.mark = true;
    }
  }
  // p < inf iff p + prop_delta < inf (prop_delta is finite)
  if (have_pf && ready && pkv < kInf) o.kp = okey(pkv);
  return o;
}

__device__ inline uint32_t scan_meta(const ScanCols& x, const ScanOut& o) {
  return (o.m & 0xffu) | ((uint32_t)o.f << 8) | ((x.c ? x.h : 0u) << 16) | (x.c << 24);
}

__device__ inline void scan_store(const Table& tb, uint32_t s, const ScanCols& x,
                                  const ScanOut& o, uint64_t* keyr, uint64_t* keyp,
                                  uint32_t* meta, uint64_t* skr, uint64_t* skp,
                                  uint2* k32, RoundPart& acc) {
  const uint64_t kr = o.kr, kp = o.kp;
  const uint32_t m = o.m;
  if (o.mark) tb.sc[s].flags = o.f;
  if (keyr) {  // the exact histogram's keys (unsampled rounds)
    keyr[s] = kr;
    keyp[s] = kp;
  }
  k32[s] = make_uint2(key32(kr), key32(kp));
  if (skr && (s & (kSample - 1)) == 0) {  // the threshold histogram's sample
    skr[s / kSample] = kr;
    skp[s / kSample] = kp;
  }
  // the candidate record's fields for k_remit: R-prefix length, flags (with
  // a pending mark this scan set), ring head and count
  meta[s] = scan_meta(x, o);
  if (kr != kMaxKey) {
    ++acc.cnt[0];
    acc.n_r += m;
    acc.mn[0] = kr < acc.mn[0] ? kr : acc.mn[0];
    acc.mx[0] = kr > acc.mx[0] ? kr : acc.mx[0];
  }
  if (kp != kMaxKey) {
    ++acc.cnt[1];
    acc.mn[1] = kp < acc.mn[1] ? kp : acc.mn[1];
    acc.mx[1] = kp > acc.mx[1] ? kp : acc.mx[1];
  }
}

__device__ inline void rpart_combine(RoundPart& a, const RoundPart& b) {
  for (int p = 0; p < 2; ++p) {
    a.cnt[p] += b.cnt[p];
    a.mn[p] = b.mn[p] < a.mn[p] ? b.mn[p] : a.mn[p];
    a.mx[p] = b.mx[p] > a.mx[p] ? b.mx[p] : a.mx[p];
  }
  a.n_r += b.n_r;
}

__device__ inline RoundPart rpart_ident() {
  return RoundPart{{0, 0}, 0, {kMaxKey, kMaxKey}, {0, 0}};
}

// One wave's partials combined across its lanes on the DPP network (row
// shifts within 16-lane rows, then the row broadcasts of lanes 15 and 31):
// ALU steps instead of ds_bpermute round trips; the wave's result is in
// lane 63 (lanes a step has no source for receive the identity).
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline uint32_t rdpp32(uint32_t v, uint32_t idn) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)idn, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline uint64_t rdpp64(uint64_t v, uint64_t idn) {
  return ((uint64_t)rdpp32<CTRL, ROWS>((uint32_t)(v >> 32), (uint32_t)(idn >> 32)) << 32) |
         rdpp32<CTRL, ROWS>((uint32_t)v, (uint32_t)idn);
}
template <int CTRL, int ROWS>
__device__ __attribute__((always_inline)) inline void rpart_dpp_step(RoundPart& a) {
  RoundPart b;
  b.cnt[0] = rdpp32<CTRL, ROWS>(a.cnt[0], 0u);
  b.cnt[1] = rdpp32<CTRL, ROWS>(a.cnt[1], 0u);
  b.n_r = rdpp64<CTRL, ROWS>(a.n_r, 0ull);
  b.mn[0] = rdpp64<CTRL, ROWS>(a.mn[0], kMaxKey);
  b.mn[1] = rdpp64<CTRL, ROWS>(a.mn[1], kMaxKey);
  b.mx[0] = rdpp64<CTRL, ROWS>(a.mx[0], 0ull);
  b.mx[1] = rdpp64<CTRL, ROWS>(a.mx[1], 0ull);
  rpart_combine(a, b);
}
// the wave's inclusive prefix sum on the same network (lane i: lanes 0..i),
// and the wave's sum in every lane
// (against the shuffle loops of rounds 1-3: emit 27.0 vs 28.2 us, pick
// 6.8 vs 7.1, rank 12.2 vs 12.6, r04g)
__device__ __attribute__((always_inline)) inline uint32_t wscan_u32(uint32_t v) {
  v += rdpp32<0x111, 0xf>(v, 0u);
  v += rdpp32<0x112, 0xf>(v, 0u);
  v += rdpp32<0x114, 0xf>(v, 0u);
  v += rdpp32<0x118, 0xf>(v, 0u);
  v += rdpp32<0x142, 0xa>(v, 0u);
  v += rdpp32<0x143, 0xc>(v, 0u);
  return v;
}
__device__ __attribute__((always_inline)) inline uint32_t wsum_all(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wscan_u32(v), 63);
}
__device__ __attribute__((always_inline)) inline RoundPart wave_rpart_dpp(RoundPart a) {
  rpart_dpp_step<0x111, 0xf>(a);  // row_shr:1
  rpart_dpp_step<0x112, 0xf>(a);  // row_shr:2
  rpart_dpp_step<0x114, 0xf>(a);  // row_shr:4
  rpart_dpp_step<0x118, 0xf>(a);  // row_shr:8
  rpart_dpp_step<0x142, 0xa>(a);  // row_bcast:15 into rows 1 and 3
  rpart_dpp_step<0x143, 0xc>(a);  // row_bcast:31 into rows 2 and 3
  return a;
}

__device__ inline uint32_t hist_shift_r(uint64_t range) {
  // smallest shift with (range >> shift) < kHistBinsR
  uint32_t bits = range ? 64 - __clzll((long long)range) : 0;
  return bits > 11 ? bits - 11 : 0;
}

// Histogram coordinate of an ordered key: linear in the key's value over the
// phase's [kmin, kmax].  Ordered-key offsets are linear in the bit pattern,
// so a key range that straddles zero or spans binades (the negative
// proportion keys of activations, :957-969) would pile most keys into a few
// bins and the threshold would admit most clients.  Monotone non-decreasing
// in the key (every step rounds monotonically), which is all the selection
// and the rank bins need.  Used only for such ranges (the value map costs a
// binary search per threshold and piles the keys near `now` into fewer bins
// than the bit-pattern map does for a range of a few binades); scale == 0:
// ordered-key offsets (also for degenerate or non-finite ranges).
struct KeyMap {
  uint64_t kmin;
  double vmin, scale;
  __device__ KeyMap(uint64_t mn, uint64_t mx) : kmin(mn), vmin(0.0), scale(0.0) {
    const double a = from_okey(mn), b = from_okey(mx);
    const double r = __dsub_rn(b, a);
    const int ea = (int)((dbits(a) >> 52) & 0x7ff), eb = (int)((dbits(b) >> 52) & 0x7ff);
    const bool wide = (a < 0.0 && b > 0.0) || ea - eb > 12 || eb - ea > 12;
    if (wide && r > 0.0 && r < kInf) {
      const double sc = __ddiv_rn(0x1p62, r);
      if (sc < kInf) {
        vmin = a;
        scale = sc;
      }
    }
  }
  __device__ KeyMap(uint64_t mn, double vm, double sc) : kmin(mn), vmin(vm), scale(sc) {}
  __device__ uint64_t operator()(uint64_t k) const {
    if (k <= kmin) return 0;
    if (scale == 0.0) return k - kmin;
    const double x = __dmul_rn(__dsub_rn(from_okey(k), vmin), scale);
    return x < 0x1p63 ? (uint64_t)x : (1ull << 63);
  }
  // the largest ordered key in [kmin, kmax] whose coordinate is <= c
  // (value map: a search from the map's inverse at c + 1, which lands within
  // a few keys of the answer, galloping outwards to bracket it, then
  // bisection -- the same key a bisection of the whole range finds, in a
  // handful of map evaluations instead of ~64: one thread runs it while its
  // block waits, 8 us of k_remit's pick in config 4's straddling P ranges)
  __device__ uint64_t max_key_at(uint64_t c, uint64_t kmax) const {
    if ((*this)(kmax) <= c) return kmax;
    if (scale == 0.0) return kmin + c;  // < kmax here
    uint64_t lo = kmin, hi = kmax;  // (*this)(lo) <= c < (*this)(hi)
    {
      const double v = __dadd_rn(vmin, __ddiv_rn((double)c + 1.0, scale));
      uint64_t g = v == v ? okey(v) : lo + (hi - lo) / 2;
      g = g <= lo ? lo + 1 : g >= hi ? hi - 1 : g;
      if (g > lo && g < hi) {
        if ((*this)(g) <= c) {
          lo = g;
          for (uint64_t st = 1; hi - lo > st; st <<= 1) {
            const uint64_t t = lo + st;
            if ((*this)(t) <= c) {
              lo = t;
            } else {
              hi = t;
              break;
            }
          }
        } else {
          hi = g;
          for (uint64_t st = 1; hi - lo > st; st <<= 1) {
            const uint64_t t = hi - st;
            if ((*this)(t) <= c) {
              lo = t;
              break;
            }
            hi = t;
          }
        }
      }
    }
    while (hi - lo > 1) {
      const uint64_t mid = lo + (hi - lo) / 2;
      if ((*this)(mid) <= c) lo = mid;
      else hi = mid;
    }
#ifdef DMC_KEYMAP_CHECK
    {  // (check builds: the plain bisection of the whole range agrees)
      uint64_t l2 = kmin, h2 = kmax;
      while (h2 - l2 > 1) {
        const uint64_t mid = l2 + (h2 - l2) / 2;
        if ((*this)(mid) <= c) l2 = mid;
        else h2 = mid;
      }
      if (l2 != lo) printf("KEYMAP MISMATCH c=%llu fast=%llu bisect=%llu\n",
                           (unsigned long long)c, (unsigned long long)lo, (unsigned long long)l2);
    }
#endif
    return lo;
  }
};

// histogram bin of a coordinate (bins 0 and kHistBinsR - 1 are open-ended)
__device__ inline uint32_t hist_bin(uint64_t k, uint64_t hmin, uint32_t sh) {
  if (k <= hmin) return 0;
  uint64_t b = (k - hmin) >> sh;
  return b >= (uint64_t)kHistBinsR ? kHistBinsR - 1 : (uint32_t)b;
}

__device__ inline uint64_t sat_add_u64(uint64_t a, uint64_t b) {
  return a + b < a ? ~0ull : a + b;
}

// Scan.  Per-block counts and key ranges (parts), staged in LDS and combined
// by wave 0 (cross-lane shuffles are ds_bpermute round trips: 12 per level
// for a RoundPart, too many to run in every wave of the block).
// (DMC_SCAN_MINW waves per SIMD: 8 = two blocks per CU, at most 64 VGPRs)
#ifndef DMC_SCAN_MINW
#define DMC_SCAN_MINW 8
#endif
// (BRK: a limit-break round's scan, its own instantiation: the general
// scan sits at its 64-register bound.  T: threads per block; bid / nblk:
// the block's index and count among the scan's blocks.  TOUCHED: slots
// the running add batch files (Table::touch == the call's epoch) are left
// to the add chain, which scans each once its adds are in -- the scan then
// runs beside the add chain, k_chain_scan)
template <bool BRK, int T = kScanBlock, bool TOUCHED = false, int SL = kScanSlots>
__device__ __attribute__((always_inline)) inline void rscan_body_g(Table tb, uint64_t* keyr, uint64_t* keyp, uint32_t* meta, RoundPart* parts, Round* rd, CallParams cp, uint64_t* skr, uint64_t* skp, uint2* k32, uint32_t* hist, uint32_t bid, uint32_t nblk) {
  if (!DMC_EARLY_LOADS && tb.gate && *tb.gate) {
    if (bid == 0 && threadIdx.x == 0) rd->skip = 1u;
    return;
  }
  const uint32_t base = bid * T * SL + threadIdx.x;
  ScanCols x[SL];
  bool mine[SL];
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    uint32_t s = base + j * T;
    x[j].c = 0;
    mine[j] = s < tb.n;
    if (s < tb.n) {
      const ScanRec r = tb.sc[s];
      if (TOUCHED && (DMC_STAMP_SC ? r.stamp == (uint8_t)cp.epoch : tb.touch[s] == cp.epoch))
        mine[j] = false;  // (the add chain's)
      x[j].c = mine[j] ? r.count : 0;
      x[j].h = r.head;
      x[j].fr = r.r;
      x[j].pk = r.pk;
      x[j].fl = r.l;
      x[j].f = r.flags;
    }
  }
  // (DMC_OPT_PIPELINE: the host finishes the last call first; the gate word
  // requested with the slots' records)
  if (DMC_EARLY_LOADS && tb.gate && *tb.gate) {
    if (bid == 0 && threadIdx.x == 0) rd->skip = 1u;
    return;
  }
  if (bid == 0 && threadIdx.x == 0) {
    Round z{};
    z.fault = cp.fault;
    z.k_total = cp.k_total;
    z.brk = cp.brk;
    z.g_last = kNoneR;
    z.next_type = DMC_NEXT_RETURNING;
    z.now = cp.now;
    z.out = cp.out;
    z.tick = cp.tick;
    z.res = cp.res;
    z.seq = cp.seq;
    z.gate = cp.gate;
    z.tdbg[0] = z.tdbg[3] = ~0ull;
    *rd = z;
  }
  __shared__ RoundPart sh[T];
  const double now = cp.now;
  RoundPart acc = rpart_ident();
  // every slot's first R prefix step in one level of loads
  ScanPre pre[SL];
  constexpr bool brk = BRK;
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    uint32_t s = base + j * T;
    pre[j] = ScanPre{0.0, 0.0, 0.0, 0.0};
    // (prop_delta only for a post-R front: a queue of one has none)
    if (mine[j] && x[j].c > 1 && x[j].fr <= now && !tb.delayed && !brk) {
      pre[j].pd = tb.rec[s].pd;
      {
        const ReqEntry& e = tb.ring[(size_t)s * tb.q + ((x[j].h + 1) & tb.qmask)];
        pre[j].r1 = e.r;
        pre[j].p1 = e.p;
        pre[j].l1 = e.l;
      }
    }
  }
  ScanOut o[SL];
  bool bad = false;  // a limit-break round's state is not break-ready
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    uint32_t s = base + j * T;
    o[j] = mine[j] ? scan_compute(tb, s, x[j], pre[j], now, brk, &bad)
                   : ScanOut{kMaxKey, kMaxKey, 0, 0, false};
  }
  // (a limit-break round has no reservation entries: its n_r counts the
  // slots that are not break-ready, for k_rhist's block 0)
  if (bad) acc.n_r += 1;
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    uint32_t s = base + j * T;
    if (mine[j])
      scan_store(tb, s, x[j], o[j], keyr, keyp, meta, skr, skp, k32, acc);
  }
  // (staged in LDS and combined by wave 0: reducing every wave's partials
  // on the DPP network first measured slower, 14.6 vs 14.3 us, r04g)
  sh[threadIdx.x] = acc;
  // the threshold histogram k_rhist fills, cleared (the previous round's
  // k_remit blocks have read it)
  {
    for (uint32_t gi = bid * T + threadIdx.x; gi < (uint32_t)(kShards * 2 * kHistBinsR);
         gi += nblk * T)
      hist[gi] = 0;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    RoundPart o = sh[threadIdx.x];
    for (int i = threadIdx.x + 64; i < T; i += 64) rpart_combine(o, sh[i]);
    o = wave_rpart_dpp(o);
    if (threadIdx.x == 63) parts[bid] = o;
  }
}
template <bool BRK>
__device__ __attribute__((always_inline)) inline void rscan_t_body(Table tb, uint64_t* keyr, uint64_t* keyp, uint32_t* meta, RoundPart* parts, Round* rd, CallParams cp, uint64_t* skr, uint64_t* skp, uint2* k32, uint32_t* hist) {
  rscan_body_g<BRK>(tb, keyr, keyp, meta, parts, rd, cp, skr, skp, k32, hist, blockIdx.x,
                    gridDim.x);
}

// a block's partials (T threads' acc) combined into parts[i]
template <int T>
__device__ inline void block_rpart_store(RoundPart acc, RoundPart* out) {
  __shared__ RoundPart sh[T];
  sh[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    RoundPart o = sh[threadIdx.x];
    for (int j = threadIdx.x + 64; j < T; j += 64) rpart_combine(o, sh[j]);
    o = wave_rpart_dpp(o);
    if (threadIdx.x == 63) *out = o;
  }
}

template <bool BRK>
__global__ void __launch_bounds__(kScanBlock, DMC_SCAN_MINW)
k_rscan_t(Table tb, uint64_t* keyr, uint64_t* keyp, uint32_t* meta,
          RoundPart* parts, Round* rd, CallParams cp, uint64_t* skr, uint64_t* skp,
          uint2* k32, uint32_t* hist) {
  rscan_t_body<BRK>(tb, keyr, keyp, meta, parts, rd, cp, skr, skp, k32, hist);
}

// the general scan (the graphs' parameter node) and the limit-break scan
constexpr auto k_rscan = k_rscan_t<false>;
constexpr auto k_rscan_brk = k_rscan_t<true>;

// The round's totals from the scan's per-block partials (every thread gets
// them).  Wide (default): every thread of the block loads its share (one
// round trip for up to blockDim partials), each wave reduces on the DPP
// network, wave 0 combines the waves'.  Narrow (rounds 1-3, A/B): wave 0
// alone, four partials per lane in flight (four round trips for 1024).
#ifndef DMC_RPARTS_WIDE
#define DMC_RPARTS_WIDE 1
#endif
__device__ inline RoundPart reduce_rparts(const RoundPart* parts, uint32_t nparts) {
  __shared__ RoundPart sh_tot;
#if DMC_RPARTS_WIDE
  __shared__ RoundPart sh_w[1024 / 64];
  RoundPart o = rpart_ident();
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x) rpart_combine(o, parts[i]);
  o = wave_rpart_dpp(o);
  if ((threadIdx.x & 63) == 63) sh_w[threadIdx.x >> 6] = o;
  __syncthreads();
  if (threadIdx.x < 64) {
    RoundPart x = threadIdx.x < (blockDim.x >> 6) ? sh_w[threadIdx.x] : rpart_ident();
    x = wave_rpart_dpp(x);
    if (threadIdx.x == 63) sh_tot = x;
  }
#else
  if (threadIdx.x < 64) {
    RoundPart o = rpart_ident();
    uint32_t i = threadIdx.x;
    for (; i + 3 * 64 < nparts; i += 4 * 64) {
      const RoundPart a = parts[i], b = parts[i + 64], c = parts[i + 128], d = parts[i + 192];
      rpart_combine(o, a);
      rpart_combine(o, b);
      rpart_combine(o, c);
      rpart_combine(o, d);
    }
    for (; i < nparts; i += 64) rpart_combine(o, parts[i]);
    o = wave_rpart_dpp(o);
    if (threadIdx.x == 63) sh_tot = o;
  }
#endif
  __syncthreads();
  RoundPart r = sh_tot;
  __syncthreads();
  return r;
}

// Histograms of both phases' first keys over their exact [kmin, kmax]:
// kHistBlocksR blocks of 1024 threads, 4 consecutive slots per thread and
// iteration with every key load issued before the first LDS atomic; the
// block's bins flush into shard block % kShards.
constexpr int kHistBlocksR = 256;
// queue groups' rounds: the thresholds and rank-bin tables picked once per
// table (k_rpick_m) instead of by every k_remit_m block; single-table rounds
// keep the pick in k_remit, whose 256 blocks run it beside their key loads
// (a pick in k_rhist's last block made it 14-17 µs for 3 µs less emit, r04ab)
#ifndef DMC_PRE_PICK_M
#define DMC_PRE_PICK_M 1
#endif
constexpr bool kPrePickM = DMC_PRE_PICK_M != 0;
#ifndef DMC_HIST_BLOCKS
#define DMC_HIST_BLOCKS 32
#endif
constexpr int kHistBlocksSampled = DMC_HIST_BLOCKS;  // 131,072 sampled slots of 1M: 4 per thread
                                        // (16 and 64 blocks measured no faster)

// Threshold and rank-bin table of one phase, by one half (kPickHalf
// threads) of a k_remit block (every block, from the same histogram: the
// same result); the other half does the other phase at the same time (the
// block barriers line up: both halves run this code).
// T: the largest key of the bin holding the need-th first key (any T at or
// above the k-th smallest entry key is exact; a bin edge only admits extra
// candidates).  The phase's kNBPhase rank bins are spread over the
// histogram bins up to T's bin in proportion to their counts (each gets 1 +
// its share), so that the rank bins stay small however the keys are
// distributed.  Table entry: first rank bin | rank bins << 16.
// k_remit's block size (1024: the measured best; 512 and 256 build and pass
// the same parity): pick_both splits it into two halves, one per phase, each
// taking kBinsPerThreadR histogram bins per thread.  Everything the pick
// writes (both phases' PhaseSel, both rank-bin tables) is a function of the
// block size, so no variant leaves a phase unset.
#ifndef DMC_EMIT_THREADS
#define DMC_EMIT_THREADS 1024
#endif
constexpr int kEmitThreads = DMC_EMIT_THREADS;
static_assert(kEmitThreads == 256 || kEmitThreads == 512 || kEmitThreads == 1024,
              "k_remit blocks of 256, 512 or 1024 threads");
constexpr int kPickHalf = kEmitThreads / 2;
static_assert(kEmitThreads == 2 * kPickHalf && kPickHalf % 64 == 0 &&
                  kHistBinsR % kPickHalf == 0 && (kPickHalf & (kPickHalf - 1)) == 0,
              "pick_both: two power-of-two halves of whole waves, one per phase");
constexpr int kBinsPerThreadR = kHistBinsR / kPickHalf;
// PhaseSel::valid of a phase the pick wrote (k_rrank fails a round whose
// selections are not both written: DMC_EDEVICE, never a short dispatch)
constexpr uint32_t kSelValid = 0x5e1ec7edu;
// (trail: a barrier after the reads, for a caller that reuses wsum; the
// pick gives each of its scans its own words instead)
#ifndef DMC_PICK_LEAN
#define DMC_PICK_LEAN 1
#endif
// (DMC_PICK_ONESCAN=1: the rank-bin table from the first scan's prefixes,
// no second scan: emit 26.8-27.3 and rank 10.9-11.0 against 26.6 and
// 10.6-10.7 us, r05x -- its spread is worse)
#ifndef DMC_PICK_ONESCAN
#define DMC_PICK_ONESCAN 0
#endif
__device__ inline uint32_t half_excl_scan(uint32_t v, uint32_t* wsum, bool trail = true) {
  const int t = threadIdx.x & (kPickHalf - 1), lane = t & 63, w = t >> 6;
  const uint32_t incl = wscan_u32(v);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int i = 0; i < w; ++i) wbase += wsum[i];
  if (trail) __syncthreads();
  return wbase + incl - v;
}

// The same for a pair of counts (the histogram's keys and non-empty bins),
// with the half's total of the first (wsum: 2 x kPickHalf / 64 words)
__device__ inline void half_excl_scan2(uint32_t v, uint32_t z, uint32_t* wsum, uint32_t* ev,
                                       uint32_t* ez, uint32_t* tv, bool trail = true) {
  constexpr int NW = kPickHalf / 64;
  const int t = threadIdx.x & (kPickHalf - 1), lane = t & 63, w = t >> 6;
  const uint32_t iv = wscan_u32(v), iz = wscan_u32(z);
  if (lane == 63) {
    wsum[w] = iv;
    wsum[NW + w] = iz;
  }
  __syncthreads();
  uint32_t bv = 0, bz = 0, tt = 0;
  for (int i = 0; i < NW; ++i) {
    if (i < w) {
      bv += wsum[i];
      bz += wsum[NW + i];
    }
    tt += wsum[i];
  }
  if (trail) __syncthreads();
  *ev = bv + iv - v;
  *ez = bz + iz - z;
  *tv = tt;
}

// (s_sel: tb, C, nz, found -- T's histogram bin, the keys and the non-empty
// bins up to it, whether the need-th key was found; s_def: C and nz up to
// the default tb, the top bin)
// (hv: this thread's kBinsPerThreadR bins, loaded by pick_load ahead of the
// caller's other loads)
// (debug, DMC_PICK_CLOCKS: k_remit's block clocks [5, 10) inside the pick)
#ifndef DMC_PICK_CLOCKS
#define DMC_PICK_CLOCKS 0
#endif
constexpr int kEClk = DMC_PICK_CLOCKS ? 10 : 5;  // k_remit block clocks per block
__device__ inline void pclock(uint64_t* pc, int i) {
  if (DMC_PICK_CLOCKS && pc && threadIdx.x == 0) pc[i] = wall_clock64();
}
struct PickBins {
  uint32_t h[kBinsPerThreadR];
};
__device__ inline PickBins pick_load(const uint32_t* hist) {
  const int t = threadIdx.x & (kPickHalf - 1), p = threadIdx.x / kPickHalf;
  const uint32_t* hp = hist + p * kHistBinsR;  // shard i at hp + i * 2 * kHistBinsR
  PickBins b;
  if (kShards == 1 && kBinsPerThreadR == 4) {
    const uint4 x = ld_as<uint4>(hp + 4 * t);
    b.h[0] = x.x;
    b.h[1] = x.y;
    b.h[2] = x.z;
    b.h[3] = x.w;
  } else {
#pragma unroll
    for (int j = 0; j < kBinsPerThreadR; ++j) {
      b.h[j] = 0;
#pragma unroll
      for (int i = 0; i < kShards; ++i) b.h[j] += hp[i * 2 * kHistBinsR + t * kBinsPerThreadR + j];
    }
  }
  return b;
}
// one phase's totals (selected from a RoundPart without indexing it: the
// caller may hold the RoundPart in registers)
struct PhaseTot {
  uint32_t cnt;
  uint64_t mn, mx;
};
__device__ inline void pick_phase(int p, uint32_t need, uint32_t need_h,
                                  const PhaseTot& tot, const KeyMap& km, uint32_t sh1,
                                  const PickBins& hv, uint32_t* sbn, PhaseSel* ps,
                                  uint32_t* wsum, uint32_t* s_sel, uint32_t* s_def,
                                  uint64_t* s_T, uint64_t* pc = nullptr) {
  const int t = threadIdx.x & (kPickHalf - 1);
  const uint32_t ne = tot.cnt;
  const uint64_t hmin = 0;
  // the default: every key (T = all, or none) up to the top bin
  const uint32_t tb0 = ne ? hist_bin(km(tot.mx), hmin, sh1) : 0;
  if (t == 0) {
    s_sel[3] = 0;
    *s_T = (need == 0 || ne == 0) ? 0 : kMaxKey - 1;
  }
  uint32_t h[kBinsPerThreadR];
  uint32_t local = 0, lz = 0;
#pragma unroll
  for (int j = 0; j < kBinsPerThreadR; ++j) {
    h[j] = hv.h[j];
    local += h[j];
    lz += h[j] ? 1u : 0u;
  }
  if (DMC_PICK_CLOCKS) asm volatile("" ::"v"(local));
  pclock(pc, 7);
  uint32_t before, zbefore, total;
  half_excl_scan2(local, lz, wsum, &before, &zbefore, &total, !DMC_PICK_LEAN);
  pclock(pc, 8);
  if (need && ne > need && before < need_h && before + local >= need_h) {
    uint32_t cum = before, cz = zbefore;
#pragma unroll
    for (int j = 0; j < kBinsPerThreadR; ++j) {
      cum += h[j];
      cz += h[j] ? 1u : 0u;
      if (cum >= need_h) {
        // the bin's upper edge: the largest key mapped into it, the same
        // candidate set as its largest key present (the open-ended last
        // bin: the largest key)
        uint32_t b = t * kBinsPerThreadR + j;
        uint64_t edge = b == kHistBinsR - 1
                            ? tot.mx
                            : km.max_key_at(sat_add_u64(hmin, ((uint64_t)(b + 1) << sh1) - 1),
                                            tot.mx);
        // (rounded up to the end of its 32-bit quantum: see key32)
        *s_T = edge >= kMaxKey - 1 ? kMaxKey - 1 : (edge | 0xffffffffull);
        s_sel[0] = b;
        s_sel[1] = cum;
        s_sel[2] = cz;
        s_sel[3] = 1;
        break;
      }
    }
  }
  if ((uint32_t)t == tb0 / kBinsPerThreadR) {
    uint32_t cum = before, cz = zbefore;
#pragma unroll
    for (int j = 0; j < kBinsPerThreadR; ++j) {
      if ((uint32_t)(t * kBinsPerThreadR + j) <= tb0) {
        cum += h[j];
        cz += h[j] ? 1u : 0u;
      }
    }
    s_def[0] = cum;
    s_def[1] = cz;
  }
  __syncthreads();
  pclock(pc, 9);
  const bool found = s_sel[3] != 0;
  const uint32_t tb = found ? s_sel[0] : tb0;
  const uint32_t C0 = found ? s_sel[1] : s_def[0];
  const uint32_t nz = found ? s_sel[2] : s_def[1];
  (void)total;
  const uint32_t C = C0 > 0 ? C0 : 1;
  // Every non-empty histogram bin up to T's gets one rank bin, and the
  // spare ones go in proportion to the counts, h * S / C in single precision
  // (any split is correct; only the balance depends on it), each clipped to
  // S so that the phase cannot pass its kNBPhase rank bins.  An empty bin
  // gets none: its keys (a sample's empty bin may hold a few) share the next
  // bin's first rank bin, which keeps the map monotone.
  const uint32_t S = kNBPhase > nz ? kNBPhase - nz : 0;
  const float q = (float)S / (float)C;
#if DMC_PICK_ONESCAN
  // (one scan: bin b's first rank bin is the non-empty bins before it plus
  // floor(the keys before it x S / C) -- both prefixes are the first scan's,
  // so no second scan; monotone, one rank bin at least per non-empty bin,
  // the spare ones in proportion to the counts as above; bins past T's are
  // never looked up, rank_bin_r clamps to the table's last bin)
  {
    uint32_t cb = before, cz = zbefore;
#pragma unroll
    for (int j = 0; j < kBinsPerThreadR; ++j) {
      const uint32_t b = t * kBinsPerThreadR + j;
      const uint32_t f0 = cz + (uint32_t)((float)cb * q);
      cb += h[j];
      cz += h[j] ? 1u : 0u;
      const uint32_t f1 = cz + (uint32_t)((float)cb * q);
      uint32_t first = f0, num = (b <= tb && h[j]) ? f1 - f0 : 0u;
      if (b > tb || first >= (uint32_t)kNBPhase) {
        first = kNBPhase - 1;
        num = num ? 1 : 0;
      } else if (first + num > (uint32_t)kNBPhase) {
        num = kNBPhase - first;
      }
      sbn[p * kHistBinsR + b] = (p * kNBPhase + first) | (num << 16);
    }
  }
#else
  uint32_t ns[kBinsPerThreadR], lns = 0;
#pragma unroll
  for (int j = 0; j < kBinsPerThreadR; ++j) {
    const uint32_t b = t * kBinsPerThreadR + j;
    uint32_t e = (uint32_t)((float)h[j] * q);
    e = e > S ? S : e;
    ns[j] = (b <= tb && h[j]) ? 1u + e : 0u;
    lns += ns[j];
  }
  uint32_t nb = half_excl_scan(lns, DMC_PICK_LEAN ? wsum + 2 * (kPickHalf / 64) : wsum,
                               !DMC_PICK_LEAN);
#pragma unroll
  for (int j = 0; j < kBinsPerThreadR; ++j) {
    const uint32_t b = t * kBinsPerThreadR + j;
    // float rounding may overshoot S by a few bins in all: the tail bins
    // are folded into the phase's last rank bin (monotone, still exact)
    uint32_t first = nb, num = ns[j];
    if (first >= (uint32_t)kNBPhase) {
      first = kNBPhase - 1;
      num = num ? 1 : 0;
    } else if (first + num > (uint32_t)kNBPhase) {
      num = kNBPhase - first;
    }
    sbn[p * kHistBinsR + b] = (p * kNBPhase + first) | (num << 16);
    nb += ns[j];
  }
#endif
  if (t == 0) {
    PhaseSel z{};
    z.kmin = tot.mn;
    z.kmax = tot.mx;
    z.T = *s_T;
    z.n_elig = ne;
    z.hshift = sh1;
    z.tbin = tb;
    z.hmin = hmin;
    z.lo0 = hmin;
    const uint64_t cmax = km(tot.mx);
    const uint64_t top = sat_add_u64(hmin, (uint64_t)(kHistBinsR - 1) << sh1);
    z.hitop = cmax > top ? cmax : top;
    z.vmin = km.vmin;
    z.scale = km.scale;
    // the rank-bin split inside a histogram bin (rank_bin_r): the interior
    // bins are 2^shift wide (an exact power-of-two scale); the open-ended
    // last bin spans [top, hitop]
    z.inv_w = bitsd((uint64_t)(1023 - sh1) << 52);
    z.inv_last = 1.0 / ((double)(z.hitop - top) + 1.0);
    z.valid = kSelValid;
    *ps = z;
  }
}

// Thresholds and rank-bin tables of both phases, by a k_remit block of
// kEmitThreads threads: phase 0 in threads [0, kPickHalf), phase 1 in
// [kPickHalf, kEmitThreads).
// needed first keys -> histogram units: exact, or for a 1/kSample sample
// need / kSample plus a margin of 2 % + 4 standard deviations + 16 (a
// sampled threshold admitting fewer than `need` first keys is caught by
// k_remit's exact count and the round re-run exactly)
// (sampled == 2, a test mode: 3 % below the expected count, so that
// validation fails and rounds are re-run)
__device__ inline uint32_t need_hist(uint32_t need, int sampled) {
  if (!sampled || need == 0xffffffffu) return need;
  const double m = (double)need / kSample;
  const double v = sampled == 2 ? m * 0.97 : m * 1.02 + 4.0 * __dsqrt_rn(m) + 16.0;
  return v >= 4294967295.0 ? 0xffffffffu : (uint32_t)v;
}

// (sbn, ps: LDS; the results are complete after the last barrier inside)
__device__ void pick_both(uint32_t k, const RoundPart& tot, const PickBins& hv,
                          uint32_t* sbn, PhaseSel* ps, int sampled, uint32_t fault,
                          uint64_t* pc = nullptr) {
  __shared__ uint32_t wsum[2][3 * kPickHalf / 64];
  __shared__ uint32_t s_sel[2][4], s_def[2][2];
  __shared__ uint64_t s_T[2];
  const bool p_runs = tot.n_r < (uint64_t)k;
  const int p = threadIdx.x / kPickHalf;
  // R: all prefixes when they hold fewer than k entries; else every client
  // whose first key is at or below the k-th smallest first key's bucket
  // (each such client contributes at least one entry <= T).  P: the rest.
  const uint32_t need = p == 0 ? (p_runs ? 0xffffffffu : k)
                               : (p_runs ? k - (uint32_t)tot.n_r : 0);
  pclock(pc, 5);
  const PhaseTot pt{p ? tot.cnt[1] : tot.cnt[0], p ? tot.mn[1] : tot.mn[0],
                    p ? tot.mx[1] : tot.mx[0]};
  const KeyMap km(pt.mn, pt.mx);
  if (DMC_PICK_CLOCKS) asm volatile("" ::"v"(km.scale));
  pclock(pc, 6);
  pick_phase(p, need, need_hist(need, sampled), pt, km, hist_shift_r(km(pt.mx)), hv,
             sbn, &ps[p], wsum[p], s_sel[p], s_def[p], &s_T[p], pc);
  // test hook (DMC_OPT_FAULT 1): phase 1's selection left unset, as a pick
  // that misses a phase would leave it; k_rrank must fail the round (lean:
  // by the thread that wrote it, before the one barrier)
  if (DMC_PICK_LEAN && (fault & 1u) && threadIdx.x == kPickHalf) ps[1].valid = 0;
  __syncthreads();  // (ps, written by thread 0 of each half)
  if (!DMC_PICK_LEAN) {
    if ((fault & 1u) && threadIdx.x == 0) ps[1].valid = 0;
    __syncthreads();
  }
}

// The same pick by one wave per phase (wave 0: R, wave 1: P), 32 histogram
// bins per lane: the prefix sums are wave scans and the threshold's bin a
// ballot, so the only barrier is the one that publishes the result to the
// block (the half-block pick above has seven, its waves' key loads in
// flight between them).  Same arithmetic, the same PhaseSel and rank-bin
// table entry for entry.  Measured slower: emit 28.8-28.9 against 27.2-27.3
// us with the half-block pick (r05k, alternated on one box) -- one wave's
// 32 bins per lane in sequence cost more than the barriers saved; kept as
// DMC_PICK_WAVE=1 (its parity tested like the default's).
#ifndef DMC_PICK_WAVE
#define DMC_PICK_WAVE 0
#endif
constexpr int kWBins = kHistBinsR / 64;  // bins per lane
struct PickW {
  uint4 h[kWBins / 4];
  RoundPart tot;
};
// (waves 0 and 1 only; issued ahead of the caller's other loads)
__device__ inline PickW pick_load_w(const uint32_t* hist, const RoundPart* tot) {
  PickW b;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 2) {
    const uint32_t* hp = hist + w * kHistBinsR + lane * kWBins;
#pragma unroll
    for (int j = 0; j < kWBins / 4; ++j) {
      b.h[j] = ld_as<uint4>(hp + 4 * j);
#pragma unroll
      for (int i = 1; i < kShards; ++i) {
        const uint4 x = ld_as<uint4>(hp + i * 2 * kHistBinsR + 4 * j);
        b.h[j].x += x.x; b.h[j].y += x.y; b.h[j].z += x.z; b.h[j].w += x.w;
      }
    }
    b.tot = *tot;
  }
  return b;
}
__device__ inline void pick_wave(int p, uint32_t k, const PickW& hw, uint32_t* sbn,
                                 PhaseSel* ps, int sampled, uint32_t fault) {
  const uint32_t lane = threadIdx.x & 63;
  const RoundPart& tot = hw.tot;
  const bool p_runs = tot.n_r < (uint64_t)k;
  const uint32_t need = p == 0 ? (p_runs ? 0xffffffffu : k)
                               : (p_runs ? k - (uint32_t)tot.n_r : 0);
  const uint32_t need_h = need_hist(need, sampled);
  // (the phase's totals selected, not indexed: no private-memory array)
  const uint32_t ne = p ? tot.cnt[1] : tot.cnt[0];
  const uint64_t kmn = p ? tot.mn[1] : tot.mn[0], kmx = p ? tot.mx[1] : tot.mx[0];
  const KeyMap km(kmn, kmx);
  const uint32_t sh1 = hist_shift_r(km(kmx));
  const uint32_t tb0 = ne ? hist_bin(km(kmx), 0, sh1) : 0;
  uint32_t h[kWBins];
#pragma unroll
  for (int j = 0; j < kWBins / 4; ++j) {
    h[4 * j] = hw.h[j].x;
    h[4 * j + 1] = hw.h[j].y;
    h[4 * j + 2] = hw.h[j].z;
    h[4 * j + 3] = hw.h[j].w;
  }
  uint32_t local = 0, lz = 0;
#pragma unroll
  for (int j = 0; j < kWBins; ++j) {
    local += h[j];
    lz += h[j] ? 1u : 0u;
  }
  const uint32_t before = wscan_u32(local) - local, zbefore = wscan_u32(lz) - lz;
  // T's bin: the first whose inclusive count reaches need_h (one lane holds
  // the crossing: the prefix sums are monotone); else every key up to tb0
  const bool mine = need && ne > need && before < need_h && before + local >= need_h;
  const uint64_t fm = __ballot(mine);
  const bool found = fm != 0;
  const int sl = found ? __ffsll((unsigned long long)fm) - 1 : (int)(tb0 / kWBins);
  uint32_t cb = 0, cum = before, cz = zbefore;
  bool done = false;
#pragma unroll
  for (int j = 0; j < kWBins; ++j) {
    const uint32_t b = lane * kWBins + j;
    if (found ? !done : b <= tb0) {
      cum += h[j];
      cz += h[j] ? 1u : 0u;
      if (found && cum >= need_h) {
        cb = b;
        done = true;
      }
    }
  }
  const uint32_t tb = found ? (uint32_t)__builtin_amdgcn_readlane((int)cb, sl) : tb0;
  const uint32_t C0 = (uint32_t)__builtin_amdgcn_readlane((int)cum, sl);
  const uint32_t nz = (uint32_t)__builtin_amdgcn_readlane((int)cz, sl);
  uint64_t T = (need == 0 || ne == 0) ? 0 : kMaxKey - 1;
  if (found) {
    // the bin's upper edge (see pick_phase), rounded up to its quantum's end
    const uint64_t edge =
        tb == kHistBinsR - 1
            ? kmx
            : km.max_key_at(sat_add_u64(0, ((uint64_t)(tb + 1) << sh1) - 1), kmx);
    T = edge >= kMaxKey - 1 ? kMaxKey - 1 : (edge | 0xffffffffull);
  }
  // the rank-bin table (pick_phase's split)
  const uint32_t C = C0 > 0 ? C0 : 1;
  const uint32_t S = kNBPhase > nz ? kNBPhase - nz : 0;
  const float q = (float)S / (float)C;
  uint32_t lns = 0;
#pragma unroll
  for (int j = 0; j < kWBins; ++j) {
    const uint32_t b = lane * kWBins + j;
    uint32_t e = (uint32_t)((float)h[j] * q);
    e = e > S ? S : e;
    h[j] = (b <= tb && h[j]) ? 1u + e : 0u;  // (h now holds the rank-bin counts)
    lns += h[j];
  }
  uint32_t nb = wscan_u32(lns) - lns;
#pragma unroll
  for (int j = 0; j < kWBins / 4; ++j) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t first = nb, num = h[4 * j + u];
      if (first >= (uint32_t)kNBPhase) {
        first = kNBPhase - 1;
        num = num ? 1 : 0;
      } else if (first + num > (uint32_t)kNBPhase) {
        num = kNBPhase - first;
      }
      v[u] = (p * kNBPhase + first) | (num << 16);
      nb += h[4 * j + u];
    }
    st_as(sbn + p * kHistBinsR + lane * kWBins + 4 * j, make_uint4(v[0], v[1], v[2], v[3]));
  }
  if (lane == 0) {
    PhaseSel z{};
    z.kmin = kmn;
    z.kmax = kmx;
    z.T = T;
    z.n_elig = ne;
    z.hshift = sh1;
    z.tbin = tb;
    z.hmin = 0;
    z.lo0 = 0;
    const uint64_t cmax = km(kmx);
    const uint64_t top = (uint64_t)(kHistBinsR - 1) << sh1;
    z.hitop = cmax > top ? cmax : top;
    z.vmin = km.vmin;
    z.scale = km.scale;
    z.inv_w = bitsd((uint64_t)(1023 - sh1) << 52);
    z.inv_last = 1.0 / ((double)(z.hitop - top) + 1.0);
    // test hook (DMC_OPT_FAULT 1): phase 1's selection left unset
    z.valid = (p == 1 && (fault & 1u)) ? 0u : kSelValid;
    *ps = z;
  }
}
// (sbn, ps: LDS; complete after the barrier inside)
__device__ inline void pick_both_w(uint32_t k, const PickW& hw, uint32_t* sbn, PhaseSel* ps,
                                   int sampled, uint32_t fault) {
  const int w = threadIdx.x >> 6;
  if (w < 2) pick_wave(w, k, hw, sbn, &ps[w], sampled, fault);
  __syncthreads();
}

// n keys per phase: every slot's first keys (keyr / keyp, exact), or the
// scan's 1/kSample sample of them (sampled: 1, or 2 in the test mode of
// need_hist).  The histogram k_rscan cleared is complete at the kernel's end;
// every k_remit block picks the thresholds and rank bins from it (no block
// ticket, no last-block tail here).  Block 0 stores the round's totals.
__device__ __attribute__((always_inline)) inline void rhist_body(uint32_t n, const uint64_t* keyr, const uint64_t* keyp, const RoundPart* parts, uint32_t nparts, Round* rd, uint32_t* hist, int sampled, unsigned long long* bcount, unsigned long long* gsup) {
  if (!DMC_EARLY_LOADS && rd->skip) return;
  __shared__ uint32_t lh[2][kHistBinsR];

  for (int b = threadIdx.x; b < kHistBinsR; b += blockDim.x) {
    lh[0][b] = 0;
    lh[1][b] = 0;
  }
  // this thread's first keys are loaded before the totals are reduced (the
  // two latencies overlap); further iterations only when n > 4 x threads
  const uint32_t stride = gridDim.x * blockDim.x * 4;
  uint32_t s = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  uint64_t kr[4], kp[4];
  auto load = [&](uint32_t s0) {
    if (s0 + 4 <= n) {
      const ulonglong2 a = ld_as<ulonglong2>(keyr + s0), b = ld_as<ulonglong2>(keyr + s0 + 2),
                       c = ld_as<ulonglong2>(keyp + s0), d = ld_as<ulonglong2>(keyp + s0 + 2);
      kr[0] = a.x; kr[1] = a.y; kr[2] = b.x; kr[3] = b.y;
      kp[0] = c.x; kp[1] = c.y; kp[2] = d.x; kp[3] = d.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kr[j] = s0 + j < n ? keyr[s0 + j] : kMaxKey;
        kp[j] = s0 + j < n ? keyp[s0 + j] : kMaxKey;
      }
    }
  };
  if (s < n) load(s);
  // (the skip word requested with the keys: one level of loads)
  if (DMC_EARLY_LOADS && rd->skip) return;
  const RoundPart tot = reduce_rparts(parts, nparts);  // (its barriers order the zeroing)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the round's totals (a limit-break round has no reservation entries: its
    // scan's n_r counts the slots that are not break-ready)
    const bool brk_bad = rd->brk && tot.n_r;
    RoundPart t2 = tot;
    if (rd->brk) t2.n_r = 0;
    rd->tot = t2;
    rd->n_r = t2.n_r;
    rd->p_runs = t2.n_r < (uint64_t)rd->k_total ? 1 : 0;
    rd->sampled = (uint32_t)sampled;
    if (brk_bad) {
      // the state is not the one a limit-break round assumes: nothing of
      // the round takes effect, the host runs general pulls instead
      rd->brk_bad = 1;
      rd->overflow = 5;
    }
  }
  if (tot.cnt[0] != 0 || tot.cnt[1] != 0) {
    const KeyMap m0(tot.mn[0], tot.mx[0]), m1(tot.mn[1], tot.mx[1]);
    const uint32_t sh0 = hist_shift_r(m0(tot.mx[0]));
    const uint32_t sh1 = hist_shift_r(m1(tot.mx[1]));
    for (; s < n; s += stride) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kr[j] != kMaxKey) atomicAdd(&lh[0][hist_bin(m0(kr[j]), 0, sh0)], 1u);
        if (kp[j] != kMaxKey) atomicAdd(&lh[1][hist_bin(m1(kp[j]), 0, sh1)], 1u);
      }
      if (s + stride < n) load(s + stride);
    }
    __syncthreads();
    uint32_t* hs = hist + (blockIdx.x % kShards) * 2 * kHistBinsR;
    for (int b = threadIdx.x; b < kHistBinsR; b += blockDim.x) {
      if (lh[0][b]) atomicAdd(&hs[b], lh[0][b]);
      if (lh[1][b]) atomicAdd(&hs[kHistBinsR + b], lh[1][b]);
    }
  }
  // the rank-bin counters and super-bin sums k_remit fills, cleared (the
  // previous round's k_rrank has read them; last: a load's wait also waits
  // for the wave's earlier stores)
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (uint32_t)(kNBR + kNSup);
       i += gridDim.x * blockDim.x) {
    if (i < (uint32_t)kNBR) bcount[i] = 0ull;
    else gsup[i - kNBR] = 0ull;
  }
}
__global__ void __launch_bounds__(1024)
k_rhist(uint32_t n, const uint64_t* keyr, const uint64_t* keyp, const RoundPart* parts,
        uint32_t nparts, Round* rd, uint32_t* hist, int sampled,
        unsigned long long* bcount, unsigned long long* gsup) {
  rhist_body(n, keyr, keyp, parts, nparts, rd, hist, sampled, bcount, gsup);
}

// Rank bin of an entry key (monotone in the key): its histogram bin's share
// of the phase's rank bins (the pick's table: first rank bin | count << 16),
// split linearly over the bin's key span -- interior bins 2^shift wide, an
// exact power-of-two scale; the open-ended last bin up to the keys seen.
__device__ inline uint32_t rank_bin_r(uint64_t k, const PhaseSel& ps, int p,
                                      const uint32_t* sbn) {
  const uint64_t c = KeyMap(ps.kmin, ps.vmin, ps.scale)(k);
  uint32_t h = hist_bin(c, ps.hmin, ps.hshift);
  if (h > ps.tbin) h = ps.tbin;
  const uint32_t e = sbn[p * kHistBinsR + h];
  const uint32_t ns = e >> 16;
  uint32_t sub = 0;
  if (ns > 1) {
    const uint64_t lo = ps.hmin + ((uint64_t)h << ps.hshift);
    const uint64_t off = c > lo ? c - lo : 0;
    const double f = (double)off * (h == kHistBinsR - 1 ? ps.inv_last : ps.inv_w);
    sub = (uint32_t)(f * (double)ns);
    if (sub >= ns) sub = ns - 1;
  }
  return (e & 0xffffu) + sub;
}

// The rank bin of an entry key rounded down to its 32-bit quantum (key32):
// monotone in the key, and a candidate's first record -- whose key is the
// first key k_remit streams quantized -- gets its bin before its walk.
__device__ inline uint32_t rank_bin_q(uint64_t k, const PhaseSel& ps, int p,
                                      const uint32_t* sbn) {
  return rank_bin_r(k & 0xffffffff00000000ull, ps, p, sbn);
}

// Rank-bin record of one entry: the order key (phase by bin, okey, slot,
// queue position), the group's run (P) and the entry's ring index.  The
// decision offset and tie flag are written into the ring entry itself
// (ReqEntry::dec / ::tie), where k_rapply's walk reads them.
struct BKey {
  uint64_t okey;
  uint32_t slot;
  uint32_t seq;
  uint32_t run;
  uint32_t ridx;  // slot * q + ring index
};

// The record as k_remit writes it (one 64-byte line): the order key, then
// the candidate index and, for a *fast* record (kFastRec: its candidate's
// only record, a single pop at queue position 0, immediate mode), the pop's
// decision payload, which k_rrank writes straight to the decision array; a
// slow record's pop is stamped into its ring entry for k_rapply's re-walk.
constexpr uint32_t kFastRec = 0x80000000u;
struct BRecR {
  BKey k;
  uint32_t ci;  // candidate index | kFastRec
  uint32_t cost;
  uint64_t handle;
  double r, p, l;
};
static_assert(sizeof(BRecR) == 64, "BRecR must be one 64-byte line");

// A fast candidate's state after its pops (k_remit computes it from the
// walk; k_rapply stores it iff k_rrank dispatched the whole group): the new
// front's keys, the reduced prev r and the reduction offset (priority pop),
// queue position 2's reduced r (no run); and, for a priority pop followed by
// a one-pop reservation run, that pop's decision payload (second line).
// decof[ci]: kSlowCand (re-walk), kNoDec (not dispatched) or the first
// pop's decision offset.
constexpr uint32_t kSlowCand = 0xfffffffeu;
struct PostRec {
  double fr, fpk, fl;  // new front r, p + prop_delta, l (queue position 1 + run)
  double prev_r;       // prev r after the pop's reduction
  double off;          // reduce_reservation_tags offset (priority pop)
  double r2;           // queue position 2's reduced r (run 0)
  uint32_t bits;       // 1: priority pop, 2: the new front's l <= now, 4: run of one
  uint32_t cand;       // the candidate's CandRec word: flags (low nibble) | R-prefix
                       // length << 8 | ring head << 16 | queued count << 24
  uint32_t cost0;      // the first pop's cost (a queue group's tally, k_rapply_m)
  uint32_t pad;
  // the run's pop (queue position 1), bits & 4
  uint64_t handle1;
  double r1, p1, l1;
  uint32_t cost1;
  uint32_t pad1[7];
};
static_assert(sizeof(PostRec) == 128, "PostRec must be two 64-byte lines");
// (k_remit stores it in 16-byte pieces in this order)
static_assert(offsetof(PostRec, prev_r) == 24 && offsetof(PostRec, r2) == 40 &&
                  offsetof(PostRec, bits) == 48 && offsetof(PostRec, cand) == 52 &&
                  offsetof(PostRec, cost0) == 56 &&
                  offsetof(PostRec, handle1) == 64 && offsetof(PostRec, p1) == 80 &&
                  offsetof(PostRec, cost1) == 96,
              "PostRec layout");

// Dense entry (radix path).
struct DEnt {
  uint64_t okey;
  uint32_t slot;
  uint32_t seq;   // queue position | phase << 31
  uint32_t run;
  uint32_t ridx;  // slot * q + ring index
};

// What a candidate's walks emitted: its record count, the first record
// (held back until the walks end, when it is known whether the candidate is
// fast) and its first pop.
// (A fast candidate's pop is queue position 0, whose staged entry holds its
// decision payload: nothing of it is kept in registers through the walks.)
struct EmitAcc {
  uint32_t ci;
  uint32_t nrec = 0, npops = 0;
  uint32_t b0 = 0, at0 = kBinCapR;  // the first record's bin and place
  uint64_t key0 = 0;                // its key
  uint32_t run0 = 0;                // its run (P group)
  uint32_t pos0 = 0;                // the first pop's queue position
  bool prio0 = false;               // ... and kind
  bool pre = false;                 // b0 / at0 reserved before the walk
};

struct EmitV {
  int ph;
  uint32_t slot;
  const PhaseSel* ps;
  // bin-rank path
  BRecR* brec;
  uint32_t* bcount;
  unsigned long long* ssup;  // the block's super-bin sums (LDS)
  const uint32_t* sbn;  // the rank-bin table, staged in LDS
  Round* rd;
  // radix path
  DEnt* dense;
  uint32_t dcap;
  uint32_t rbase, head, qmask;  // ring index of queue position i
  EmitAcc* acc;
  __device__ void put(uint64_t key, uint32_t pos, uint32_t run) {
    uint32_t ridx = rbase + ((head + pos) & qmask);
    if (brec) {
      const uint32_t b = rank_bin_q(key, *ps, ph, sbn);
      unsigned long long* bc = reinterpret_cast<unsigned long long*>(bcount);
      if (acc->nrec == 0 && acc->pre) {
        // the first record: its place was reserved before the walk with a
        // group size of 1; a P group's run is added now (rare), and a bin
        // that differs from the reserved one (cannot happen: the same
        // quantized key) fails the round safely
        if (b != acc->b0) atomicOr(&rd->bin_ovf, 1u);
        if (ph == 1 && run) {
          atomicAdd(bc + b, (unsigned long long)run << 32);
          atomicAdd(&ssup[b / kSupBins], (unsigned long long)run << 32);
        }
        if (acc->at0 >= kBinCapR) atomicOr(&rd->bin_ovf, 1u);
        acc->key0 = key;
        acc->run0 = run;
        ++acc->nrec;
        return;
      }
      // one 64-bit atomic per record: the bin's record count in the low word,
      // its group sizes in the high word (bcount: kNBR 8-byte counters)
      const unsigned long long inc =
          ((unsigned long long)(ph == 0 ? 1u : 1u + run) << 32) | 1ull;
      const uint32_t at = (uint32_t)atomicAdd(bc + b, inc);
      atomicAdd(&ssup[b / kSupBins], inc);
      if (at >= kBinCapR) {
        atomicOr(&rd->bin_ovf, 1u);  // read by the last block (memory side)
      } else if (acc->nrec == 0) {
        acc->b0 = b;  // written by emit_one once the walks have ended
        acc->at0 = at;
        acc->key0 = key;
        acc->run0 = run;
      } else {
        // a second record: the candidate is slow (both go out now)
        if (acc->nrec == 1 && acc->at0 < kBinCapR) first_slow();
        brec[(size_t)b * kBinCapR + at] = BRecR{BKey{key, slot, pos, run, ridx}, acc->ci};
      }
      ++acc->nrec;
    } else {
      // wave-aggregated: one counter add per wave (massively tied rounds
      // emit every entry here; per-entry atomics on one address serialise)
      const uint64_t m = __ballot(1);
      const int lane = threadIdx.x & 63;
      const int leader = __ffsll((unsigned long long)m) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&rd->dense_n, (uint32_t)__popcll(m));
      base = __shfl(base, leader);
      const uint32_t at = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (at < dcap) dense[at] = DEnt{key, slot, pos | ((uint32_t)ph << 31), run, ridx};
    }
  }
  // the held-back first record, written as a slow one (its queue position
  // is the first pop's)
  __device__ void first_slow() {
    brec[(size_t)acc->b0 * kBinCapR + acc->at0] =
        BRecR{BKey{acc->key0, slot, acc->pos0, acc->run0,
                   rbase + ((head + acc->pos0) & qmask)},
              acc->ci};
  }
  uint32_t gpos = 0;
  __device__ void pop(uint32_t i, const Tag3& t, uint32_t, uint64_t, uint32_t kind,
                      uint32_t, uint32_t) {
    if (acc->npops++ == 0) {
      acc->pos0 = i;
      acc->prio0 = kind != kPopR;
    }
    if (ph == 0) put(okey(t.r), i, 0);
    else if (kind == kPopHead) gpos = i;
  }
  __device__ void group(uint64_t key, uint32_t run) { put(key, gpos, run); }
};

// A client is a candidate iff its first R key is <= T_R or (the priority
// pulls run and) its first P key is <= T_P.
// (the thresholds are read from LDS: wave-uniform, moved to scalar registers)
__device__ inline uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
struct CandPred {
  uint64_t TR, TP;  // 0: no candidates in that phase
  uint32_t TR32, TP32;
  __device__ CandPred(const PhaseSel* ph, bool p_runs)
      : TR(uniform_u64(ph[0].T)), TP(p_runs ? uniform_u64(ph[1].T) : 0),
        TR32(key32(TR) > 0xfffffffeu ? 0xfffffffeu : key32(TR)),
        TP32(key32(TP) > 0xfffffffeu ? 0xfffffffeu : key32(TP)) {}
  // exact: T is kMaxKey - 1 or the end of its quantum (see key32)
  __device__ bool operator()(uint32_t kr32, uint32_t kp32) const {
    return (TR && kr32 <= TR32) || (TP && kp32 <= TP32);
  }
};

// A candidate as compacted by k_remit: slot; flags (low nibble) and its
// first-key predicates (bit 4: R, bit 5: P); R-prefix length; ring head and
// count as k_rscan saw them (nothing changes them before k_rapply), so that
// the walkers request the ring entries together with the client record.
struct CandRec {
  uint32_t slot;
  uint8_t fb, m, h, c;
  __device__ uint8_t f() const { return fb & 0x0f; }
  __device__ bool cr() const { return (fb >> 4) & 1; }
  __device__ bool cp() const { return (fb >> 5) & 1; }
};
static_assert(sizeof(CandRec) == 8, "CandRec must be 8 bytes");

// The walkers' view of a candidate: head / count from its CandRec, the
// inverses and prop_delta from the table (one level of loads with the ring
// entries), cur_delta / cur_rho only in delayed mode.
__device__ inline CView cand_view(const Table& tb, const CandRec& cr) {
  const uint32_t s = cr.slot;
  CView v;
  v.h = cr.h;
  v.c = cr.c;
  v.cd = v.cr = 0;
  if (tb.delayed) {
    v.cd = tb.aux[s].cur_delta;
    v.cr = tb.aux[s].cur_rho;
  }
  v.rinv = tb.rec[s].r_inv;
  v.winv = tb.rec[s].w_inv;
  v.linv = tb.rec[s].l_inv;
  v.pd = tb.rec[s].pd;
  view_tag_info(tb, s, v);
  return v;
}

// One candidate's entries: R pops with r <= min(now, T_R); then, if the
// priority pulls run, the P groups with key <= T_P from the post-R state.
// Bin-rank path: into the rank bins; radix path: appended to the dense list.
#ifndef DMC_EMIT_STAGE
#define DMC_EMIT_STAGE 3
#endif
constexpr int kEmitStage = DMC_EMIT_STAGE;  // queue positions staged per walker (LDS; 2: no faster)
#ifndef DMC_EMIT_STAGE_THREADS
#define DMC_EMIT_STAGE_THREADS 448  // (LDS: 160 KB per block with the key array)
#endif
constexpr int kEmitStageThreads = DMC_EMIT_STAGE_THREADS;  // walkers with a staging slice
// (BRK: a limit-break round, its own instantiation of k_remit: the general
// walkers carry none of walk_p's break-mode code.  DL: the table's tag mode
// as a compile-time constant, 0 immediate, 1 delayed, -1 read from the table
// -- with it fixed, the walker's loads are one straight-line burst, and the
// compiler's wait counting sees no delayed-mode loads in flight across the
// candidate loop)
#ifndef DMC_EMIT_MODE_SPLIT
#define DMC_EMIT_MODE_SPLIT 1
#endif
#ifndef DMC_EMIT_PEEL
#define DMC_EMIT_PEEL 1
#endif
template <bool BRK, int DL = -1>
__device__ inline uint32_t emit_one(const Table& tb0, Round* rd, double now, const PhaseSel* ph,
                                const CandRec& c,
                                uint32_t ci, BRecR* brec, uint32_t* bcount,
                                unsigned long long* ssup,
                                const uint32_t* sbn, DEnt* dense, uint32_t dcap,
                                PostRec* post, uint32_t* decof,
                                ReqEntry* st, uint32_t key32_0, uint64_t* ck = nullptr) {
  // ck (debug): [0] entry, [1] client record and ring staged, [2] walks and
  // their rank records done
  Table tb = tb0;
  if (DL >= 0) tb.delayed = DL;
  if (ck) ck[0] = wall_clock64();
  const uint32_t s = c.slot;
  const uint64_t TR = uniform_u64(ph[0].T), TP = uniform_u64(ph[1].T);
  Tag3 pf;
  uint32_t fc;
  EmitAcc acc;
  acc.ci = ci;
#ifndef DMC_EMIT_PRERESERVE
#define DMC_EMIT_PRERESERVE 1
#endif
  // the first record's rank-bin place, reserved before the walk (its key is
  // the first key of the candidate's first phase, key32_0 is its quantum;
  // its bin comes from LDS alone).  DMC_EMIT_RESERVE_FIRST: the returning
  // atomic is issued ahead of the client record and ring loads, so that its
  // round trip overlaps theirs (on gfx950 vector memory results return in
  // issue order: the wait for the staged entries covers it); else after
  // them (round 5: a second dependent round trip per walker)
#ifndef DMC_EMIT_RESERVE_FIRST
#define DMC_EMIT_RESERVE_FIRST 1
#endif
  unsigned long long rsv = 0;  // the atomic's whole 64-bit result (below)
  auto reserve = [&]() {
    const int ph0 = c.cr() ? 0 : 1;
    acc.b0 = rank_bin_q((uint64_t)key32_0 << 32, ph[ph0], ph0, sbn);
    rsv = atomicAdd(reinterpret_cast<unsigned long long*>(bcount) + acc.b0,
                    (1ull << 32) | 1ull);
    atomicAdd(&ssup[acc.b0 / kSupBins], (1ull << 32) | 1ull);
    acc.pre = true;
  };
  if (DMC_EMIT_PRERESERVE && DMC_EMIT_RESERVE_FIRST && brec) reserve();
  // one level of loads: the staged ring entries, then the client record (a
  // wait for the record's fields is then a wait for the whole level)
  const StageLoads<kEmitStage> sl = stage_load<kEmitStage, true>(tb, s, c.h, c.c, st);
  const CView cv = cand_view(tb, c);
  const double prev_r = tb.rec[s].prev_r;  // (the inverses' line)
  const uint32_t h = cv.h;
  const RingView rv = stage_put<kEmitStage>(tb, s, h, sl, st);
  if (DMC_EMIT_PRERESERVE && !DMC_EMIT_RESERVE_FIRST && brec) reserve();
  // (both halves of the result stay live to here: a register of the
  // returning atomic reused before it returns would be a wait for it ahead
  // of the loads above; and the record's fields are waited for here on
  // every path, so that no load is in flight across the candidate loop's
  // back edge -- the compiler would otherwise wait for it, and everything
  // issued before it, ahead of the next candidate's loads)
  asm volatile("" ::"v"(rsv), "v"(prev_r), "v"(cv.rinv), "v"(cv.pd));
  if (acc.pre) acc.at0 = (uint32_t)rsv;
  if (ck) {
    keep(cv.rinv);
    keep(cv.pd);
    ck[1] = wall_clock64();
  }
  if (c.cr()) {
    EmitV v{0, s, &ph[0], brec, bcount, ssup, sbn, rd, dense, dcap,
            s * tb.q, h, tb.qmask, &acc};
    walk_r(tb, rv, cv, now, TR, 0xffffffffu, v, nullptr, &pf, &fc);
  }
  if (c.cp()) {
    // the priority pulls run only after every R pop
    const uint32_t m = c.m;
    bool ready0 = m == 0 && (c.f() & F_READY);
    EmitV v{1, s, &ph[1], brec, bcount, ssup, sbn, rd, dense, dcap,
            s * tb.q, h, tb.qmask, &acc};
    walk_p(tb, rv, cv, now, TP, 0xffffffffu, v, nullptr, nullptr, nullptr, m,
           pf, m && tb.delayed, ready0, 0, BRK);
  }
  // Fast candidate: one record at queue position 0 in immediate mode -- one
  // reservation pop, or a priority pop with a reservation run of at most one
  // pop.  Its first decision goes out with its record (k_rrank writes it);
  // its state after the group (apply_one's arithmetic for that case) and the
  // run's decision are stored here.
  const uint32_t run = acc.npops - 1;  // (a one-record candidate: its group's run)
  const bool fast = brec && !tb.delayed && !BRK && acc.nrec == 1 && acc.pos0 == 0 &&
                    acc.at0 < kBinCapR && (run == 0 || (run == 1 && acc.prio0));
  if (fast) {
    // (stored piecewise as computed: the record, then the PostRec's lines --
    // a whole PostRec and BRecR held in registers at once spill)
    const uint32_t cc = cv.c;
    const bool prio = acc.prio0;
    double off = 0.0;
    uint32_t cost0 = 0;
    {
      // the pop's payload: queue position 0 as stored (immediate mode: a
      // priority pop with no earlier one has its stored r)
      const ReqEntry e0 = rv.at(0);
      cost0 = e0.cost;
      if (prio) off = resv_offset(cv.rinv, e0.cost, e0.rho);
      brec[(size_t)acc.b0 * kBinCapR + acc.at0] =
          BRecR{BKey{acc.key0, s, 0u, run, s * tb.q + h}, ci | kFastRec, e0.cost, e0.handle,
                e0.r, e0.p, e0.l};
    }
    char* const dst = reinterpret_cast<char*>(post + ci);  // PostRec's 16-byte words
    {
      double fr = 0.0, fpk = 0.0, fl = 0.0, r2 = 0.0;
      uint32_t bits = (prio ? 1u : 0u) | (run ? 4u : 0u);
      if (cc >= 2 + run) {
        const ReqEntry ef = rv.at(1 + run);  // staged: 1 + run < kEmitStage
        fr = prio ? __dsub_rn(ef.r, off) : ef.r;
        fpk = __dadd_rn(ef.p, cv.pd);
        fl = ef.l;
        if (ef.l <= now) bits |= 2u;
      }
      if (prio && !run && cc >= 3) r2 = __dsub_rn(rv.r_at(2), off);
      const double pr_prev = prio ? __dsub_rn(prev_r, off) : prev_r;
      const uint32_t cw = (uint32_t)c.fb | ((uint32_t)c.m << 8) | ((uint32_t)c.h << 16) |
                          ((uint32_t)c.c << 24);
      // PostRec line 1: fr, fpk | fl, prev_r | off, r2 | bits, cand, pad
      st_as(dst, make_ulonglong2(dbits(fr), dbits(fpk)));
      st_as(dst + 16, make_ulonglong2(dbits(fl), dbits(pr_prev)));
      st_as(dst + 32, make_ulonglong2(dbits(off), dbits(r2)));
      st_as(dst + 48, make_ulonglong2((unsigned long long)bits | ((unsigned long long)cw << 32),
                                      (unsigned long long)cost0));
    }
    if (run) {
      // line 2, the run's pop: queue position 1 with its reduced r (its
      // decision tag): handle1, r1 | p1, l1 | cost1
      const ReqEntry e1 = rv.at(1);
      st_as(dst + 64, make_ulonglong2(e1.handle, dbits(__dsub_rn(e1.r, off))));
      st_as(dst + 80, make_ulonglong2(dbits(e1.p), dbits(e1.l)));
      st_as(dst + 96, make_ulonglong2((unsigned long long)e1.cost, 0ull));
      st_as(dst + 112, make_ulonglong2(0ull, 0ull));
    }
    decof[ci] = kNoDec;
  } else {
    if (brec && acc.nrec == 1 && acc.at0 < kBinCapR) {
      EmitV v{0, s, nullptr, brec, bcount, ssup, sbn, rd, dense, dcap, s * tb.q, h,
              tb.qmask, &acc};
      v.first_slow();
    }
    decof[ci] = kSlowCand;
  }
  if (ck) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ck[2] = wall_clock64();
  }
  return fast ? 0u : acc.nrec > 1 ? 1u : acc.npops > 1 ? 2u : 3u;
}

// ---------------------------------------------------------------- k_remit
// Candidate selection and emission in one pass over the client table:
// blocks of kEmitThreads own kEmitChunk consecutive slots, 4 per thread,
// with the first keys, R-prefix lengths, ring head / count and flags loaded
// coalesced.  A slot is a candidate iff its first R key is <= T_R or (the
// priority pulls run and) its first P key is <= T_P; non-candidates settle
// their pending limit-scan marks here (k_rapply settles the candidates').
// Each wave compacts its candidates (about 17 of its 256 slots in a
// config-3 round) into the block's list in LDS, at a base one LDS atomic
// hands it, and its lanes walk them at once, with the rank-bin table staged
// in LDS; a candidate's first record reserves its rank-bin place before its
// walk (rank_bin_q).  Bin-rank path: the last block to finish
// computes the rank-bin prefixes (k_rrank's offsets); radix path: entries go
// to the dense list.
#ifndef DMC_EMIT_PER
#define DMC_EMIT_PER 4
#endif
constexpr int kEmitPer = DMC_EMIT_PER;  // slots per thread (8 with 512-thread blocks: no faster)
static_assert(kEmitPer % 4 == 0 && kEmitPer <= 16, "kEmitPer: 4, 8 or 16 (the slot predicates: 2 bits each in a word)");
constexpr uint32_t kEmitChunk = kEmitThreads * kEmitPer;
// Queue groups (k_remit_m, with its k_rapply_m): 8 slots per thread, 8,192
// per block, and 128 staging walkers (LDS): a group's 8 x 2M-slot tables
// run 16 generations of one block per CU at 4 slots; at 8 each block's fixed
// costs are paid half as often (config 5 0.787-0.801 against 0.890-0.895
// ms/step).  A single table keeps 4: its 256 blocks fill the chip once.
#ifndef DMC_EMIT_PER_M
#define DMC_EMIT_PER_M 8
#endif
#ifndef DMC_EMIT_STAGE_THREADS_M
#define DMC_EMIT_STAGE_THREADS_M 128
#endif
constexpr int kEmitPerM = DMC_EMIT_PER_M;
static_assert(kEmitPerM % 4 == 0 && kEmitPerM <= 16, "kEmitPerM: 4, 8 or 16");
constexpr uint32_t kEmitChunkM = kEmitThreads * kEmitPerM;
constexpr int kEmitStageThreadsM = DMC_EMIT_STAGE_THREADS_M;
// walkers with a staging slice per wave: its first lanes (a wave with more
// candidates walks the rest from global memory)
constexpr int kEmitStageLanes0 = kEmitStageThreads / (kEmitThreads / 64);
constexpr int kEmitStageLanes = kEmitStageLanes0 < 64 ? kEmitStageLanes0 : 64;
// (the host sizes its grids, the apply blocks and the candidate buffers from
// kEmitChunk and kApplyPerEmit; pick_both from kEmitThreads)
// (4 waves per SIMD: at most 128 VGPRs, 16 waves per CU -- one 1024-thread
// block, or two 512-thread blocks when their LDS fits twice)
#ifndef DMC_EMIT_MINW
#define DMC_EMIT_MINW 4
#endif
template <bool BRK, bool PRE, int PER, int STH>
__device__ __attribute__((always_inline)) inline void remit_t_body(Table tb, Round* rd, const uint2* k32, const uint32_t* meta, CandRec* cand, uint32_t* bcand, PostRec* post, uint32_t* decof, BRecR* brec, uint32_t* bcount, unsigned long long* gsup, const uint32_t* hist, DEnt* dense, uint32_t dcap, uint64_t* eclk) {
  // (PER slots per thread, CH per block; STH walkers with a staging slice,
  // SL lanes of each wave)
  constexpr uint32_t CH = kEmitThreads * PER;
  constexpr int SL = STH / (kEmitThreads / 64) < 64 ? STH / (kEmitThreads / 64) : 64;
  if (!DMC_EARLY_LOADS && rd->skip) return;
  // eclk (debug): per block [0] start [1] keys + thresholds picked [2]
  // candidates compacted [3] walks done [4] block done
  if (eclk && threadIdx.x == 0) eclk[kEClk * blockIdx.x] = wall_clock64();
  __shared__ CandRec bl[CH];
  __shared__ uint32_t bk[CH];  // their first phase's quantized first key
  // each thread's slot predicates and flags, parked for the mark settling
  // after the walks (fewer registers live across them: no spills)
  __shared__ uint32_t s_fbits[kEmitThreads];
  __shared__ uint32_t s_fw[PER / 4][kEmitThreads];  // (flags, 4 slots a word)
  __shared__ uint32_t ltab[2 * kHistBinsR];
  __shared__ ReqEntry stage[STH * kEmitStage];
  __shared__ uint32_t s_tot;
  __shared__ uint32_t s_cnt[2], s_ec[4];
  __shared__ PhaseSel s_ph[2];
  __shared__ unsigned long long s_sup[kNSup];
  if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0;
  if (threadIdx.x < 4) s_ec[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_tot = 0;
  if (threadIdx.x < kNSup) s_sup[threadIdx.x] = 0;
#ifdef DMC_TAIL_TIMING
  if (threadIdx.x == 0) atomicMin(&rd->tdbg[3], (unsigned long long)wall_clock64());
#endif
  const uint32_t n = tb.n;
  const uint32_t s0 = blockIdx.x * CH + threadIdx.x * PER;
  // the pick's histogram bins first: its compute then waits for them only,
  // while the slots' keys below are still in flight
  // (PRE: the tables k_rpick_m picked, this thread's share)
  constexpr int kPT = 2 * kHistBinsR / 4 / kEmitThreads;
#if DMC_PICK_WAVE
  PickW hv;
#else
  PickBins hv;
#endif
  uint4 pt[kPT];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < kPT; ++j)
      pt[j] = ld_as<uint4>(hist + kShards * 2 * kHistBinsR + 4 * (threadIdx.x + j * kEmitThreads));
  } else {
#if DMC_PICK_WAVE
    hv = pick_load_w(hist, &rd->tot);
#else
    hv = pick_load(hist);
#endif
  }
  // the round's totals and call parameters, requested with the histogram
  // (the pick's first use of them is then no load level of its own)
  RoundPart tot_e;
  uint32_t k_e = 0, sampled_e = 0, fault_e = 0;
  const double now_e = rd->now;  // (the walkers' clock, requested here too)
  if constexpr (!PRE) {
    tot_e = rd->tot;
    k_e = rd->k_total;
    sampled_e = rd->sampled;
    fault_e = rd->fault;
  }
  if (DMC_EARLY_LOADS && rd->skip) return;
  const bool p_runs = rd->p_runs != 0;
  const int lane = threadIdx.x & 63;
  uint32_t kr[PER], kp[PER];  // 32-bit quantized first keys (key32)
  uint32_t mt[PER];  // k_rscan's meta: R-prefix length | flags << 8 | head << 16 | count << 24
  if (s0 + PER <= n) {
#pragma unroll
    for (int j = 0; j < PER / 2; ++j) {
      const uint4 a = ld_as<uint4>(k32 + s0 + 2 * j);
      kr[2 * j] = a.x; kp[2 * j] = a.y; kr[2 * j + 1] = a.z; kp[2 * j + 1] = a.w;
    }
#pragma unroll
    for (int j = 0; j < PER / 4; ++j) {
      const uint4 m = ld_as<uint4>(meta + s0 + 4 * j);
      mt[4 * j] = m.x; mt[4 * j + 1] = m.y; mt[4 * j + 2] = m.z; mt[4 * j + 3] = m.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      bool in = s0 + j < n;
      const uint2 k = in ? k32[s0 + j] : make_uint2(0xffffffffu, 0xffffffffu);
      kr[j] = k.x;
      kp[j] = k.y;
      mt[j] = in ? meta[s0 + j] : 0;
    }
  }
  // the thresholds and the rank-bin table, picked from the round's
  // histogram while the keys are in flight (its barriers also order the
  // zeroing of s_cnt / s_tot before any wave adds to them)
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < kPT; ++j) st_as(ltab + 4 * (threadIdx.x + j * kEmitThreads), pt[j]);
    if (threadIdx.x < 2) s_ph[threadIdx.x] = rd->ph[threadIdx.x];
    __syncthreads();  // (also orders the zeroing of s_cnt / s_tot)
  } else {
#if DMC_PICK_WAVE
    pick_both_w(rd->k_total, hv, ltab, s_ph, (int)rd->sampled, rd->fault);
#else
    pick_both(k_e, tot_e, hv, ltab, s_ph, (int)sampled_e, fault_e,
              eclk ? eclk + kEClk * blockIdx.x : nullptr);
#endif
    if (blockIdx.x == 0 && threadIdx.x < 2) rd->ph[threadIdx.x] = s_ph[threadIdx.x];  // (the summary)
  }
  const CandPred pred(s_ph, p_runs);
  if (eclk && threadIdx.x == 0) eclk[kEClk * blockIdx.x + 1] = wall_clock64();
  uint8_t f[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) f[j] = (uint8_t)(mt[j] >> 8);
  uint32_t bits = 0;  // per slot: bit 2j R predicate, bit 2j+1 P predicate
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (s0 + j >= n) continue;
    const bool cr = pred.TR && kr[j] <= pred.TR32;
    const bool cp = pred.TP && kp[j] <= pred.TP32;
    if (cr || cp) bits |= ((cr ? 1u : 0u) | (cp ? 2u : 0u)) << (2 * j);
  }
  uint32_t cnt = 0, nr = 0, np = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    cnt += ((bits >> (2 * j)) & 3u) ? 1u : 0u;
    nr += (bits >> (2 * j)) & 1u;
    np += (bits >> (2 * j + 1)) & 1u;
  }
  const bool sampled = rd->sampled != 0;
  if (sampled) {
    // the exact number of first keys at or below each threshold (validates
    // the sampled thresholds in the last block): per block, then one atomic
    // per phase into the block's XCD shard (same-address atomics serialise)
    nr = wsum_all(nr);
    np = wsum_all(np);
    if (lane == 0) {
      atomicAdd(&s_cnt[0], nr);
      atomicAdd(&s_cnt[1], np);
    }
  }
  // Wave-local compaction (static indices only: no private-memory arrays):
  // each wave appends its candidates to the block's list at a base one LDS
  // atomic hands it, and its lanes walk them at once -- no block barrier
  // between a wave's key loads and its walkers' first loads.
  const uint32_t incl = wscan_u32(cnt);
  const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  uint32_t wbase = 0;
  if (lane == 0 && wtot) wbase = atomicAdd(&s_tot, wtot);
  wbase = __shfl(wbase, 0);
  {
    uint32_t o = wbase + incl - cnt;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t b = (bits >> (2 * j)) & 3u;
      if (b) {
        bk[o] = (b & 1u) ? kr[j] : kp[j];
        bl[o++] = CandRec{s0 + j, (uint8_t)(f[j] | (b << 4)),
                          (uint8_t)mt[j], (uint8_t)(mt[j] >> 16), (uint8_t)(mt[j] >> 24)};
      }
    }
  }
  s_fbits[threadIdx.x] = bits;
#pragma unroll
  for (int q = 0; q < PER / 4; ++q) {
    uint32_t fw = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) fw |= (uint32_t)f[4 * q + j] << (8 * j);
    s_fw[q][threadIdx.x] = fw;
  }
  // (the wave's list entries, written by its lanes, are read by other lanes
  // of the same wave: LDS operations of one wave complete in order)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (eclk && threadIdx.x == 0) eclk[kEClk * blockIdx.x + 2] = wall_clock64();
  // candidate index: the block's segment of the candidate arrays (CH
  // per block; k_rapply's blocks take their emit block's segment)
  const uint32_t cbase = blockIdx.x * CH;
  // this lane's staging slice (its address computed here, not held -- and
  // spilled -- from the kernel's start)
  uint32_t sli = (threadIdx.x >> 6) * SL + lane;
  asm volatile("" : "+v"(sli));
  auto walk_all = [&](auto dl) {
    auto walk_cand = [&](uint32_t j) {
      const uint32_t i = wbase + j;
      const uint32_t cat = emit_one<BRK, decltype(dl)::value>(
          tb, rd, now_e, s_ph, bl[i], cbase + i, brec, bcount, s_sup, ltab, dense, dcap, post, decof,
          lane < SL ? stage + sli * kEmitStage : nullptr,
          bk[i], eclk && i < 512 ? eclk + 5 * 4096 + 8 + 4 * (blockIdx.x * 512 + i) : nullptr);
      atomicAdd(&s_ec[cat], 1u);
    };
    uint32_t j = lane;
    // immediate mode: a lane's first candidate (most lanes' only one) walked
    // outside the loop -- straight-line code, whose loads the compiler's wait
    // counting does not hold behind loads left in flight by a previous
    // iteration (a wave walks more than 64 candidates rarely)
    if (decltype(dl)::value == 0 && DMC_EMIT_PEEL && j < wtot) {
      walk_cand(j);
      j += 64;
    }
    for (; j < wtot; j += 64) walk_cand(j);
  };
  // (nothing of the selection is in flight any more; said explicitly, so that
  // the compiler's wait counting starts the walkers from an empty queue and
  // holds none of their loads behind a load it cannot see completed)
  if (DMC_EMIT_PEEL) __builtin_amdgcn_s_waitcnt(0x0f70);  // s_waitcnt vmcnt(0)
  if (!DMC_EMIT_MODE_SPLIT) walk_all(std::integral_constant<int, -1>{});
  else if (tb.delayed) walk_all(std::integral_constant<int, 1>{});
  else walk_all(std::integral_constant<int, 0>{});
  __syncthreads();
  const uint32_t tot = s_tot;
  if (threadIdx.x < 4 && s_ec[threadIdx.x]) atomicAdd(&rd->ecnt[threadIdx.x], s_ec[threadIdx.x]);
  // the block's super-bin sums (memory-side atomics, read by k_rrank)
  if (brec && threadIdx.x < kNSup && s_sup[threadIdx.x])
    atomicAdd(&gsup[threadIdx.x], s_sup[threadIdx.x]);
  // the candidate count (a statistic) and the sampled counts, published
  // after the walks (same-address atomics, serialised over the grid; on
  // gfx950 a wave's load waits also wait for its earlier memory operations)
  if (threadIdx.x == 64) {
    if (tot) atomicAdd(&rd->n_cand, tot);
    if (sampled) {
      uint32_t* cc = rd->ccnt + 2 * (blockIdx.x % kCntShards);
      if (s_cnt[0]) atomicAdd(&cc[0], s_cnt[0]);
      if (s_cnt[1]) atomicAdd(&cc[1], s_cnt[1]);
    }
  }
  if (eclk && threadIdx.x == 0) eclk[kEClk * blockIdx.x + 3] = wall_clock64();
  // the block's candidates, copied from LDS in one coalesced pass
  for (uint32_t i = threadIdx.x; i < tot; i += kEmitThreads) cand[cbase + i] = bl[i];
  if (threadIdx.x == 0) bcand[blockIdx.x] = tot;
  // non-candidates settle their pending limit-scan marks (after the walks:
  // a store ahead of a walk's loads would delay them)
  {
    uint32_t ti = threadIdx.x;
    asm volatile("" : "+v"(ti));  // (its LDS address recomputed here, not held)
    const uint32_t fbits = s_fbits[ti];
    uint32_t fws[PER / 4];
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) fws[q] = s_fw[q][ti];
    const uint32_t s0b = blockIdx.x * CH + ti * PER;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t fj = (fws[j / 4] >> (8 * (j % 4))) & 0xffu;
      if (s0b + j < n && !((fbits >> (2 * j)) & 3u) && (fj & F_PMARK))
        tb.sc[s0b + j].flags = (uint8_t)((fj & ~F_PMARK) | (p_runs ? F_READY : 0));
    }
  }
  if (eclk && threadIdx.x == 0) eclk[kEClk * blockIdx.x + 4] = wall_clock64();
}
template <bool BRK>
__global__ void __launch_bounds__(kEmitThreads, DMC_EMIT_MINW)
k_remit_t(Table tb, Round* rd, const uint2* k32,
        const uint32_t* meta, CandRec* cand, uint32_t* bcand, PostRec* post,
        uint32_t* decof, BRecR* brec,
        uint32_t* bcount, unsigned long long* gsup, const uint32_t* hist, DEnt* dense,
        uint32_t dcap, uint64_t* eclk = nullptr) {
  remit_t_body<BRK, false, kEmitPer, kEmitStageThreads>(tb, rd, k32, meta, cand, bcand, post,
                                                         decof, brec, bcount, gsup, hist,
                    dense, dcap, eclk);
}

// the general emission and the limit-break rounds'
constexpr auto k_remit = k_remit_t<false>;
constexpr auto k_remit_brk = k_remit_t<true>;

// ---------------------------------------------------------------- k_rrank
// One block per rank bin ranks it in LDS by (okey, slot, position); R bins
// precede P bins, so the decision offset of an entry is the sum of the group
// sizes (1 for R pops, 1 + run for P groups) of all earlier bins (the
// super-bin sums before its super-bin and the bins before it in its own)
// plus those of its own bin that precede it.  Decides: a fast record's
// decision is written (and its offset recorded for k_rapply); a slow record's
// entry (slot * q + position) gets its decision offset and tie flag stamped
// into the ring entry (the priority pop's entry for a P group).

#ifndef DMC_DEEP_BATCH
#define DMC_DEEP_BATCH 8
#endif
constexpr int kDeepBatch = DMC_DEEP_BATCH;   // queued requests reduced per batch of loads

// Rank of record i of a bin among all `cnt` of them, compared in `parts`
// slices of `per` records by adjacent lanes whose counts are summed by
// shuffles; lanes with i >= cnt take part in the shuffles only.  The lane
// that owns a record then decides it: a fast record's decision is written
// and its offset recorded for k_rapply (which stores the candidate's
// precomputed state); a slow record's pop is stamped into its ring entry.
// (Storing the fast candidates' state here instead, in the rank lanes, was
// measured slower: rank 9.8 -> 21.2 us for apply 11.5 -> 6.3, §10.)
// A ranked record's stores: its decision offset goff (the group sizes of
// the bin's records before it plus the bin's offset), stamped or written.
// A queue group's per-slot completion tallies (the trackers' track_resp,
// dmc_tracker.h), made where a decision is written -- k_rrank_m's fast
// records, k_rapply_m's pops -- instead of by a pass over the decisions
// after the round (k_tally_m then counts only what later, host-driven rounds
// wrote).  A round that fails writes no decision and tallies nothing.
struct TallyP {
  uint32_t* d = nullptr;
  uint32_t* r = nullptr;
};
__device__ inline void tally_one(const TallyP& t, uint32_t slot, uint32_t cost, bool resv) {
  if (!t.d) return;
  atomicAdd(&t.d[slot], cost);
  if (resv) atomicAdd(&t.r[slot], cost);
}
__device__ inline void place_rec(Round* rd, const BKey& me, uint32_t ci, uint32_t cost,
                                 uint64_t handle, double tr, double tp, double tl,
                                 uint32_t rank, uint32_t gl, uint32_t tie, bool isp, uint32_t k,
                                 uint32_t n_pgroups, uint32_t soff, uint32_t poff,
                                 ReqEntry* ring, dmc_decision* out, uint32_t* decof, const TallyP& tly) {
  uint32_t goff = soff + gl;
  uint32_t size = isp ? 1u + me.run : 1u;
  if (goff < k) {
    if ((ci & kFastRec) && goff + size > k) {
      // a fast group cut by the round's end: k_rapply re-walks it
      ring[me.ridx].dec = goff;
      ring[me.ridx].tie = tie;
      decof[ci & ~kFastRec] = kSlowCand;
    } else if (ci & kFastRec) {
      // a fast record: its first pop's decision, and its offset for
      // k_rapply (which writes the run's pop and the candidate's state)
      dmc_decision d;
      d.handle = handle;
      d.tag_r = tr;
      d.tag_p = tp;
      d.tag_l = tl;
      d.slot = me.slot;
      d.cost = cost;
      d.phase = isp ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
      d.flags = tie;
      out[goff] = d;
      decof[ci & ~kFastRec] = goff;
      (void)tly;  // (its tally: k_rapply, with the run's, PostRec::cost0)
    } else {
      ring[me.ridx].dec = goff;  // the stamp k_rapply's walk follows
      ring[me.ridx].tie = tie;
    }
    if (isp) {
      uint32_t prank = poff + rank;  // among P groups
      if (goff + size >= k || prank == n_pgroups - 1) {
        // the last applied group: its priority pop is the round's last
        // limit-scanning pull
        rd->g_last = goff;
        rd->n_prio = prank + 1;
      }
    }
  }
}

// A record's order key as k_rrank stages it in LDS: 16 bytes (the queue
// position and the group's run packed), so that a bin's 512 keys take 8 KB
// and nearly every non-empty bin's block is resident at once (24-byte keys:
// 15.9 KB per block, ten per CU -- two generations of blocks per round);
// the ring index is read from the record when the pop is placed.
struct BKeyS {
  uint64_t okey;
  uint64_t lo;  // slot << 32 | queue position << 16 | run
  __device__ uint32_t slot() const { return (uint32_t)(lo >> 32); }
  __device__ uint32_t seq() const { return (uint32_t)(lo >> 16) & 0xffffu; }
  __device__ uint32_t run() const { return (uint32_t)lo & 0xffffu; }
};
static_assert(sizeof(BKeyS) == 16, "BKeyS must be 16 bytes");
__device__ inline BKeyS bkey_s(const BKey& k) {
  return BKeyS{k.okey, ((uint64_t)k.slot << 32) | ((k.seq & 0xffffu) << 16) | (k.run & 0xffffu)};
}

// Rank of record i of a bin among all `cnt` of them, compared in `parts`
// slices of `per` records by adjacent lanes whose counts are summed by
// shuffles; lanes with i >= cnt take part in the shuffles only.  The order
// (okey, slot, queue position) is one 128-bit comparison of (okey, lo): two
// records of a bin never share slot and position, so lo's run bits never
// decide it -- the borrow of a 128-bit subtraction, added into the rank
// (VALU-bound: a heavy bin's block runs one wave per SIMD, and the compare
// chain is most of its time).  The lane that owns a record then decides it:
// a fast record's decision is written and its offset recorded for k_rapply
// (which stores the candidate's precomputed state); a slow record's pop is
// stamped into its ring entry.  (ISP: a P bin, whose records' group sizes
// 1 + run give the decision offsets; an R bin's offset is its rank.)
#ifndef DMC_RANK_OKEY_FIRST
#define DMC_RANK_OKEY_FIRST 1
#endif
template <bool ISP>
__device__ inline void rank_rec(Round* rd, const BKeyS* sh, const BRecR* src, uint32_t cnt,
                                bool anyrun, uint32_t parts, uint32_t per, uint32_t i,
                                uint32_t part, uint32_t k,
                                uint32_t n_pgroups, uint32_t soff, uint32_t poff,
                                ReqEntry* ring, dmc_decision* out, uint32_t* decof, const TallyP& tly) {
  const bool valid = i < cnt;
  const BKeyS me = sh[valid ? i : 0];
  const uint32_t me_slot = me.slot();
  // the writer lane's payload (an L2 hit: the block staged the line), in
  // flight during the comparisons
  // (every lane loads a record -- its own, or the bin's first -- and only the
  // writer uses it: a load under a condition merges with a default value,
  // which the compiler resolves with a copy, and a wait for the load, right
  // after it, ahead of the comparisons it should overlap)
  const BRecR& x = src[valid ? i : 0];
  const uint32_t ci = x.ci, cost = x.cost, ridx = x.k.ridx;
  const uint64_t handle = x.handle;
  const double tr = x.r, tp = x.p, tl = x.l;
  uint32_t f0 = part * per, f1 = f0 + per < cnt ? f0 + per : cnt;
  if (!valid) f1 = f0;
  uint32_t rank = 0, gl = 0, tie = 0;
#if DMC_RANK_OKEY_FIRST
  // The order key decides unless it is equal: the main pass counts the
  // records with a smaller okey (and, in a P bin whose records have runs,
  // their runs) and those with an equal one; only a record whose okey is
  // shared (eq > 1: itself and another) walks the bin again for the exact
  // (okey, slot, queue position) order among the equal ones and the tie
  // flag.  Four VALU operations per compared record instead of eleven, and
  // the next keys' LDS reads issued before this batch's compares (one wave
  // per SIMD: nothing else hides their latency).
  uint32_t lt = 0, eq = 0, rs = 0;
  {
    // (okeys only; reads past f1 stay inside sh -- f1 <= cnt <= kRankSortMin,
    // sh holds kBinCapR -- and are masked)
    // whole batches of U unmasked (every load of a batch issued before its
    // compares), then one masked batch.  A P bin whose records have runs
    // reads the whole 16-byte keys (the run is in lo) in batches of 4,
    // other bins the okeys in batches of 8 (no LDS read inside a compare)
    auto batches = [&](auto cu, auto wide) {
      constexpr uint32_t U = decltype(cu)::value;
      constexpr bool W = decltype(wide)::value;
      uint32_t f = f0;
      for (; f + U <= f1; f += U) {
        uint64_t ck[U];
        uint32_t cr[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
          if (W) {
            const BKeyS b = sh[f + j];
            ck[j] = b.okey;
            cr[j] = (uint32_t)b.lo & 0xffffu;
          } else {
            ck[j] = sh[f + j].okey;
            cr[j] = 0;
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
          const bool l = ck[j] < me.okey;
          lt += l ? 1u : 0u;
          eq += ck[j] == me.okey ? 1u : 0u;
          if (W) rs += l ? cr[j] : 0u;
        }
      }
      if (f < f1) {
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
          const BKeyS b = sh[f + j];
          const bool in = f + j < f1;
          const bool l = in && b.okey < me.okey;
          lt += l ? 1u : 0u;
          eq += (in && b.okey == me.okey) ? 1u : 0u;
          if (W) rs += l ? ((uint32_t)b.lo & 0xffffu) : 0u;
        }
      }
    };
    if (ISP && anyrun)
      batches(std::integral_constant<uint32_t, 4>{}, std::true_type{});
    else
      batches(std::integral_constant<uint32_t, 8>{}, std::false_type{});
  }
  for (uint32_t d = 1; d < parts; d <<= 1) {
    lt += __shfl_xor(lt, d);
    eq += __shfl_xor(eq, d);
    if (ISP && anyrun) rs += __shfl_xor(rs, d);
  }
  rank = lt;
  gl = lt + rs;
#ifndef DMC_RANK_NOSLOW
#define DMC_RANK_NOSLOW 0  // (A/B probe only: wrong on equal keys)
#endif
  if (!DMC_RANK_NOSLOW && valid && part == 0 && eq > 1) {
    // (rare: keys shared by several records) the equal okeys, in order
    for (uint32_t f = 0; f < cnt; ++f) {
      const BKeyS o = sh[f];
      if (o.okey != me.okey) continue;
      if (o.lo < me.lo) {
        ++rank;
        gl += 1u + (ISP ? ((uint32_t)o.lo & 0xffffu) : 0u);
      }
      tie |= (uint32_t)((uint32_t)(o.lo >> 32) != me_slot);
    }
  }
  if (!ISP) gl = rank;
#else
  (void)anyrun;
#pragma unroll 4
  for (uint32_t f = f0; f < f1; ++f) {
    const BKeyS o = sh[f];
    unsigned long long b0, b1;
    (void)__builtin_subcll(o.lo, me.lo, 0ull, &b0);
    (void)__builtin_subcll(o.okey, me.okey, b0, &b1);  // b1: o < me
    rank += (uint32_t)b1;
    if (ISP) gl += b1 ? 1u + ((uint32_t)o.lo & 0xffffu) : 0u;
    tie |= (uint32_t)(o.okey == me.okey) & (uint32_t)((uint32_t)(o.lo >> 32) != me_slot);
  }
  for (uint32_t d = 1; d < parts; d <<= 1) {
    rank += __shfl_xor(rank, d);
    if (ISP) gl += __shfl_xor(gl, d);
    tie |= __shfl_xor(tie, d);
  }
  if (!ISP) gl = rank;
#endif
  if (valid && part == 0)
    place_rec(rd, BKey{me.okey, me_slot, me.seq(), me.run(), ridx}, ci, cost, handle, tr, tp, tl,
              rank, gl, tie, ISP, k, n_pgroups, soff, poff, ring, out, decof, tly);
}

// One block per rank bin.  The bin's order keys are staged in LDS; each
// record is ranked against all of them by `parts` adjacent lanes, each
// comparing a slice (parts = the largest power of two with cnt * parts <=
// 256, at most 64): a big bin (skewed keys) costs cnt^2 / 256 compare steps
// per lane instead of cnt.  A bin of more than kBlockR records (parts = 1)
// takes ceil(cnt / kBlockR) passes of one record per thread.  The comparison
// is branchless (wave-uniform trip counts, broadcast LDS reads).  (One wave
// per bin, four bins per block, was measured slower: the skewed P bins of up
// to ~190 records then take three serial passes in one wave.)  A bin's
// records take consecutive decision offsets, so fast records' decision
// stores from one block fill one stretch of the decision array.
constexpr int kRankBlocksR = kNBR;

// A bin of more than kRankSortMin records (skewed keys: config 4's activated
// clients emit several P groups each) is sorted instead: a bitonic sort of
// the record indices by the same order (okey, slot, queue position) in LDS,
// one compare-exchange per thread per step (45 steps for 512), then the
// group offsets by a block scan of the sizes in sorted order, and a tie
// where the record's run of equal keys holds another slot.  Counting costs
// cnt^2 / 256 compare steps per lane: 973 for a full bin.
#ifndef DMC_RANK_SORT_MIN
#define DMC_RANK_SORT_MIN 256
#endif
constexpr uint32_t kRankSortMin = DMC_RANK_SORT_MIN;
// (rank_rec's unmasked okey reads run up to 8 records past a counted bin)
static_assert(kRankSortMin + 16 <= kBinCapR, "rank reads past the bin stay in sh");
__device__ inline bool bkey_less(const BKeyS& x, const BKeyS& y) {
  return x.okey < y.okey || (x.okey == y.okey && x.lo < y.lo);
}
// The bin's records sorted in registers: a bitonic network over 512 (key,
// record index) elements, thread t holding elements 4t..4t+3 -- the
// compare-exchanges of distance 1 and 2 inside a thread, 4..128 with the
// partner lane's elements (shuffles), 256 with the other wave's (their
// indices through LDS, the keys re-read from sh).  Padding (index >= cnt)
// orders after every record.  ord[r]: the record at sorted position r.
// (The LDS network before it, one compare-exchange per thread and step with
// a barrier each, took ~20 us for a full bin: k_rrank's tail.)
#ifndef DMC_RANK_REGSORT
#define DMC_RANK_REGSORT 1
#endif
struct SK {
  uint64_t k, l;
  uint32_t i;
};
__device__ inline SK sk_at(const BKeyS* sh, uint32_t i, uint32_t cnt) {
  if (i < cnt) {
    const BKeyS b = sh[i];
    return SK{b.okey, b.lo, i};
  }
  return SK{~0ull, ~0ull, i};
}
__device__ inline bool sk_less(const SK& a, const SK& b) {
  return a.k < b.k || (a.k == b.k && a.l < b.l);
}
// a keeps the smaller of (a, b) when `mn`, else the larger
__device__ inline SK sk_keep(const SK& a, const SK& b, bool mn) {
  const bool take = mn ? sk_less(b, a) : sk_less(a, b);
  return SK{take ? b.k : a.k, take ? b.l : a.l, take ? b.i : a.i};
}
__device__ inline void sk_cx(SK& a, SK& b, bool asc) {
  const bool sw = asc ? sk_less(b, a) : sk_less(a, b);
  const SK x = a, y = b;
  a = SK{sw ? y.k : x.k, sw ? y.l : x.l, sw ? y.i : x.i};
  b = SK{sw ? x.k : y.k, sw ? x.l : y.l, sw ? x.i : y.i};
}
__device__ inline SK sk_shfl_xor(const SK& a, uint32_t m) {
  SK o;
  o.k = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(a.k >> 32), (int)m) << 32) |
        (uint32_t)__shfl_xor((int)(uint32_t)a.k, (int)m);
  o.l = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(a.l >> 32), (int)m) << 32) |
        (uint32_t)__shfl_xor((int)(uint32_t)a.l, (int)m);
  o.i = (uint32_t)__shfl_xor((int)a.i, (int)m);
  return o;
}
__device__ inline void sort_bin_regs(const BKeyS* sh, uint32_t cnt, uint16_t* ord) {
  static_assert(kBinCapR == 512 && kRankThreads == 128, "4 elements per thread, 2 waves");
  const uint32_t t = threadIdx.x;
  __syncthreads();  // (sh: staged by the whole block)
  SK v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = sk_at(sh, 4 * t + r, cnt);
  for (uint32_t k = 2; k <= kBinCapR; k <<= 1) {
    const bool asc = ((4 * t) & k) == 0;  // (k >= 4: the same for the thread's 4)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j == 1) {
        sk_cx(v[0], v[1], k == 2 ? true : asc);
        sk_cx(v[2], v[3], k == 2 ? false : asc);
      } else if (j == 2) {
        sk_cx(v[0], v[2], asc);
        sk_cx(v[1], v[3], asc);
      } else {
        const uint32_t m = j >> 2;  // the partner thread: t ^ m
        const bool mn = ((t & m) == 0) == asc;
        if (m < 64) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = sk_keep(v[r], sk_shfl_xor(v[r], m), mn);
        } else {
          __syncthreads();  // (ord's previous readers)
#pragma unroll
          for (int r = 0; r < 4; ++r) ord[4 * t + r] = (uint16_t)v[r].i;
          __syncthreads();
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = sk_keep(v[r], sk_at(sh, ord[4 * (t ^ m) + r], cnt), mn);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) ord[4 * t + r] = (uint16_t)v[r].i;
  __syncthreads();
}

__device__ inline void rank_sorted(Round* rd, const BKeyS* sh, const BRecR* src, uint32_t cnt,
                                   bool isp, uint32_t k, uint32_t n_pgroups, uint32_t soff,
                                   uint32_t poff, ReqEntry* ring, dmc_decision* out,
                                   uint32_t* decof, const TallyP& tly) {
  constexpr uint32_t RP = kBinCapR / kRankThreads;  // sorted positions per thread
  static_assert(kBinCapR % kRankThreads == 0 && RP <= 8, "whole positions per thread");
  __shared__ uint16_t ord[kBinCapR];
  __shared__ uint32_t wsum[kRankThreads / 64];
  const uint32_t t = threadIdx.x;
#if DMC_RANK_REGSORT
  sort_bin_regs(sh, cnt, ord);
#else
  uint32_t P = 2;
  while (P < cnt) P <<= 1;
  for (uint32_t i = t; i < P; i += kRankThreads) ord[i] = (uint16_t)i;
  __syncthreads();
  for (uint32_t kk = 2; kk <= P; kk <<= 1) {
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t u = t; u < P / 2; u += kRankThreads) {
        const uint32_t i = ((u & ~(j - 1)) << 1) | (u & (j - 1)), l = i | j;
        const uint32_t a = ord[i], c = ord[l];
        const bool c_lt_a = c < cnt && (a >= cnt || bkey_less(sh[c], sh[a]));
        const bool a_lt_c = a < cnt && (c >= cnt || bkey_less(sh[a], sh[c]));
        if ((i & kk) == 0 ? c_lt_a : a_lt_c) {
          ord[i] = (uint16_t)c;
          ord[l] = (uint16_t)a;
        }
      }
      __syncthreads();
    }
  }
#endif
  // positions RP t .. RP t + RP - 1: their records, sizes, the exclusive prefix
  uint32_t z[RP], ix[RP], zs = 0;
#pragma unroll
  for (uint32_t h = 0; h < RP; ++h) {
    const uint32_t r = RP * t + h;
    ix[h] = r < cnt ? ord[r] : 0u;
    z[h] = r < cnt ? (isp ? 1u + sh[ix[h]].run() : 1u) : 0u;
    zs += z[h];
  }
  const uint32_t lane = t & 63, w = t >> 6;
  const uint32_t incl = wscan_u32(zs);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t q = 0; q < w; ++q) pre += wsum[q];
  uint32_t ex = pre + incl - zs;
  // tie flags in O(1) per record: a record ties iff the run of equal keys
  // holding it (contiguous in the sorted order) holds two slots, i.e. two
  // adjacent members with different slots -- runs numbered by a prefix
  // count of their heads, each run's flag set by any such pair (heavily
  // tied bins, config 4's activated clients, made the scans of the run
  // from every member quadratic)
  __shared__ uint8_t runtie[kBinCapR];  // (bytes: the block's LDS stays under 10 KB)
  __shared__ uint32_t wrun[kRankThreads / 64];
  uint32_t hd = 0, dd = 0, nh = 0;  // per position h: bit h
#pragma unroll
  for (uint32_t h = 0; h < RP; ++h) {
    const uint32_t r = RP * t + h;
    if (r >= cnt) continue;
    const BKeyS me = sh[ix[h]];
    bool head = true, diff = false;
    if (r > 0) {
      const BKeyS pv = sh[ord[r - 1]];
      head = pv.okey != me.okey;
      diff = !head && pv.slot() != me.slot();
    }
    hd |= (head ? 1u : 0u) << h;
    dd |= (diff ? 1u : 0u) << h;
    nh += head ? 1u : 0u;
    runtie[r] = 0;
  }
  const uint32_t rincl = wscan_u32(nh);
  if (lane == 63) wrun[w] = rincl;
  __syncthreads();
  uint32_t rbase = 0;
  for (uint32_t q = 0; q < w; ++q) rbase += wrun[q];
  rbase += rincl - nh;  // heads before this thread's positions
  uint32_t runid[RP];
  {
    uint32_t c = rbase;
#pragma unroll
    for (uint32_t h = 0; h < RP; ++h) {
      c += (hd >> h) & 1u;
      runid[h] = c - 1u;  // (position 0 is a head: c >= 1 for every position < cnt)
      if ((dd >> h) & 1u) runtie[c - 1u] = 1;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t h = 0; h < RP; ++h) {
    const uint32_t r = RP * t + h;
    const uint32_t exh = ex;
    ex += z[h];
    if (r >= cnt) continue;
    const uint32_t i = ix[h];
    const uint32_t tie = runtie[runid[h]];
    const BRecR& x = src[i];
    place_rec(rd, x.k, x.ci, x.cost, x.handle, x.r, x.p, x.l, r, exh, tie, isp, k,
              n_pgroups, soff, poff, ring, out, decof, tly);
  }
}

// A sampled round whose thresholds admitted fewer first keys than needed
// (k_remit's exact counts): it is re-run with the exact histogram (nothing
// of it is applied); every entry the k pulls take has a key at or below an
// admitted threshold otherwise
__device__ inline bool sample_failed(const Round* rd) {
  if (!rd->sampled) return false;
  const uint32_t k = rd->k_total;
  const uint32_t needR = rd->p_runs ? 0xffffffffu : k;
  const uint32_t needP = rd->p_runs ? k - (uint32_t)rd->n_r : 0u;
  const uint64_t TR = rd->ph[0].T, TP = rd->p_runs ? rd->ph[1].T : 0;
  uint32_t c0 = 0, c1 = 0;
  for (int i = 0; i < kCntShards; ++i) {
    c0 += rd->ccnt[2 * i];
    c1 += rd->ccnt[2 * i + 1];
  }
  return (TR && TR != kMaxKey - 1 && c0 < needR) || (TP && TP != kMaxKey - 1 && c1 < needP);
}

// Rank diagnostics: the largest bin per phase, recorded by the bins above
// this size only (a handful per round; an overflowing bin always)
constexpr uint32_t kBinMaxReport = 128;

__device__ __attribute__((always_inline)) inline void rrank_body(Round* rd, const unsigned long long* bcount, const unsigned long long* gsup, const BRecR* brec, ReqEntry* ring, uint32_t* decof, uint64_t* wtime, TallyP tly = TallyP{}) {
  // the rank-bin counters requested with the skip word (one level of loads)
  unsigned long long sv = 0, bv = 0;
  if (threadIdx.x < 64) {
    sv = gsup[threadIdx.x];
    bv = bcount[(blockIdx.x / kSupBins) * kSupBins + threadIdx.x];
  }
  if (rd->skip) return;
  __shared__ BKeyS sh[kBinCapR];
  // the bin's records, its group and P-group offsets, P groups, the round's
  // outcome check
  __shared__ uint32_t s_hdr[5];
  uint64_t t0 = wall_clock64();
  const uint32_t b = blockIdx.x;
  const bool isp = b >= (uint32_t)kNBPhase;
  const BRecR* src = brec + (size_t)b * kBinCapR;
  // the round's inputs, read once before any store (block 0 writes the
  // outcome into the same record)
  const uint32_t ovf0 = rd->overflow, bovf = rd->bin_ovf;
  const bool sfail = sample_failed(rd);
  const uint32_t k = rd->k_total;
  const uint32_t p_runs = rd->p_runs;
  dmc_decision* const out = rd->out;
  const bool fail0 = ovf0 || bovf || sfail;
  if (threadIdx.x < 64) {
    // one level of loads: the 64 super-bin sums and the 64 bins of this
    // bin's super-bin (the rank-bin counters k_remit's walkers filled:
    // records | group sizes << 32)
    const uint32_t lane = threadIdx.x, sb = b / kSupBins, ib = b % kSupBins;
    const uint32_t sc = (uint32_t)sv, sz = (uint32_t)(sv >> 32);
    const uint32_t bc = (uint32_t)bv, bz = (uint32_t)(bv >> 32);
    const bool psup = lane >= (uint32_t)(kNSup / 2);  // (P bins: super-bins 32..63)
    const uint32_t zoff = wsum_all((lane < sb ? sz : 0u) + (lane < ib ? bz : 0u));
    const uint32_t poff =
        wsum_all((lane < sb && psup ? sc : 0u) + (isp && lane < ib ? bc : 0u));
    const uint32_t tp = wsum_all(psup ? sc : 0u);
    const uint32_t cnt = __shfl(bc, (int)ib);
    // The round's outcome check (every block, from the same inputs: all
    // agree): both phases' selections written by the pick; with the priority
    // pulls running, every R-prefix entry emitted, and a round short of k
    // only if the P threshold admitted every eligible client; without them,
    // at least k R records.  A violation fails the round (overflow = 7:
    // nothing is applied, the call returns DMC_EDEVICE) instead of
    // dispatching short.  (dmclock_server.h:1115-1186: k pulls take
    // min(k, eligible) requests.)
    const uint32_t tz = wsum_all(sz), tcr = wsum_all(psup ? 0u : sc);
    bool bad = false;
    if (!fail0) {
      const PhaseSel& p1 = rd->ph[1];
      bad = rd->ph[0].valid != kSelValid || p1.valid != kSelValid;
      if (!bad && p_runs) {
        bad = (uint64_t)tcr != rd->n_r ||
              (tz < k && !(p1.T == kMaxKey - 1 || (p1.T == 0 && p1.n_elig == 0)));
      } else if (!bad) {
        bad = tcr < k;
      }
    }
    if (b == 0) {
      // the round's totals and outcome (the summary k_rapply publishes)
      const uint32_t tc = wsum_all(sc);
      if (lane == 0 && !ovf0) {
        if (bad) {
          rd->overflow = 7;
        } else if (sfail) {
          rd->overflow = 3;  // re-run with the exact histogram
        } else if (bovf) {
          // re-run with fewer pulls or on the radix path: the emitted
          // entries (overflowed bins included) size a radix retry's dense
          // buffer, bin_max (below) a smaller round
          rd->dense_n = tc;
          rd->overflow = 2;
        } else {
          rd->n_dec = tz < k ? tz : k;
          rd->terminal = (p_runs && tz < k) ? 1 : 0;
          rd->n_pgroups = tp;
          rd->n_emit = tc;
        }
      }
    }
    if (lane == 0) {
      s_hdr[0] = cnt;
      s_hdr[1] = zoff;
      s_hdr[2] = poff;
      s_hdr[3] = tp;
      s_hdr[4] = bad ? 1u : 0u;
      if (cnt > kBinMaxReport) atomicMax(&rd->bin_max[isp ? 1 : 0], cnt);
    }
  }
  __shared__ uint32_t s_anyrun;
  if (threadIdx.x == 0) s_anyrun = 0;
  __syncthreads();
  const uint32_t cnt = s_hdr[0];
  if (cnt == 0 || fail0 || s_hdr[4]) return;
  const uint32_t soff = s_hdr[1], poff = s_hdr[2], n_pgroups = s_hdr[3];
  {
    // (a P bin's records with runs: their group sizes enter the offsets;
    // most bins have none, and the rank skips them)
    uint32_t ar = 0;
    for (uint32_t i = threadIdx.x; i < cnt; i += kRankThreads) {
      const BKeyS b = bkey_s(src[i].k);
      sh[i] = b;
      ar |= (uint32_t)b.lo & 0xffffu;
    }
    if (ar) s_anyrun = 1;  // (benign race: every writer stores 1)
  }
  if (cnt > kRankSortMin) {
    rank_sorted(rd, sh, src, cnt, isp, k, n_pgroups, soff, poff, ring, out, decof, tly);
    if (wtime && threadIdx.x == 0) {
      wtime[2 * b] = t0;
      wtime[2 * b + 1] = wall_clock64();
    }
    return;
  }
  __syncthreads();
  const bool anyrun = s_anyrun != 0;
  const uint32_t t = threadIdx.x;
  // passes of kRankThreads / parts records, parts lanes per record, parts
  // sized per pass (a bin of 190: 128 records with 1 lane each, then 62 with 2)
  for (uint32_t rb = 0; rb < cnt;) {
    const uint32_t rem = cnt - rb;
    uint32_t parts = 1;
    while (parts < 64 && rem * parts * 2 <= (uint32_t)kRankThreads) parts <<= 1;
    const uint32_t per = (cnt + parts - 1) / parts;
    if (isp)
      rank_rec<true>(rd, sh, src, cnt, anyrun, parts, per, rb + t / parts, t % parts, k, n_pgroups,
                     soff, poff, ring, out, decof, tly);
    else
      rank_rec<false>(rd, sh, src, cnt, false, parts, per, rb + t / parts, t % parts, k, n_pgroups,
                      soff, poff, ring, out, decof, tly);
    rb += kRankThreads / parts;
  }
  if (wtime && threadIdx.x == 0) {
    wtime[2 * b] = t0;
    wtime[2 * b + 1] = wall_clock64();
  }
}
__global__ void __launch_bounds__(kRankThreads)
k_rrank(Round* rd, const unsigned long long* bcount, const unsigned long long* gsup,
        const BRecR* brec, ReqEntry* ring, uint32_t* decof, uint64_t* wtime = nullptr) {
  rrank_body(rd, bcount, gsup, brec, ring, decof, wtime);
}

// ---------------------------------------------------------------- radix path
// (the dense entries are sorted by dmc_sort.h's exact LSD passes)
__global__ void k_dsizes(const Round* rd, uint32_t dcap, uint32_t E,
                         const uint32_t* sval, const DEnt* dense, uint32_t* gsz,
                         uint32_t* isp) {
  uint32_t n = (!rd->overflow && rd->dense_n <= dcap) ? rd->dense_n : 0;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < E;
       p += gridDim.x * blockDim.x) {
    uint32_t g = 0, ip = 0;
    if (p < n) {
      const DEnt& d = dense[sval[p]];
      ip = d.seq >> 31;
      g = ip ? 1 + d.run : 1;
    }
    gsz[p] = g;
    isp[p] = ip;
  }
}

__device__ inline bool dtie_at(const DEnt* dense, const uint32_t* sval,
                               uint32_t n, uint32_t pos) {
  const DEnt& e = dense[sval[pos]];
  for (int d = -1; d <= 1; d += 2) {
    int64_t o = (int64_t)pos + d;
    if (o < 0 || o >= (int64_t)n) continue;
    const DEnt& f = dense[sval[o]];
    if ((f.seq >> 31) == (e.seq >> 31) && f.okey == e.okey && f.slot != e.slot)
      return true;
  }
  return false;
}

// decisions are the prefix of the sorted entries' groups up to k
__global__ void k_ddecide(Round* rd, uint32_t dcap, const uint32_t* sval,
                          const DEnt* dense, const uint32_t* gsz,
                          const uint32_t* goff, const uint32_t* gp,
                          ReqEntry* ring) {
  if (rd->overflow || rd->dense_n > dcap) return;
  uint32_t n = rd->dense_n, k = rd->k_total;
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (n == 0) {
    if (tid == 0) {
      rd->n_dec = 0;
      rd->terminal = rd->p_runs && k > 0 ? 1 : 0;
    }
    return;
  }
  uint32_t np = gp[n - 1] + (dense[sval[n - 1]].seq >> 31);  // P groups (incl.)
  for (uint32_t pos = tid; pos < n; pos += gridDim.x * blockDim.x) {
    const DEnt& d = dense[sval[pos]];
    uint32_t o = goff[pos];
    bool isp = d.seq >> 31;
    if (pos == n - 1) {
      uint32_t tot = o + gsz[pos];
      rd->n_dec = tot < k ? tot : k;
      rd->terminal = (rd->p_runs && tot < k) ? 1 : 0;
    }
    if (o < k) {
      ring[d.ridx].dec = o;
      ring[d.ridx].tie = dtie_at(dense, sval, n, pos) ? 1 : 0;
      if (isp && (pos == n - 1 || goff[pos + 1] >= k)) {
        rd->g_last = o;
        rd->n_prio = gp[pos] + 1;  // exclusive P count before + this one
      }
    }
  }
  (void)np;
}

// ---------------------------------------------------------------- k_rapply
struct ApplyV {
  dmc_decision* out;
  uint32_t slot;
  TallyP tp;
  uint32_t inrun = 0, gidx = 0;
  uint32_t last_idx = 0;
  uint32_t nprio = 0;  // priority pops (limit-break rounds count them here)
  bool any = false;
  __device__ void pop(uint32_t, const Tag3& t, uint32_t cost, uint64_t h,
                      uint32_t kind, bool pphase, uint32_t edec, uint32_t etie) {
    uint32_t idx, tie;
    const bool prio = kind != kPopR;
    if (!pphase) {
      idx = edec;
      tie = etie;
    } else {
      if (kind == kPopHead) {
        gidx = edec;
        inrun = 0;
      }
      idx = gidx + inrun;
      tie = kind == kPopHead ? etie : 0;
      ++inrun;
    }
    nprio += prio ? 1u : 0u;
    dmc_decision d;
    d.handle = h;
    d.tag_r = t.r;
    d.tag_p = t.p;
    d.tag_l = t.l;
    d.slot = slot;
    d.cost = cost;
    d.phase = prio ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
    d.flags = tie;
    tally_one(tp, slot, cost, !prio);
    // the first decision is held back and stored with the client's state at
    // the end (flush): no store sits ahead of the walk's and the reductions'
    // loads (a load wait also waits for the wave's earlier stores)
    if (!any) {
      first = d;
      first_idx = idx;
    } else {
      st_glb<dmc_decision, 16>(out + idx, d);  // (48-byte records of a 16-aligned buffer)
    }
    last_idx = idx;
    any = true;
  }
  dmc_decision first;
  uint32_t first_idx = 0;
  __device__ void flush() {
    if (any) st_glb<dmc_decision, 16>(out + first_idx, first);
  }
};
struct ApplyVR {
  ApplyV* a;
  __device__ void pop(uint32_t i, const Tag3& t, uint32_t c, uint64_t h, uint32_t k,
                      uint32_t d, uint32_t ti) {
    a->pop(i, t, c, h, k, false, d, ti);
  }
  __device__ void group(uint64_t, uint32_t) {}
};
struct ApplyVP {
  ApplyV* a;
  __device__ void pop(uint32_t i, const Tag3& t, uint32_t c, uint64_t h, uint32_t k,
                      uint32_t d, uint32_t ti) {
    a->pop(i, t, c, h, k, true, d, ti);
  }
  __device__ void group(uint64_t, uint32_t) {}
};

// One thread per slot.  Clients with dispatched pops replay their walks for
// exactly those pops (R pops, then P groups from the post-R state), write the
// decision records and store the new state: ring head/count, front cache,
// reduced reservation tags (immediate: every queued request, in order,
// :1088-1095; delayed: the front, :1077-1085), prev tag, and the front's ready
// flag: a front left by reservation pops only was seen by the round's first
// limit scan iff the priority pulls ran; one left by priority pops iff a later
// limit-scanning pull happened (or the round's terminal pull).  Untouched
// fronts turn their pending mark into F_READY iff the priority pulls ran.
// Block 0 also counts the round's decisions (sched[0] reservation, sched[1]
// priority, :1469,1479).
// The round's scalars, read once per thread (stores through the table could
// alias the round record, which would force re-loads inside the walks).
struct RoundC {
  uint64_t* dbg;  // debug: per-candidate stage clocks (8 per candidate) or null
  double now;
  uint64_t tick;
  dmc_decision* out;
  uint32_t g_last, terminal;
  uint32_t k;
  bool p_runs, ovf, brk;
  uint32_t* brk_prio;  // limit-break rounds: the priority pops' count
  TallyP tp;           // a queue group's tallies (null: none)
};

#ifndef DMC_APPLY_STAGE
#define DMC_APPLY_STAGE 4
#endif
constexpr int kApplyStage = DMC_APPLY_STAGE;  // queue positions staged per candidate (LDS)
// A popped slot's new ScanRec: its front keys and cursor bytes (head, count,
// flags), never its stamp and batch count (bytes 27-31): the next call's
// filing (k_add_link's atomic on the count, its stamp) may run beside this
// round's apply in one launch (k_apply_link, the deferred apply of
// pipelined calls).  Outside a batch the count is 0 already.
__device__ inline void sc_store_front(const Table& tb, uint32_t s, const ScanRec& o) {
  char* d = reinterpret_cast<char*>(tb.sc + s);
  st_as(d, make_ulonglong2(dbits(o.r), dbits(o.pk)));
  st_as(d + 16, dbits(o.l));
  st_as(d + 24, (uint16_t)(o.head | ((uint32_t)o.count << 8)));
  st_as(d + 26, o.flags);
}
__device__ inline void apply_one(const Table& tb, const RoundC& rc, const CandRec& cd,
                                 ReqEntry* st) {
  // every load that depends only on the candidate record is issued before
  // the first branch: one memory round trip for the client record and its
  // ring entries (the record's head / count and flags are k_remit's;
  // nothing between the two kernels changes them)
  const uint32_t s = cd.slot;
  const uint8_t f0 = cd.f();
  const CView cv = cand_view(tb, cd);
  Tag3 prev{tb.rec[s].prev_r, tb.rec[s].prev_p, tb.rec[s].prev_l, tb.rec[s].prev_arr};
  if (rc.ovf) {
    if (f0 & F_PMARK) tb.sc[s].flags = (uint8_t)(f0 & ~F_PMARK);
    return;
  }
  const double now = rc.now;
  const uint64_t tick = rc.tick;
  const uint32_t g_last = rc.g_last;
  const uint32_t terminal = rc.terminal;
  const bool p_runs = rc.p_runs;
  const uint32_t c = cv.c, h = cv.h;
  const RingView rv = stage_ring<kApplyStage>(tb, s, h, c, st);
  if (rc.dbg) rc.dbg[1] = wall_clock64();
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  ApplyV v{rc.out, s, rc.tp};
  Tag3 front{};
  uint32_t fcost = 0;
  uint32_t popsR = 0, popsP = 0;
  uint64_t pmask = 0;
  // exactly the pops the ranking stamped: the R prefix's, then the P groups'
  {
    ApplyVR vr{&v};
    popsR = walk_r(tb, rv, cv, now, kMaxKey, 0xffffffffu, vr, &prev, &front, &fcost,
                   true);
  }
  if (p_runs) {
    ApplyVP vp{&v};
    bool ready0 = popsR == 0 && (f0 & F_READY);
    WalkP w = walk_p(tb, rv, cv, now, kMaxKey, 0xffffffffu, vp, &prev, &front, &fcost,
                     popsR, front, popsR && tb.delayed, ready0, rc.k, rc.brk);
    popsP = w.pops;
    pmask = w.pmask;
  }
  uint32_t pops = popsR + popsP;
  if (rc.dbg) rc.dbg[2] = wall_clock64();
  if (pops == 0) {  // a candidate none of whose entries was dispatched
    if (f0 & F_PMARK)
      tb.sc[s].flags = (uint8_t)((f0 & ~F_PMARK) | (p_runs ? F_READY : 0));
    return;
  }
  uint32_t nc2 = c - pops, nh = (h + pops) & tb.qmask;
  if (!tb.delayed) {
    double front_r = 0.0;
    if (pmask) {
      const double rinv = cv.rinv;
      // remaining requests: all reductions, in order (from the entries as
      // they were: the staged copy is not rewritten)
      // (kDeepBatch at a time: the batch's loads before its stores)
      for (uint32_t k0 = pops; k0 < c; k0 += kDeepBatch) {
        double v[kDeepBatch];
#pragma unroll
        for (int j = 0; j < kDeepBatch; ++j)
          if (k0 + j < c) v[j] = reduced_r(rv, k0 + j, pmask, rinv);
#pragma unroll
        for (int j = 0; j < kDeepBatch; ++j)
          if (k0 + j < c) ring[(h + k0 + j) & tb.qmask].r = v[j];
        if (k0 == pops) front_r = v[0];
      }
      double pr = prev.r;
      for (uint32_t j = 0; j < pops; ++j)
        if ((pmask >> j) & 1ull) pr = __dsub_rn(pr, rv.offset_at(j, rinv));
      tb.rec[s].prev_r = pr;
    }
    if (nc2) {
      const ReqEntry fe = rv.at(pops);
      front = Tag3{pmask ? front_r : fe.r, fe.p, fe.l, fe.arrival};
    }
  } else {
    // delayed: the walks recomputed the new front and prev
    if (nc2) {
      ReqEntry& fe = ring[nh];
      fe.r = front.r;
      fe.p = front.p;
      fe.l = front.l;
      fe.delta = cv.cd;
      fe.rho = cv.cr;
    }
    tb.rec[s].prev_r = prev.r;
    tb.rec[s].prev_p = prev.p;
    tb.rec[s].prev_l = prev.l;
    tb.rec[s].prev_arr = prev.arrival;
    if (c >= 2) {
      tb.aux[s].last_tick = tick;
      if (tb.binfo) {  // U1: the first pop's get_cli_info became client.info
        tb.rec[s].r_inv = cv.tr;
        tb.rec[s].w_inv = cv.tw;
        tb.rec[s].l_inv = cv.tl;
      }
    }
  }
  if (rc.dbg) rc.dbg[3] = wall_clock64();
  v.flush();
  if (rc.brk && v.nprio) atomicAdd(rc.brk_prio, v.nprio);
  // the new front's heap keys, cursor and flags: one 32-byte ScanRec store
  uint8_t f = f0 & (uint8_t)~(F_READY | F_PMARK);
  ScanRec o{0.0, 0.0, 0.0, (uint8_t)nh, (uint8_t)nc2, 0, 0, 0};
  if (nc2) {
    o.r = front.r;
    o.pk = __dadd_rn(front.p, cv.pd);
    o.l = front.l;
    // (a limit-break group's run ends at a front with l > now, or at the
    // round's end before any pull scanned it: never ready)
    bool seen = rc.brk ? false
                       : popsP ? (terminal || (g_last != kNoneR && v.last_idx < g_last))
                               : p_runs;
    if (seen && front.l <= now) f |= F_READY;
  }
  o.flags = f;
  sc_store_front(tb, s, o);
}

// Candidates (the dense list) with dispatched pops replay their walks for
// exactly those pops (R pops, then P groups from the post-R state), write the
// decision records and store the new state: ring head/count, front cache,
// reduced reservation tags (immediate: every queued request, in order,
// :1088-1095; delayed: the front, :1077-1085), prev tag, and the front's
// ready flag: a front left by reservation pops only was seen by the round's
// first limit scan iff the priority pulls ran; one left by priority pops iff
// a later limit-scanning pull happened (or the round's terminal pull).
// (Non-candidates settled their pending marks in k_remit.)  Block 0 also
// counts the round's decisions (sched[0] reservation, sched[1] priority,
// :1469,1479).
// Round end (one block of 64): the device-API result record when the host
// expects this round to end the call (no overflow retry; a terminal round
// under AtLimit::Allow is followed by host-driven steps, which rewrite it),
// then the Round summary to host memory and its sequence number last.
// (from k_rapply: `round_end`; the terminal pull's re-publication leaves
// the gate alone)
__device__ inline void rfinish_body(const Round* rd, HostRound* h, bool round_end = false) {
  h += rd->seq & 1;
  // a pipelined round (DMC_OPT_PIPELINE): the gate stays open iff the round
  // ends its call (the host has nothing left to do for it)
  if (round_end && threadIdx.x == 0 && rd->gate)
    *rd->gate = round_ends_call(*rd) ? 0u : 1u;
  constexpr uint32_t W = sizeof(Round) / 4;
  const char* src = reinterpret_cast<const char*>(rd);
  char* dst = reinterpret_cast<char*>(&h->r);
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x)
    st_as<uint32_t>(dst + 4 * i, ld_as<uint32_t>(src + 4 * i));
  if (threadIdx.x == 0 && rd->res && !rd->overflow) {
    dmc_pull_result r{};
    r.n_decisions = rd->n_dec;
    bool stop = rd->terminal && rd->n_dec < rd->k_total;
    r.next_type = stop ? rd->next_type : DMC_NEXT_RETURNING;
    r.when = stop ? rd->when : 0.0;
    r.n_priority = rd->n_prio;
    r.n_reservation = rd->n_dec - rd->n_prio;
    *rd->res = r;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(&h->seq, rd->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A fast candidate (k_remit precomputed its state after its group: a pop at
// queue position 0 and at most one run pop; decof: kNoDec if it was not
// dispatched, else its first decision's offset): the stores apply_one would
// make for that case, with no walk -- the run pop's decision, the reduced
// reservation tags of the queued requests (the new front's and position 2's
// precomputed; from position 3 on read, reduced and written, every load
// issued before the first store), prev r, and the new front's ScanRec with
// its ready flag.  A front left by a priority pop was seen by a later
// limit-scanning pull iff the group's last decision precedes the round's
// last priority pull (or the round is terminal); one left by a reservation
// pop iff the priority pulls ran.
// A PostRec's first line (everything but a run's pop): what k_rapply loads
// for every fast candidate; a run's second line is loaded by apply_fast
// itself (DMC_POST_LINE1; 0: both lines with the first, round 4's form)
#ifndef DMC_POST_LINE1
#define DMC_POST_LINE1 1
#endif
struct PostL1 {
  double fr, fpk, fl, prev_r, off, r2;
  uint32_t bits, cand, cost0;
};
__device__ inline PostL1 post_l1(const PostRec& p) {
  return PostL1{p.fr, p.fpk, p.fl, p.prev_r, p.off, p.r2, p.bits, p.cand, p.cost0};
}
__device__ inline void apply_fast(const Table& tb, const RoundC& rc, const CandRec& cd,
                                  uint32_t d, const PostL1& pr, const PostRec* pp,
                                  const PostRec* both) {
  const uint32_t s = cd.slot;
  const uint8_t f0 = cd.f();
  if (d == kNoDec) {  // not dispatched: the pending mark settles
    if (f0 & F_PMARK)
      tb.sc[s].flags = (uint8_t)((f0 & ~F_PMARK) | (rc.p_runs ? F_READY : 0));
    return;
  }
  const uint32_t bits = pr.bits;
  const bool prio = bits & 1u;
  const uint32_t run = (bits >> 2) & 1u;
  const uint32_t c = cd.c, h = cd.h;
  const uint32_t pops = 1 + run;
  const uint32_t nc2 = c - pops, nh = (h + pops) & tb.qmask;
  if (prio) {
    ReqEntry* ring = tb.ring + (size_t)s * tb.q;
    const double off = pr.off;
    // positions >= 3, kDeepBatch at a time: loads, then stores
    for (uint32_t k0 = 3; k0 < c; k0 += kDeepBatch) {
      double v[kDeepBatch];
#pragma unroll
      for (int j = 0; j < kDeepBatch; ++j)
        if (k0 + j < c) v[j] = ring[(h + k0 + j) & tb.qmask].r;
#pragma unroll
      for (int j = 0; j < kDeepBatch; ++j)
        if (k0 + j < c) ring[(h + k0 + j) & tb.qmask].r = __dsub_rn(v[j], off);
    }
    if (nc2) ring[nh].r = pr.fr;
    if (!run && c >= 3) ring[(h + 2) & tb.qmask].r = pr.r2;
    tb.rec[s].prev_r = pr.prev_r;
  }
  uint32_t run_cost = 0;
  if (run) {
    const PostRec& p2 = both ? *both : *pp;  // (the second line)
    dmc_decision x;
    x.handle = p2.handle1;
    x.tag_r = p2.r1;
    x.tag_p = p2.p1;
    x.tag_l = p2.l1;
    x.slot = s;
    x.cost = p2.cost1;
    x.phase = DMC_PHASE_RESERVATION;
    x.flags = 0;
    rc.out[d + 1] = x;
    run_cost = x.cost;
  }
  // (a queue group's tallies: the group's first pop -- priority or
  // reservation -- and the run's reservation pop, one update per counter)
  if (rc.tp.d) {
    atomicAdd(&rc.tp.d[s], pr.cost0 + run_cost);
    const uint32_t rr = (prio ? 0u : pr.cost0) + run_cost;
    if (rr) atomicAdd(&rc.tp.r[s], rr);
  }
  uint8_t f = f0 & (uint8_t)~(F_READY | F_PMARK);
  ScanRec o{0.0, 0.0, 0.0, (uint8_t)nh, (uint8_t)nc2, 0, 0, 0};
  if (nc2) {
    o.r = pr.fr;
    o.pk = pr.fpk;
    o.l = pr.fl;
    const uint32_t last = d + run;  // the group's last decision
    const bool seen =
        prio ? (rc.terminal || (rc.g_last != kNoneR && last < rc.g_last)) : rc.p_runs;
    if (seen && (bits & 2u)) f |= F_READY;
  }
  o.flags = f;
  sc_store_front(tb, s, o);
}

// Candidates, one thread each; k_rapply's blocks 2j and 2j + 1 take emit
// block j's segment of the candidate arrays, its last block ends the round
// (the summary to host memory, the device-API result record).  Fast
// candidates store their precomputed state (apply_fast); the others
// (several records, a fast group cut by the round's end, delayed mode,
// limit-break rounds, the radix path) replay their walks
// for exactly the pops the ranking stamped (R pops, then P groups from the
// post-R state), write the decision records and store the new state: ring
// head/count, front cache, reduced reservation tags (immediate: every queued
// request, in order, :1088-1095; delayed: the front, :1077-1085), prev tag,
// and the front's ready flag: a front left by reservation pops only was seen
// by the round's first limit scan iff the priority pulls ran; one left by
// priority pops iff a later limit-scanning pull happened (or the round's
// terminal pull).  (Non-candidates settled their pending marks in k_remit.)
// Block 0 also counts the round's decisions (sched[0] reservation, sched[1]
// priority, :1469,1479).
// apply blocks per emit block (about 70 candidates per 1024 slots in a
// config-3 round)
constexpr uint32_t apply_per_emit(uint32_t chunk) { return chunk >= 4096 ? chunk / 2048 : 1; }
constexpr uint32_t kApplyPerEmit = apply_per_emit(kEmitChunk);
#ifndef DMC_APPLY_PER_EMIT_M
#define DMC_APPLY_PER_EMIT_M 1  // (one apply block per 8,192-slot emit block: config 5 0.778-0.785 against 0.809-0.837 ms at 4, 0.779-0.791 at 2)
#endif
constexpr uint32_t kApplyPerEmitM = DMC_APPLY_PER_EMIT_M;  // (queue groups)
#ifndef DMC_APPLY_MINB
// (apply_one needs ≈164 VGPRs: 2 waves per SIMD, which the grid of two
// 256-thread blocks per CU needs; a higher bound only warns)
#define DMC_APPLY_MINB 2
#endif
// (bid / nblk: the block's index among the apply blocks and their count --
// k_rapply's own grid, or the first nblk blocks of k_apply_link)
template <uint32_t CH = kEmitChunk, uint32_t APE = kApplyPerEmit>
__device__ __attribute__((always_inline)) inline void rapply_body(Table tb, Round* rd, const CandRec* cand, const uint32_t* bcand, const uint32_t* decof, const PostRec* post, unsigned long long* sched, HostRound* h, uint64_t* dbg, uint32_t bid, uint32_t nblk, TallyP tp = TallyP{}) {
  if (rd->skip) return;
  // A limit-break round's priority pops (group heads and their runs'
  // readied fronts) are counted here: its summary goes out once every block
  // has counted (a ticket), not from the extra block at once
  const bool brk = rd->brk && !rd->overflow;
  if (bid == nblk - 1 && !brk) {
    // the extra block publishes the round's summary (complete since k_rrank)
    // to host memory at once: the host learns the outcome while the other
    // blocks store the state, and its next launch is stream-ordered behind them
    rfinish_body(rd, h, true);
    return;
  }
  if (bid == 0 && threadIdx.x == 0 && !rd->overflow && !brk) {
    sched[0] += rd->n_dec - rd->n_prio;
    sched[1] += rd->n_prio;
  }
  if (bid < nblk - 1) {
    // (APE apply blocks per emit block of CH slots)
    const uint32_t eb = bid / APE;
    const uint32_t nc = bcand[eb];
    const uint32_t base = eb * CH;
    RoundC rc{nullptr, rd->now, rd->tick, rd->out, rd->g_last, rd->terminal, rd->k_total,
              rd->p_runs != 0, rd->overflow != 0, brk, &rd->brk_prio, tp};
    __shared__ ReqEntry stage[kBlockR * kApplyStage];
    // (interleaved: the emit block's candidates, about 280, split evenly over
    // its apply blocks rather than filling the first one)
    for (uint32_t i = threadIdx.x * APE + (bid % APE); i < nc; i += APE * kBlockR) {
      const uint32_t ci = base + i;
      uint64_t t0 = dbg ? wall_clock64() : 0;
      // one level of coalesced loads: the candidate, its decision offset and
      // its precomputed state (both lines: a run's second line is no further
      // round trip)
      const CandRec c = cand[ci];
      const uint32_t d = decof[ci];
      if (DMC_POST_LINE1) {
        const PostRec* pp = post + ci;
        const PostL1 pr{pp->fr, pp->fpk, pp->fl, pp->prev_r, pp->off, pp->r2, pp->bits,
                        pp->cand, pp->cost0};
        if (d != kSlowCand && !rc.ovf) {
          apply_fast(tb, rc, c, d, pr, pp, nullptr);
          continue;
        }
      } else {
        const PostRec pr = post[ci];
        if (d != kSlowCand && !rc.ovf) {
          apply_fast(tb, rc, c, d, post_l1(pr), post + ci, &pr);
          continue;
        }
      }
      rc.dbg = (dbg && ci < 65536) ? dbg + 8 * ci : nullptr;
      if (rc.dbg) rc.dbg[1] = rc.dbg[2] = rc.dbg[3] = 0;
      apply_one(tb, rc, c, stage + threadIdx.x * kApplyStage);
      if (rc.dbg) {
        rc.dbg[0] = t0;
        rc.dbg[4] = wall_clock64();
      }
    }
  }
  if (!brk) return;
  // ticket: the block's count atomics have completed (memory side) before
  // one lane takes it; the last block publishes
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&rd->brk_done, 1u) == nblk - 1;
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t np = atomicAdd(&rd->brk_prio, 0u);
    rd->n_prio = np;
    sched[0] += rd->n_dec - np;
    sched[1] += np;
  }
  __syncthreads();
  rfinish_body(rd, h, true);
}
__global__ void __launch_bounds__(kBlockR, DMC_APPLY_MINB)
k_rapply(Table tb, Round* rd, const CandRec* cand, const uint32_t* bcand,
         const uint32_t* decof, const PostRec* post, unsigned long long* sched,
         HostRound* h, uint64_t* dbg = nullptr) {
  rapply_body(tb, rd, cand, bcand, decof, post, sched, h, dbg, blockIdx.x, gridDim.x);
}

__global__ void k_rfinish(const Round* rd, HostRound* h) { rfinish_body(rd, h); }

// ------------------------------------------------------- multi-table rounds
// One launch per kernel over the S server tables of a queue group
// (dmc_group, config 5's per-GPU shape: servers are independent queues,
// sim/src/simulate.h:118-136): blockIdx.y selects the table, whose arguments
// the kernel reads from a device array; blockIdx.x / gridDim.x keep their
// per-table meaning, so each body is exactly the single-table kernel's.
// The latency-bound walkers of all tables overlap, and a step of S servers
// is one graph of seven launches instead of S x seven.
struct RScanArgs {
  Table tb;
  uint64_t *keyr, *keyp;
  uint32_t* meta;
  RoundPart* parts;
  Round* rd;
  CallParams cp;
  uint64_t *skr, *skp;
  uint2* k32;
  uint32_t* hist;
};
struct RHistArgs {
  uint32_t n, nparts;
  const uint64_t *keyr, *keyp;
  const RoundPart* parts;
  Round* rd;
  uint32_t* hist;
  int sampled;
  unsigned long long *bcount, *gsup;
};
struct REmitArgs {
  Table tb;
  Round* rd;
  const uint2* k32;
  const uint32_t* meta;
  CandRec* cand;
  uint32_t* bcand;
  PostRec* post;
  uint32_t* decof;
  BRecR* brec;
  uint32_t* bcount;
  unsigned long long* gsup;
  const uint32_t* hist;
  DEnt* dense;
  uint32_t dcap;
};
struct RRankArgs {
  Round* rd;
  const unsigned long long *bcount, *gsup;
  const BRecR* brec;
  ReqEntry* ring;
  uint32_t* decof;
  TallyP tp;  // the member's tallies (trackers), or none
};
struct RApplyArgs {
  Table tb;
  Round* rd;
  const CandRec* cand;
  const uint32_t *bcand, *decof;
  const PostRec* post;
  unsigned long long* sched;
  HostRound* h;
  TallyP tp;  // the member's tallies (trackers), or none
};

__global__ void __launch_bounds__(kScanBlock, DMC_SCAN_MINW) k_rscan_m(const RScanArgs* a) {
  const RScanArgs& x = a[blockIdx.y];
  rscan_t_body<false>(x.tb, x.keyr, x.keyp, x.meta, x.parts, x.rd, x.cp, x.skr, x.skp, x.k32,
                      x.hist);
}
__global__ void __launch_bounds__(1024) k_rhist_m(const RHistArgs* a) {
  const RHistArgs& x = a[blockIdx.y];
  rhist_body(x.n, x.keyr, x.keyp, x.parts, x.nparts, x.rd, x.hist, x.sampled, x.bcount, x.gsup);
}
// queue groups (kPrePickM): each table's thresholds and rank-bin tables
// picked once, by one block per table, into the histogram buffer's tail and
// the Round's selections, for every k_remit_m block to load
__global__ void __launch_bounds__(kEmitThreads) k_rpick_m(const RHistArgs* a) {
  const RHistArgs& x = a[blockIdx.y];
  Round* rd = x.rd;
  if (rd->skip) return;
  __shared__ uint32_t sbn[2 * kHistBinsR];
  __shared__ PhaseSel s_ph[2];
#if DMC_PICK_WAVE
  const PickW hv = pick_load_w(x.hist, &rd->tot);
  pick_both_w(rd->k_total, hv, sbn, s_ph, (int)rd->sampled, rd->fault);
#else
  const PickBins hv = pick_load(x.hist);
  pick_both(rd->k_total, rd->tot, hv, sbn, s_ph, (int)rd->sampled, rd->fault);
#endif
  for (int i = threadIdx.x; i < 2 * kHistBinsR / 4; i += kEmitThreads)
    st_as(x.hist + kShards * 2 * kHistBinsR + 4 * i, ld_as<uint4>(sbn + 4 * i));
  if (threadIdx.x < 2) rd->ph[threadIdx.x] = s_ph[threadIdx.x];
}
__global__ void __launch_bounds__(kEmitThreads, DMC_EMIT_MINW) k_remit_m(const REmitArgs* a) {
  const REmitArgs& x = a[blockIdx.y];
  remit_t_body<false, kPrePickM, kEmitPerM, kEmitStageThreadsM>(x.tb, x.rd, x.k32, x.meta, x.cand, x.bcand, x.post, x.decof,
                                 x.brec, x.bcount, x.gsup, x.hist, x.dense, x.dcap, nullptr);
}
// Queue groups, split emission (DMC_SPLIT_EMIT_M): k_remit_m's two halves
// as two launches.  A k_remit_m block (one per CU: its candidate list and
// ring staging fill the LDS) walks the few candidates of its 4,096 slots
// (about 140 per table block at config 5's 2M slots: eight per wave) before
// the next block may start, so a group's 4,096 emit blocks ran in sixteen
// generations, each as long as one walk.  Here the selection streams the
// keys and writes each block's candidates (and each candidate's first-key
// quantum, in decof until the walk replaces it) with small LDS, and the
// walks run in blocks of kWalkThreads with one staging slice per thread:
// several blocks per CU, many walks in flight.  The records, their order
// and every state change are k_remit_m's (the same emit_one).
#ifndef DMC_SPLIT_EMIT_M
#define DMC_SPLIT_EMIT_M 0
#endif
static_assert(!DMC_SPLIT_EMIT_M || kEmitPerM == kEmitPer,
              "the split emission's blocks are kEmitChunk wide: build it with DMC_EMIT_PER_M = DMC_EMIT_PER");
#ifndef DMC_WALK_THREADS
#define DMC_WALK_THREADS 128
#endif
constexpr int kWalkThreads = DMC_WALK_THREADS;
__device__ __attribute__((always_inline)) inline void rsel_body(Table tb, Round* rd, const uint2* k32, const uint32_t* meta, CandRec* cand, uint32_t* bcand, uint32_t* decof) {
  if (rd->skip) return;
  __shared__ uint32_t s_tot;
  __shared__ uint32_t s_cnt[2];
  __shared__ PhaseSel s_ph[2];
  if (threadIdx.x < 2) {
    s_cnt[threadIdx.x] = 0;
    s_ph[threadIdx.x] = rd->ph[threadIdx.x];
  }
  if (threadIdx.x == 0) s_tot = 0;
  const uint32_t n = tb.n;
  const uint32_t s0 = blockIdx.x * kEmitChunk + threadIdx.x * kEmitPer;
  const bool p_runs = rd->p_runs != 0;
  const int lane = threadIdx.x & 63;
  uint32_t kr[kEmitPer], kp[kEmitPer], mt[kEmitPer];
  if (s0 + kEmitPer <= n) {
#pragma unroll
    for (int j = 0; j < kEmitPer / 2; ++j) {
      const uint4 a = ld_as<uint4>(k32 + s0 + 2 * j);
      kr[2 * j] = a.x; kp[2 * j] = a.y; kr[2 * j + 1] = a.z; kp[2 * j + 1] = a.w;
    }
#pragma unroll
    for (int j = 0; j < kEmitPer / 4; ++j) {
      const uint4 m = ld_as<uint4>(meta + s0 + 4 * j);
      mt[4 * j] = m.x; mt[4 * j + 1] = m.y; mt[4 * j + 2] = m.z; mt[4 * j + 3] = m.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kEmitPer; ++j) {
      const bool in = s0 + j < n;
      const uint2 k = in ? k32[s0 + j] : make_uint2(0xffffffffu, 0xffffffffu);
      kr[j] = k.x;
      kp[j] = k.y;
      mt[j] = in ? meta[s0 + j] : 0;
    }
  }
  __syncthreads();  // (s_ph, s_cnt, s_tot)
  const CandPred pred(s_ph, p_runs);
  uint32_t bits = 0, cnt = 0, nr = 0, np = 0;
#pragma unroll
  for (int j = 0; j < kEmitPer; ++j) {
    if (s0 + j >= n) continue;
    const bool cr = pred.TR && kr[j] <= pred.TR32;
    const bool cp = pred.TP && kp[j] <= pred.TP32;
    if (cr || cp) bits |= ((cr ? 1u : 0u) | (cp ? 2u : 0u)) << (2 * j);
    cnt += (cr || cp) ? 1u : 0u;
    nr += cr ? 1u : 0u;
    np += cp ? 1u : 0u;
  }
  const bool sampled = rd->sampled != 0;
  if (sampled) {
    nr = wsum_all(nr);
    np = wsum_all(np);
    if (lane == 0) {
      atomicAdd(&s_cnt[0], nr);
      atomicAdd(&s_cnt[1], np);
    }
  }
  const uint32_t incl = wscan_u32(cnt);
  const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  uint32_t wbase = 0;
  if (lane == 0 && wtot) wbase = atomicAdd(&s_tot, wtot);
  wbase = __shfl(wbase, 0);
  const uint32_t cbase = blockIdx.x * kEmitChunk;
  uint32_t o = wbase + incl - cnt;
#pragma unroll
  for (int j = 0; j < kEmitPer; ++j) {
    const uint32_t b = (bits >> (2 * j)) & 3u;
    const uint8_t f = (uint8_t)(mt[j] >> 8);
    if (b) {
      cand[cbase + o] = CandRec{s0 + j, (uint8_t)(f | (b << 4)), (uint8_t)mt[j],
                                (uint8_t)(mt[j] >> 16), (uint8_t)(mt[j] >> 24)};
      decof[cbase + o] = (b & 1u) ? kr[j] : kp[j];  // (the walk's first-key quantum)
      ++o;
    } else if (s0 + j < n && (f & F_PMARK)) {
      // a non-candidate settles its pending limit-scan mark
      tb.sc[s0 + j].flags = (uint8_t)((f & ~F_PMARK) | (p_runs ? F_READY : 0));
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bcand[blockIdx.x] = s_tot;
    if (s_tot) atomicAdd(&rd->n_cand, s_tot);
    if (sampled) {
      uint32_t* cc = rd->ccnt + 2 * (blockIdx.x % kCntShards);
      if (s_cnt[0]) atomicAdd(&cc[0], s_cnt[0]);
      if (s_cnt[1]) atomicAdd(&cc[1], s_cnt[1]);
    }
  }
}
// the walks of emit block `seg`'s candidates (blockIdx.x = seg)
__device__ __attribute__((always_inline)) inline void rwalk_body(Table tb, Round* rd, const CandRec* cand, const uint32_t* bcand, PostRec* post, uint32_t* decof, BRecR* brec, uint32_t* bcount, unsigned long long* gsup, const uint32_t* hist, DEnt* dense, uint32_t dcap) {
  if (rd->skip) return;
  __shared__ uint32_t ltab[2 * kHistBinsR];
  __shared__ PhaseSel s_ph[2];
  __shared__ unsigned long long s_sup[kNSup];
  __shared__ uint32_t s_ec[4];
  __shared__ ReqEntry stage[kWalkThreads * kEmitStage];
  const uint32_t seg = blockIdx.x;
  const uint32_t tot = bcand[seg];
  if (tot == 0) return;
  for (int i = threadIdx.x; i < 2 * kHistBinsR / 4; i += kWalkThreads)
    st_as(ltab + 4 * i, ld_as<uint4>(hist + kShards * 2 * kHistBinsR + 4 * i));
  if (threadIdx.x < 2) s_ph[threadIdx.x] = rd->ph[threadIdx.x];
  if (threadIdx.x < kNSup) s_sup[threadIdx.x] = 0;
  if (threadIdx.x < 4) s_ec[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t cbase = seg * kEmitChunk;
  const double now_w = rd->now;
  for (uint32_t i = threadIdx.x; i < tot; i += kWalkThreads) {
    const uint32_t ci = cbase + i;
    const CandRec c = cand[ci];
    const uint32_t key0 = decof[ci];
    const uint32_t cat = emit_one<false>(tb, rd, now_w, s_ph, c, ci, brec, bcount, s_sup, ltab, dense,
                                         dcap, post, decof, stage + threadIdx.x * kEmitStage,
                                         key0);
    atomicAdd(&s_ec[cat], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 4 && s_ec[threadIdx.x]) atomicAdd(&rd->ecnt[threadIdx.x], s_ec[threadIdx.x]);
  if (brec && threadIdx.x < kNSup && s_sup[threadIdx.x])
    atomicAdd(&gsup[threadIdx.x], s_sup[threadIdx.x]);
}
__global__ void __launch_bounds__(kEmitThreads) k_rsel_m(const REmitArgs* a) {
  const REmitArgs& x = a[blockIdx.y];
  rsel_body(x.tb, x.rd, x.k32, x.meta, x.cand, x.bcand, x.decof);
}
__global__ void __launch_bounds__(kWalkThreads) k_rwalk_m(const REmitArgs* a) {
  const REmitArgs& x = a[blockIdx.y];
  rwalk_body(x.tb, x.rd, x.cand, x.bcand, x.post, x.decof, x.brec, x.bcount, x.gsup, x.hist,
             x.dense, x.dcap);
}

__global__ void __launch_bounds__(kRankThreads) k_rrank_m(const RRankArgs* a) {
  const RRankArgs& x = a[blockIdx.y];
  rrank_body(x.rd, x.bcount, x.gsup, x.brec, x.ring, x.decof, nullptr, x.tp);
}
__global__ void __launch_bounds__(kBlockR, DMC_APPLY_MINB) k_rapply_m(const RApplyArgs* a) {
  const RApplyArgs& x = a[blockIdx.y];
  rapply_body<kEmitChunkM, kApplyPerEmitM>(x.tb, x.rd, x.cand, x.bcand, x.decof, x.post, x.sched, x.h, nullptr,
                           blockIdx.x, gridDim.x, x.tp);
}

// device-API result written by the host's view of a multi-round call
__global__ void k_put_result(dmc_pull_result* res, dmc_pull_result r) { *res = r; }

}  // namespace dmc
