// SPDX-License-Identifier: LGPL-2.1
//
// dmc_heap.h -- tie-exact dispatch (DMC_OPT_HEAP_ORDER): the reference's
// three indirect heaps kept on the device and driven in the reference's
// order, so that among equal keys the winner is the reference's heap top.
//
// The engine's rounds break ties by lowest slot: the
// reference's winner among equal keys is whichever tied client sits at index
// 0 of its IndIntruHeap, a function of every sift since the queue was built
// (support/src/indirect_intrusive_heap.h:240-564; comparators
// src/dmclock_server.h:722-757).  No client attribute predicts it, so a
// caller that needs the reference's exact dispatch sequence on tie-heavy
// traces turns this mode on: every add and pull then runs in call order on
// one wave of the device.
//
// Layout (per heap h = resv, limit, ready): `ent[h][i]`, the heap array of
// 16-byte entries {ordered key, class, slot} -- the client's comparison key
// kept inline, so a compare needs no load of the client's record -- and
// `hix[h][slot]`, each slot's index (IndIntruHeap's intrusive index).  An
// entry is a pure function of the slot's ScanRec (hent): whenever a kernel
// here changes a ScanRec it rewrites the slot's three entries, sifted or in
// place, before anything compares against them, so every comparison sees
// what the reference's comparator would read from the client record.
//
// Sifts are wave-parallel but make exactly the reference's moves.  A
// sift_down loads the whole subtree of the next D levels below the moving
// element at once (62 entries for K = 2: one lane each) and resolves the
// path in registers, IndIntruHeap's rule at each level (the first smallest
// child, moved up iff strictly less, :479-548); a sift_up loads every
// ancestor at once and moves up while strictly less (:462-474); sift
// (:550-564) loads the ancestors and the first subtree together and picks
// the direction from the parent.  One dependent memory round trip per D
// levels instead of two per level.
//
// Heap order per operation (what the reference calls, in its order):
//   register      resv.push, limit.push, ready.push            (:925-931)
//   add           the idle reset (:937-985); initial_tag; Reject returns
//                 before any heap call (:989-993); a first request adjusts
//                 the three heaps (:996-1006), every accepted one again
//                 (:1011-1016)
//   pull          the resv top if due (:1124-1128); the limit loop's ready
//                 marks with ready.promote / limit.demote (:1135-1144); the
//                 ready top if ready (:1146-1151); Allow's fallbacks
//                 (:1157-1165); future / none (:1170-1185).  A pop
//                 (:1046-1073): pop the front, update_next_tag, then
//                 resv.demote, limit.adjust, ready.demote; a priority pop
//                 then reduce_reservation_tags and resv.promote (:1098-1111)
//   erase         resv, limit, ready remove (delete_from_heaps, :1259-1275)
//   filter, remove_by_client   adjust x 3 for each modified client (:567-625)
// (included by dmc_engine.hip inside its anonymous namespace, after the
// step path's helpers)
#pragma once

enum : int { kHResv = 0, kHLim = 1, kHReady = 2 };

// A heap entry: ClientCompare's order (:722-757) as (cls, key) ascending.
//   resv:  cls 0 = has a request, key r
//   limit: cls 0 = has a request and not ready, 1 = ready (ReadyOption::lowers), key l
//   ready: cls 0 = has a request and ready, 1 = not ready (raises), key p + prop_delta
//   no request: cls 3, key 0 (such clients compare equal: neither is less)
// key = okey(v) with -0.0 read as +0.0 (the comparator's `<` does not order
// them).  Tags are never NaN (make_tag refuses none of them; a NaN arrival
// time is outside the reference's contract).
struct alignas(16) HEnt {
  uint64_t key;
  uint32_t cls;
  uint32_t slot;
};
static_assert(sizeof(HEnt) == 16, "HEnt must be 16 bytes");
constexpr uint32_t kClsNone = 3;
// entries of each heap kept in LDS while a heap kernel runs: the top 11
// levels of a binary heap (3 x 32 KB); a sift from the root then reaches
// memory only below them
#ifndef DMC_HEAP_LDS
#define DMC_HEAP_LDS 2047
#endif
constexpr uint32_t kHeapLds = DMC_HEAP_LDS;

// (DMC_HEAP_DP: a priority pop's resv demote + promote as one operation,
// k2_demote_promote; 0: the two sifts in turn)
#ifndef DMC_HEAP_DP
#define DMC_HEAP_DP 1
#endif
// (debug, DMC_HEAP_CLOCKS: shader-clock cycles per phase, printed by
// k_heap_pull)
#ifndef DMC_HEAP_CLOCKS
#define DMC_HEAP_CLOCKS 0
#endif

struct HeapDev {
  HEnt* ent;      // [3][n] heap arrays
  uint32_t* hix;  // [3][n] each slot's index in each heap
  uint32_t* cnt;  // [3] heap sizes
  uint32_t n, k;  // capacity, branching (IndIntruHeap's K)
};

__device__ inline uint64_t okey0(double v) { return okey(v == 0.0 ? 0.0 : v); }
__device__ inline double hval(const HEnt& e) { return from_okey(e.key); }

__device__ inline HEnt hent(int h, const ScanRec& r, uint32_t s) {
  HEnt e;
  e.slot = s;
  if (!r.count) {
    e.key = 0;
    e.cls = kClsNone;
    return e;
  }
  const bool rdy = (r.flags & F_READY) != 0;
  if (h == kHResv) {
    e.key = okey0(r.r);
    e.cls = 0;
  } else if (h == kHLim) {
    e.key = okey0(r.l);
    e.cls = rdy ? 1u : 0u;
  } else {
    e.key = okey0(r.pk);
    e.cls = rdy ? 0u : 1u;
  }
  return e;
}

// strict less (ClientCompare)
__device__ inline bool hlt(const HEnt& a, const HEnt& b) {
  return a.cls < b.cls || (a.cls == b.cls && a.key < b.key);
}

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// one lane's entry, wave-uniform
__device__ inline HEnt hread(const HEnt& e, uint32_t lane) {
  HEnt o;
  const uint32_t lo = (uint32_t)e.key, hi = (uint32_t)(e.key >> 32);
  o.key = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, (int)lane) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, (int)lane) << 32);
  o.cls = (uint32_t)__builtin_amdgcn_readlane((int)e.cls, (int)lane);
  o.slot = (uint32_t)__builtin_amdgcn_readlane((int)e.slot, (int)lane);
  return o;
}
__device__ inline uint32_t uread(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
__device__ inline double dread(double v, uint32_t lane) {
  const uint64_t u = dbits(v);
  return bitsd((uint64_t)uread((uint32_t)u, lane) | ((uint64_t)uread((uint32_t)(u >> 32), lane) << 32));
}
// lane 0's stores before the wave's later loads (same wave, other lanes)
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One heap of IndIntruHeap's algorithms, driven by all 64 lanes of a wave
// with uniform arguments; every function returns the moving element's final
// index.  Only lanes' own loads and stores differ.
struct WHeap {
  HEnt* a;        // the heap array
  uint32_t* x;    // slot -> index
  uint32_t k;     // branching
  uint32_t lane;
  HEnt* c;        // the LDS copy of a[0, T): the heap's top levels (heap_cache_fill)
  uint32_t T;

  // LDS and memory each through its own address space: ds_read / ds_write
  // and global_load / global_store.  (Through one generic pointer the two
  // merge into flat accesses, and a flat load may alias a pending flat
  // store in either memory: every round would wait for the previous round's
  // stores to complete before issuing its loads.)
  __device__ __forceinline__ HEnt ld(uint32_t i) const {
    if (i < T) return ld_lds<HEnt>(c + i);
    return ld_glb<HEnt>(a + i);
  }
  __device__ __forceinline__ void st(uint32_t i, const HEnt& e) const {
    if (i < T) st_lds(c + i, e);
    else st_glb(a + i, e);
  }
  __device__ __forceinline__ void put(uint32_t i, const HEnt& e) const {  // (uniform: lane 0 stores)
    if (lane == 0) {
      st(i, e);
      x[e.slot] = i;
    }
  }

  // lanes [base, 64) as the levels 1..D below a root: lane -> (level, offset)
  // and the node's index from the root's; D = the levels that fit
  struct Sub {
    uint32_t lv, off, D;
    uint64_t pw, g;  // K^lv, 1 + K + ... + K^(lv-1)
  };
  __device__ __forceinline__ Sub layout(uint32_t base) const {
    Sub L{0, 0, 0, 1, 0};
    uint32_t avail = lane >= base ? 64u : 0u;
    // D: levels whose lanes all fit in [base, 64)
    uint64_t pw = k, used = 0, g = 1;
    for (uint32_t l = 1; l <= 32; ++l) {
      if (used + pw > 64 - base) break;
      L.D = l;
      if (avail && lane - base >= used && lane - base < used + pw) {
        L.lv = l;
        L.off = lane - base - (uint32_t)used;
        L.pw = pw;
        L.g = g;
      }
      used += pw;
      g += pw;
      pw *= k;
    }
    return L;
  }
  // first lane of level l's block (levels 1..D, from `base`)
  __device__ __forceinline__ uint32_t level_lane(uint32_t base, uint32_t l) const {
    uint32_t u = 0;
    uint64_t pw = k;
    for (uint32_t t = 1; t < l; ++t) {
      u += (uint32_t)pw;
      pw *= k;
    }
    return base + u;
  }

  // the subtree below root r (this lane's node, if any and < n)
  __device__ __forceinline__ HEnt sub_load(const Sub& L, uint32_t r, uint32_t n, uint32_t* idx) const {
    HEnt e{~0ull, kClsNone + 1, 0};
    *idx = 0xffffffffu;
    if (L.lv) {
      const uint64_t i = L.pw * (uint64_t)r + L.g + L.off;
      if (i < n) {
        *idx = (uint32_t)i;
        e = ld((uint32_t)i);
      }
    }
    return e;
  }

  // sift_down of X from i over the loaded subtree (lanes [base, 64), D
  // levels): IndIntruHeap's moves; the moved lanes store themselves one
  // level up.  Returns true when X went below the subtree's last level
  // (*i is then the node to continue from).
  __device__ __forceinline__ bool down_sub(const Sub& L, uint32_t base, const HEnt& e, uint32_t eidx, uint32_t n,
                           const HEnt& X, uint32_t* i) const {
    uint32_t c = *i, co = 0;
    uint32_t tgt = 0xffffffffu;
    bool cont = true;
    for (uint32_t l = 0; l < L.D; ++l) {
      const uint64_t li = (uint64_t)k * c + 1;
      if (li >= n) {
        cont = false;
        break;
      }
      const uint32_t nc = (uint32_t)min((uint64_t)k, n - li);
      const uint32_t l0 = level_lane(base, l + 1) + co * k;
      uint32_t mj = 0;
      HEnt mb = hread(e, l0);
      for (uint32_t j = 1; j < nc; ++j) {
        const HEnt cj = hread(e, l0 + j);
        if (hlt(cj, mb)) {
          mb = cj;
          mj = j;
        }
      }
      if (!hlt(mb, X)) {
        cont = false;
        break;
      }
      if (lane == l0 + mj) tgt = c;
      c = (uint32_t)li + mj;
      co = co * k + mj;
    }
    if (tgt != 0xffffffffu) {
      st(tgt, e);
      x[e.slot] = tgt;
    }
    (void)eidx;
    *i = c;
    return cont && L.D > 0;
  }

  // sift_down (:479-548) of X from i, n = the count it sees
  __device__ __forceinline__ uint32_t sift_down(uint32_t i, uint32_t n, const HEnt& X) const {
    if (k == 2) return k2_sift_down(i, n, X);
    if (i < n) {
      const Sub L = layout(0);
      for (;;) {
        uint32_t eidx;
        const HEnt e = sub_load(L, i, n, &eidx);
        if (!down_sub(L, 0, e, eidx, n, X, &i)) break;
      }
    }
    put(i, X);
    return i;
  }

  // ancestor t + 1 of i (lanes t < depth): index, and the depth of i
  __device__ __forceinline__ uint32_t ancestors(uint32_t i, uint32_t* anc) const {
    uint32_t d = 0, p = i, my = 0;
    while (p > 0) {
      p = k == 2 ? (p - 1) >> 1 : (p - 1) / k;
      if (lane == d) my = p;
      ++d;
    }
    *anc = my;
    return d;
  }

  // sift_up (:462-474) of X from i over the loaded ancestors (lane t holds
  // ancestor t + 1, t < d): X passes the leading run of ancestors it is
  // strictly less than, each moving down one node of the path
  __device__ __forceinline__ uint32_t up_anc(uint32_t i, const HEnt& X, uint32_t d, uint32_t anc,
                             const HEnt& ae, uint32_t* pm = nullptr) const {
    const bool lt = lane < d && hlt(X, ae);
    const uint64_t bal = __ballot(lt);
    const uint32_t m = (uint32_t)__builtin_ctzll(~bal);
    if (pm) *pm = m;
    uint32_t dst = (uint32_t)__shfl_up((int)anc, 1);  // the path's node below it
    if (lane == 0) dst = i;
    if (lane < m) {
      st(dst, ae);
      x[ae.slot] = dst;
    }
    const uint32_t f = m ? uread(anc, m - 1) : i;
    put(f, X);
    return f;
  }

  __device__ __forceinline__ uint32_t sift_up(uint32_t i, const HEnt& X) const {
    uint32_t anc;
    const uint32_t d = k == 2 ? k2_ancestors(i, &anc) : ancestors(i, &anc);
    HEnt ae{~0ull, kClsNone + 1, 0};
    if (lane < d) ae = ld(anc);
    return up_anc(i, X, d, anc, ae);
  }

  // ---- K = 2 (the reference's default): a fixed subtree layout -- lane j <
  // 62 holds node (level L = log2(j + 2), offset j + 2 - 2^L) of the five
  // levels below the root, whose index is ((r + 1) << L) - 1 + offset; lane
  // j's children are lanes 2j + 2 and 2j + 3.  Each lane j < 30 loads its
  // two children as well as its node, and lane 62 the root's two children
  // (lanes 0 and 1): every lane picks its smaller child (IndIntruHeap's K ==
  // 2 rule: the right one only if strictly less, :514-548) and whether it
  // moves up past X, and the path is walked on the two ballots in scalar
  // registers.
  __device__ __forceinline__ uint32_t k2_lv() const {
    return lane < 62 ? 31u - __builtin_clz(lane + 2) : 0u;
  }
  // this lane's node below root r (~0: none, or >= n)
  __device__ __forceinline__ uint32_t k2_idx(uint32_t r, uint32_t n) const {
    const uint32_t L = k2_lv();
    if (!L) return 0xffffffffu;
    const uint64_t i = (((uint64_t)r + 1) << L) - 1 + (lane + 2 - (1u << L));
    return i < n ? (uint32_t)i : 0xffffffffu;
  }
  // one round's loads below root r: the lane's node and the children it
  // compares (one round trip: three loads per lane)
  struct K2Sub {
    HEnt e, lc, rc;
    uint32_t idx;
    bool hasl, hasr;
  };
  __device__ __forceinline__ K2Sub k2_load(uint32_t r, uint32_t n) const {
    K2Sub s;
    s.e = s.lc = s.rc = HEnt{~0ull, kClsNone + 1, 0};
    s.idx = k2_idx(r, n);
    // the node whose children this lane compares (lanes < 30: its own; 62: r)
    const bool own = lane < 30 && s.idx != 0xffffffffu;
    const uint64_t li = 2ull * (own ? s.idx : r) + 1;
    s.hasl = (own || lane == 62) && li < n;
    s.hasr = s.hasl && li + 1 < n;
    if (s.idx != 0xffffffffu) s.e = ld(s.idx);
    if (s.hasl) s.lc = ld((uint32_t)li);
    if (s.hasr) s.rc = ld((uint32_t)li + 1);
    return s;
  }
  // the path of X down the loaded subtree below r (*moved: its lanes,
  // which move up one level); returns true when X passed the subtree's last
  // level (*r is then the node to continue from), else X's node in *r
  __device__ __forceinline__ bool k2_path(const K2Sub& s, const HEnt& X, uint32_t* r,
                                          uint64_t* moved) const {
    const bool pickr = s.hasr && hlt(s.rc, s.lc);
    const bool mv = s.hasl && hlt(pickr ? s.rc : s.lc, X);
    const uint64_t M = __ballot(mv), P = __ballot(pickr);
    *moved = 0;
    if (!((M >> 62) & 1ull)) return false;  // (X stays at r)
    uint32_t c = (uint32_t)((P >> 62) & 1ull);
    uint64_t m = 1ull << c;
    bool cont = true;
    for (int L = 1; L < 5; ++L) {
      if (!((M >> c) & 1ull)) {
        cont = false;
        break;
      }
      c = 2 * c + 2 + (uint32_t)((P >> c) & 1ull);
      m |= 1ull << c;
    }
    *moved = m;
    *r = uread(s.idx, c);
    return cont;
  }
  // the moved lanes' entries one level up
  __device__ __forceinline__ void k2_move(const K2Sub& s, uint64_t moved) const {
    if ((moved >> lane) & 1ull) {
      const uint32_t pi = (s.idx - 1) >> 1;
      st(pi, s.e);
      x[s.e.slot] = pi;
    }
  }
  // sift_down of X from i, whose first subtree is loaded (a).  Software
  // pipelined: a round's path decided, the next round's loads are issued
  // before the round's moves are stored, into the other of two buffers --
  // a load into registers that a pending store still reads would first
  // wait for that store, and a load wait waits for the stores issued before
  // it (one memory counter for both): so each round costs one round trip,
  // the stores' and the loads' overlapped.
  __device__ __forceinline__ uint32_t k2_sift_down_from(K2Sub a, uint32_t i, uint32_t n,
                                                        const HEnt& X) const {
    K2Sub b;
    uint64_t mv;
    for (;;) {
      uint32_t ni = i;
      const bool ca = k2_path(a, X, &ni, &mv);
      if (ca) b = k2_load(ni, n);
      k2_move(a, mv);
      i = ni;
      if (!ca) break;
      const bool cb = k2_path(b, X, &ni, &mv);
      if (cb) a = k2_load(ni, n);
      k2_move(b, mv);
      i = ni;
      if (!cb) break;
    }
    put(i, X);
    return i;
  }
  __device__ __forceinline__ uint32_t k2_sift_down(uint32_t i, uint32_t n, const HEnt& X) const {
    if (i >= n) {
      put(i, X);
      return i;
    }
    return k2_sift_down_from(k2_load(i, n), i, n, X);
  }
  // ancestors of i: lane t < d holds ancestor t + 1, ((i + 1) >> (t + 1)) - 1
  __device__ __forceinline__ uint32_t k2_ancestors(uint32_t i, uint32_t* anc) const {
    const uint32_t d = 31u - __builtin_clz(i + 1);
    *anc = lane < d ? ((i + 1) >> (lane + 1)) - 1 : 0u;
    return d;
  }
  __device__ __forceinline__ uint32_t k2_sift(uint32_t i, uint32_t n, const HEnt& X) const {
    if (i == 0) return k2_sift_down(i, n, X);
    uint32_t anc;
    const uint32_t d = k2_ancestors(i, &anc);
    // the ancestors and the first subtree in one round trip
    HEnt ae{~0ull, kClsNone + 1, 0};
    if (lane < d) ae = ld(anc);
    const K2Sub sub = k2_load(i, n);  // (nothing when i >= n)
    if (hlt(X, hread(ae, 0))) return up_anc(i, X, d, anc, ae);
    if (i >= n) {
      put(i, X);
      return i;
    }
    return k2_sift_down_from(sub, i, n, X);
  }
  // The moved lanes of one demote round appended to the path registers
  // (lane k: path node p_k's index and entry before the demote; p_0 = the
  // start).  A round's moved lanes are one per level, in lane order.
  __device__ __forceinline__ void k2_rec_path(const K2Sub& s, uint64_t mv, uint32_t* m,
                                              uint32_t* pI, HEnt* pE) const {
    while (mv) {
      const uint32_t c = (uint32_t)__builtin_ctzll(mv);
      mv &= mv - 1;
      const uint32_t k = ++*m;
      const HEnt e = hread(s.e, c);
      const uint32_t ix = uread(s.idx, c);
      if (lane == k) {
        *pE = e;
        *pI = ix;
      }
    }
  }
  // resv.demote of the popped client's entry (Xd: its new front, unreduced,
  // :1063) and then resv.promote of the same entry (Xu: reduced, :1110),
  // as one operation.  The demote's rounds store nothing and keep the path
  // in registers; the promote's ancestors are that path (with the values
  // the demote moved into it) followed by i's ancestors, loaded with the
  // demote's first subtree -- so the promote needs no round trip -- and
  // each changed node is stored once, with its value after both calls.
  // Along the chain N_0 = the demote's end f, N_u = f's ancestor u: after
  // the demote N_0 holds Xd and N_u (u <= m, m = the levels it moved) the
  // entry that was at N_{u-1}; the promote passes the first m' of them,
  // each moving down one node.  So N_u ends with N_{u+1}'s value (u < m'),
  // Xu (u = m') or its post-demote value (u > m'), and a node is stored
  // iff that differs from what memory holds: u = m', m' < u <= m, or
  // m <= u < m' (for u < min(m, m') it is N_u's entry before both).
  __device__ __forceinline__ uint32_t k2_demote_promote(uint32_t i, uint32_t n, const HEnt& Xd,
                                                        const HEnt& Xu) const {
    uint32_t anc;
    const uint32_t d = k2_ancestors(i, &anc);
    HEnt ae{~0ull, kClsNone + 1, 0};
    if (lane < d) ae = ld(anc);
    uint32_t pI = lane == 0 ? i : 0u, m = 0, f = i;
    HEnt pE{~0ull, kClsNone + 1, 0};
    if (i < n) {
      K2Sub a = k2_load(i, n), b;
      uint64_t mv;
      for (;;) {
        uint32_t ni = f;
        const bool ca = k2_path(a, Xd, &ni, &mv);
        if (ca) b = k2_load(ni, n);
        k2_rec_path(a, mv, &m, &pI, &pE);
        f = ni;
        if (!ca) break;
        const bool cb = k2_path(b, Xd, &ni, &mv);
        if (cb) a = k2_load(ni, n);
        k2_rec_path(b, mv, &m, &pI, &pE);
        f = ni;
        if (!cb) break;
      }
    }
    // the chain: lane t holds N_{t+1} -- t < m: p_{m-1-t} with p_{m-t}'s
    // entry; t >= m: i's ancestor t - m + 1 (lane t - m of anc / ae)
    const uint32_t D = m + d;
    const bool onp = lane < m;
    const int s1 = (int)((onp ? m - 1 - lane : 0u) << 2), s2 = (int)((onp ? m - lane : 0u) << 2);
    const int s3 = (int)((!onp && lane < D ? lane - m : 0u) << 2);
    auto bp = [](int src, uint32_t v) {
      return (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)v);
    };
    auto bpe = [&](int src, const HEnt& e) {
      HEnt o;
      o.key = (uint64_t)bp(src, (uint32_t)e.key) | ((uint64_t)bp(src, (uint32_t)(e.key >> 32)) << 32);
      o.cls = bp(src, e.cls);
      o.slot = bp(src, e.slot);
      return o;
    };
    const uint32_t pIx = bp(s1, pI), aIx = bp(s3, anc);
    const HEnt pEx = bpe(s2, pE), aEx = bpe(s3, ae);
    uint32_t cI = onp ? pIx : aIx;
    HEnt cV = onp ? pEx : aEx;
    if (lane >= D) cV = HEnt{~0ull, kClsNone + 1, 0};
    // the promote: Xu passes the leading run of chain entries it is less than
    const uint64_t bal = __ballot(lane < D && hlt(Xu, cV));
    const uint32_t mp = (uint32_t)__builtin_ctzll(~bal);
    // lane u: node N_u (lane u - 1's chain node; N_0 = f holding Xd)
    const int su = (int)((lane ? lane - 1 : 0u) << 2);
    uint32_t nI = bp(su, cI);
    HEnt nV = bpe(su, cV);
    if (lane == 0) {
      nI = f;
      nV = Xd;
    }
    const bool store = lane == mp || (lane > mp && lane <= m) || (lane >= m && lane < mp);
    const HEnt F = lane < mp ? cV : lane == mp ? Xu : nV;
    if (store) {
      st(nI, F);
      x[F.slot] = nI;
    }
    return uread(nI, mp);
  }
  // ---- signalled forms (k_heap_pull_async's heap waves): sig() is called
  // exactly once, as soon as the heap's top (index 0, in LDS) holds its
  // value after this call; the rest of the sift runs on behind it.
  // sift_down (:479-548): from i > 0 it cannot change the top
  template <typename F>
  __device__ __forceinline__ uint32_t k2_sift_down_sig(uint32_t i, uint32_t n, const HEnt& X,
                                                       F sig) const {
    if (i != 0 || i >= n) {
      sig();
      return k2_sift_down(i, n, X);
    }
    K2Sub a = k2_load(0, n), b;
    uint32_t ni = 0;
    uint64_t mv;
    const bool ca = k2_path(a, X, &ni, &mv);
    if (ca) b = k2_load(ni, n);
    k2_move(a, mv);  // (the root's new entry, when X moved)
    if (!mv) {
      put(0, X);
      sig();
      return 0;
    }
    sig();
    if (!ca) {
      put(ni, X);
      return ni;
    }
    return k2_sift_down_from(b, ni, n, X);
  }
  // sift (:550-564): the top changes only when X climbs to it
  template <typename F>
  __device__ __forceinline__ uint32_t k2_sift_sig(uint32_t i, uint32_t n, const HEnt& X, F sig) const {
    if (i == 0) return k2_sift_down_sig(i, n, X, sig);
    uint32_t anc;
    const uint32_t d = k2_ancestors(i, &anc);
    HEnt ae{~0ull, kClsNone + 1, 0};
    if (lane < d) ae = ld(anc);
    const K2Sub sub = k2_load(i, n);
    if (hlt(X, hread(ae, 0))) {
      const uint32_t f = up_anc(i, X, d, anc, ae);
      sig();
      return f;
    }
    sig();
    if (i >= n) {
      put(i, X);
      return i;
    }
    return k2_sift_down_from(sub, i, n, X);
  }
  // k2_sift, and whether a second sift of the same X right after it
  // provably moves nothing (*settled; the add path's two adjusts of a
  // client's first request, :996-1016).  After a sift down (or no move) X's
  // node has no child less than X (where the walk stopped) and a parent X is
  // not less than (the entry that moved up past X, or the parent checked
  // first).  After a sift up to ancestor m its parent stopped the climb, and
  // its children are the node below it on the path -- now holding the entry
  // X passed, which X is less than -- and that node's sibling, loaded here
  // with the ancestors: settled iff the sibling is not less than X.
  // (Whether the heap is otherwise in order does not matter: only X's own
  // node and neighbours decide what the second sift does.)
  __device__ __forceinline__ uint32_t k2_sift_s(uint32_t i, uint32_t n, const HEnt& X,
                                                bool* settled) const {
    *settled = true;
    if (i == 0) return k2_sift_down(i, n, X);
    uint32_t anc;
    const uint32_t d = k2_ancestors(i, &anc);
    HEnt ae{~0ull, kClsNone + 1, 0}, sb = ae;
    if (lane < d) ae = ld(anc);
    // lane d + t: the sibling of path node t (i's ancestor t, t = 0: i)
    if (lane >= d && lane < 2 * d) {
      const uint32_t a = ((i + 1) >> (lane - d)) - 1;
      const uint32_t si = (a & 1u) ? a + 1 : a - 1;
      if (si < n) sb = ld(si);
    }
    const K2Sub sub = k2_load(i, n);  // (nothing when i >= n)
    if (hlt(X, hread(ae, 0))) {
      uint32_t m;
      const uint32_t f = up_anc(i, X, d, anc, ae, &m);
      *settled = !hlt(hread(sb, d + m - 1), X);
      return f;
    }
    if (i >= n) {
      put(i, X);
      return i;
    }
    return k2_sift_down_from(sub, i, n, X);
  }

  // sift (:550-564): up if less than the parent, else down.  The ancestors
  // and the first subtree below i are loaded together.
  __device__ __forceinline__ uint32_t sift(uint32_t i, uint32_t n, const HEnt& X) const {
    if (k == 2) return k2_sift(i, n, X);
    if (i == 0) return sift_down(i, n, X);
    uint32_t anc;
    const uint32_t d = ancestors(i, &anc);
    const Sub L = layout(d);
    HEnt ae{~0ull, kClsNone + 1, 0};
    uint32_t eidx = 0xffffffffu;
    HEnt e = ae;
    if (lane < d) ae = ld(anc);
    else if (i < n) e = sub_load(L, i, n, &eidx);
    if (hlt(X, hread(ae, 0))) return up_anc(i, X, d, anc, ae);
    if (L.D == 0) return sift_down(i, n, X);  // (no lanes left for a subtree)
    if (i < n && down_sub(L, d, e, eidx, n, X, &i)) return sift_down(i, n, X);
    put(i, X);
    return i;
  }
};

// Waves of the pull and event kernels: 3 = one wave per heap (the three
// heaps' sifts of a pop, a limit-loop step or an add event run side by side;
// the pull kernel's waves meet at a block barrier after each), 1 = one wave
// makes all three in turn.
#ifndef DMC_HEAP_WAVES
#define DMC_HEAP_WAVES 3
#endif
constexpr uint32_t kHeapWaves = DMC_HEAP_WAVES;
static_assert(kHeapWaves == 1 || kHeapWaves == 3, "DMC_HEAP_WAVES: 1 or 3");

struct WHeaps {
  const Table& tb;
  const HeapDev& hd;
  WHeap h[3];
  uint32_t lane;
  uint32_t wid;  // split: this wave's heap
  bool split;    // one wave per heap (else this wave owns all three)
  bool lead;     // makes the uniform stores (the limit heap's wave, or the only wave)
  // (cache: the LDS copy of each heap's first T entries, kHeapLds apart)
  __device__ WHeaps(const Table& t, const HeapDev& d, HEnt* cache, uint32_t T, bool split_ = false)
      : tb(t), hd(d) {
    lane = lane_id();
    split = split_;
    wid = split ? threadIdx.x >> 6 : 0u;
    lead = !split || wid == (uint32_t)kHLim;  // (the limit heap's sifts are the shortest)
    _Pragma("unroll") for (int j = 0; j < 3; ++j)
      h[j] = WHeap{d.ent + (size_t)j * d.n, d.hix + (size_t)j * d.n, d.k, lane,
                   cache + j * kHeapLds, T};
  }
  __device__ __forceinline__ bool owns(int j) const { return !split || (uint32_t)j == wid; }
  // the heaps' state (LDS tops, global records) the same for every wave after it
  __device__ __forceinline__ void sync() const {
    if (split) __syncthreads();
    else wave_sync();
  }
  __device__ __forceinline__ uint32_t count() const { return hd.cnt[0]; }
  __device__ __forceinline__ HEnt top(int j) const { return h[j].ld(0); }
  // slot s's index in each heap (lanes 0-2 load; uniform)
  __device__ __forceinline__ void index3(uint32_t s, uint32_t* ix) const {
    uint32_t v = 0;
    if (lane < 3) v = hd.hix[(size_t)lane * hd.n + s];
    _Pragma("unroll") for (int j = 0; j < 3; ++j) ix[j] = uread(v, j);
  }
  // the slot's three entries from its ScanRec (loaded by every lane: one
  // request) and its three indices
  __device__ __forceinline__ void load3(uint32_t s, HEnt* X, uint32_t* ix) const {
    const ScanRec r = tb.sc[s];
    index3(s, ix);
    _Pragma("unroll") for (int j = 0; j < 3; ++j) X[j] = hent(j, r, s);
  }
  // adjust x 3 (:996-1016, :567-625): sift in each heap (this wave's), in
  // heap order
  __device__ __forceinline__ void adjust3(uint32_t s, const HEnt* X, uint32_t* ix) const {
    const uint32_t n = count();
    _Pragma("unroll") for (int j = 0; j < 3; ++j) if (owns(j)) ix[j] = h[j].sift(ix[j], n, X[j]);
  }
  // adjust x 3 twice with the same entries (a first request's :996-1006 and
  // :1011-1016): per heap, the second sift is made only when the first
  // cannot prove it moves nothing (k2_sift_s; the heaps are independent, so
  // each heap's two calls may run back to back)
  template <int J>
  __device__ __forceinline__ void twice_one(uint32_t n, const HEnt* X, uint32_t* ix) const {
    if (owns(J)) {
      bool st = false;
      if (h[J].k == 2) ix[J] = h[J].k2_sift_s(ix[J], n, X[J], &st);
      else ix[J] = h[J].sift(ix[J], n, X[J]);
      if (!st) ix[J] = h[J].sift(ix[J], n, X[J]);
    }
  }
  __device__ __forceinline__ void adjust3_twice(uint32_t s, const HEnt* X, uint32_t* ix) const {
    const uint32_t n = count();
    twice_one<0>(n, X, ix);
    twice_one<1>(n, X, ix);
    twice_one<2>(n, X, ix);
  }
  __device__ __forceinline__ void adjust3(uint32_t s) const {
    HEnt X[3];
    uint32_t ix[3];
    load3(s, X, ix);
    adjust3(s, X, ix);
  }
  // the entries rewritten in place (a key that changed without a heap call:
  // the idle reset before a Reject, :937-993)
  __device__ __forceinline__ void refresh3(uint32_t s) const {
    HEnt X[3];
    uint32_t ix[3];
    load3(s, X, ix);
    _Pragma("unroll") for (int j = 0; j < 3; ++j) if (owns(j)) h[j].put(ix[j], X[j]);
  }
  // erase (delete_from_heaps): IndIntruHeap::remove (:433-445) -- the last
  // element swapped in and sifted with the count already reduced
  __device__ __forceinline__ void remove3(uint32_t s) const {
    uint32_t ix[3];
    index3(s, ix);
    const uint32_t last = count() - 1;
    _Pragma("unroll") for (int j = 0; j < 3; ++j) {
      const HEnt X = h[j].ld(last);
      h[j].sift(ix[j], last, X);
    }
    wave_sync();
    if (lane < 3) hd.cnt[lane] = last;
    wave_sync();
  }
};

// The heaps' first entries into LDS at a kernel's start (every thread of the
// block), and back at its end: T = min(count, kHeapLds).
__device__ inline uint32_t heap_cache_fill(const HeapDev& hd, HEnt* c) {
  const uint32_t T = min(hd.cnt[0], kHeapLds);
  _Pragma("unroll") for (int j = 0; j < 3; ++j)
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x)
      c[j * kHeapLds + i] = hd.ent[(size_t)j * hd.n + i];
  __syncthreads();
  return T;
}
__device__ inline void heap_cache_flush(const HeapDev& hd, const HEnt* c, uint32_t T) {
  __syncthreads();
  _Pragma("unroll") for (int j = 0; j < 3; ++j)
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x)
      hd.ent[(size_t)j * hd.n + i] = c[j * kHeapLds + i];
}

// ------------------------------------------------------------------ kernels
// registration (client_map.emplace + three pushes, in the given order): new
// clients have no request, so each push's sift_up never moves (nothing is
// strictly greater than a client without a request): the pushes append in
// order, one thread per client.  `base` = the heaps' count before.
__global__ void k_heap_push(Table tb, HeapDev hd, const uint32_t* slots, uint32_t n) {
  const uint32_t base = hd.cnt[0];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slots[i];
  const ScanRec r = tb.sc[s];
  _Pragma("unroll") for (int j = 0; j < 3; ++j) {
    hd.ent[(size_t)j * hd.n + base + i] = hent(j, r, s);
    hd.hix[(size_t)j * hd.n + s] = base + i;
  }
}
__global__ void k_heap_count_add(HeapDev hd, uint32_t n) {
  if (threadIdx.x < 3) hd.cnt[threadIdx.x] += n;
}

// erase (delete_from_heaps, before the client's state goes)
__global__ void __launch_bounds__(64) k_heap_remove(Table tb, HeapDev hd, const uint32_t* slots,
                                                    uint32_t n) {
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  WHeaps W(tb, hd, cache, T);
  for (uint32_t i = 0; i < n; ++i) W.remove3(slots[i]);
  heap_cache_flush(hd, cache, T);
}

// clients whose queues a filter / remove_by_client modified, ascending
__global__ void __launch_bounds__(64) k_heap_adjust(Table tb, HeapDev hd, const uint32_t* slots,
                                                    uint32_t n) {
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  WHeaps W(tb, hd, cache, T);
  for (uint32_t i = 0; i < n; ++i) W.adjust3(slots[i]);
  heap_cache_flush(hd, cache, T);
}

// The heap calls of an add batch, in batch order.  The batched add path
// (k_add_link, k_add_chain and, with idle clients, the activation kernels)
// has made every request's state change with the reference's values -- tags,
// Reject checks, idle resets -- and left in hev[i] the heap calls the
// reference makes for request i: 3 a client's first request (adjust x 3 at
// :996-1006 and again at :1011-1016), 2 any other accepted one (:1011-1016),
// 1 a refused activation of a client with requests (its idle reset moved
// the ready key, and no heap call follows, :989-993: the entries are
// rewritten in place), 0 none.  Every call sees the slot's state after the
// batch, which is its state at each of its events: a client's front changes
// only at its first accepted request of the batch, its prop_delta only at
// its activation, before any of its adjusts.  64 events are read at once.
//
// With one wave per heap (kHeapWaves = 3) each wave replays the whole event
// list on its own heap: the heaps share no state, and a heap's calls are the
// same calls in the same order whichever wave makes the other heaps'.
__global__ void __launch_bounds__(64 * kHeapWaves) k_heap_events(Table tb, HeapDev hd,
                                                                 const dmc_request* reqs,
                                                                 const uint8_t* ev, uint32_t n) {
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  WHeaps W(tb, hd, cache, T, kHeapWaves == 3);
  const uint32_t lane = W.lane;
  const uint32_t cnt = W.count();
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    // a window of 64 events, one per lane: the requests and the slots'
    // states are the kernel's inputs (the batched add path made every state
    // change; only the heaps change here), loaded once per window
    const uint32_t i = i0 + lane;
    uint32_t e = 0, sl = 0;
    if (i < n) {
      e = ev[i];
      if (e) sl = reqs[i].slot;
    }
    ScanRec r{0.0, 0.0, 0.0, 0, 0, 0, 0, 0};
    if (e) r = tb.sc[sl];
    // the window's events from `start` on: after each ordered event the
    // heaps' indices and entries are read again (it moved them), the rest
    // of the window is not
    for (uint32_t start = 0; start < 64;) {
      const bool live = e && lane >= start;
      uint32_t hx[3] = {0, 0, 0};
      if (live) {
        _Pragma("unroll") for (int j = 0; j < 3; ++j) if (W.owns(j)) hx[j] = hd.hix[(size_t)j * hd.n + sl];
      }
      // Which of them must run in order.  A repeat request of a client (code
      // 2) whose entries (in this wave's heaps) already hold its key, none
      // less than its parent and none with a child less than it, makes sifts
      // that move nothing (K = 2 checked here; other K run every event): the
      // events before the first that may move are skipped -- each of them
      // saw the heaps as the window found them, unchanged by the ones before.
      bool ord = live && (e == 1 || e == 3 || (e == 2 && hd.k != 2));
      if (live && e == 2 && hd.k == 2) {
        _Pragma("unroll") for (int j = 0; j < 3; ++j) {
          if (!W.owns(j)) continue;
          const HEnt X = hent(j, r, sl);
          const uint32_t v = hx[j];
          const HEnt own = W.h[j].ld(v);
          if (own.key != X.key || own.cls != X.cls) ord = true;
          if (v > 0 && hlt(X, W.h[j].ld((v - 1) >> 1))) ord = true;
          const uint64_t li = 2ull * v + 1;
          if (li < cnt) {
            const HEnt c1 = W.h[j].ld((uint32_t)li);
            HEnt mc = c1;
            if (li + 1 < cnt) {
              const HEnt c2 = W.h[j].ld((uint32_t)li + 1);
              if (hlt(c2, c1)) mc = c2;
            }
            if (hlt(mc, X)) ord = true;
          }
        }
      }
      const uint64_t m = __ballot(ord);
      if (!m) break;
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      const uint32_t ej = uread(e, j), s = uread(sl, j);
      HEnt X[3];
      uint32_t ix[3];
      {
        ScanRec rj{0.0, 0.0, 0.0, 0, 0, 0, 0, 0};
        rj.r = dread(r.r, j);
        rj.pk = dread(r.pk, j);
        rj.l = dread(r.l, j);
        rj.count = (uint8_t)uread(r.count, j);
        rj.flags = (uint8_t)uread(r.flags, j);
        _Pragma("unroll") for (int h = 0; h < 3; ++h) {
          X[h] = hent(h, rj, s);
          ix[h] = uread(hx[h], j);
        }
      }
      if (ej == 1) {  // (refresh3 with the window's loads)
        _Pragma("unroll") for (int h = 0; h < 3; ++h) if (W.owns(h)) W.h[h].put(ix[h], X[h]);
      } else if (ej == 3) {
        W.adjust3_twice(s, X, ix);
      } else {
        W.adjust3(s, X, ix);
      }
      wave_sync();
      start = j + 1;
    }
  }
  heap_cache_flush(hd, cache, T);
}

constexpr int kHeapThreads = 256;

// The idle reset's minimum (:957-978) over every registered non-idle client
// but `self`: the block reduces (front p or prev p) + prop_delta as ordered
// keys; every thread returns it.
__device__ inline double heap_idle_lowest(const Table& tb, uint64_t* sh) {
  uint64_t m = kMaxKey;
  for (uint32_t s = threadIdx.x; s < tb.n; s += blockDim.x) {
    const ScanRec r = tb.sc[s];
    if (!(r.flags & F_REG) || (r.flags & F_IDLE)) continue;
    const double v = r.count ? r.pk : __dadd_rn(tb.rec[s].prev_p, tb.rec[s].pd);
    const uint64_t o = okey(v);
    m = o < m ? o : m;
  }
  for (int d = 32; d > 0; d >>= 1) {
    const uint64_t o = shfl_down_u64(m, d);
    m = o < m ? o : m;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  uint64_t r = kMaxKey;
  for (uint32_t w = 0; w < blockDim.x / 64; ++w) r = sh[w] < r ? sh[w] : r;
  __syncthreads();
  return r == kMaxKey ? 1.7976931348623157e308 : from_okey(r);
}

// n add_request_time calls in order (do_add_request, :913-1018).  Wave 0
// runs them; waves 1-3 wait at the block barrier and join only for an idle
// reset's minimum (a scan of every client, as the reference's).
__global__ void __launch_bounds__(kHeapThreads) k_heap_add(Table tb, HeapDev hd, AddParams p) {
  __shared__ uint64_t sh[kHeapThreads / 64];
  __shared__ uint32_t s_cmd;  // 1: an idle reset's minimum, 2: done
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  if (threadIdx.x >= 64) {
    for (;;) {
      __syncthreads();
      if (s_cmd == 2) break;
      heap_idle_lowest(tb, sh);
    }
    heap_cache_flush(hd, cache, T);
    return;
  }
  WHeaps W(tb, hd, cache, T);
  const uint32_t lane = W.lane;
  for (uint32_t i = 0; i < p.n; ++i) {
    const uint32_t s = p.reqs[i].slot;
    const bool ok = s < tb.n;
    const uint8_t fl = ok ? tb.sc[s].flags : 0;
    const bool idle = ok && (fl & (F_REG | F_IDLE)) == (F_REG | F_IDLE);
    double lowest = 0.0;
    if (idle) {  // (the client itself is idle: not counted)
      if (lane == 0) s_cmd = 1;
      __syncthreads();
      lowest = heap_idle_lowest(tb, sh);
    }
    uint32_t acc = 0, first = 0;
    if (lane == 0) {
      if (!ok || !(fl & F_REG)) {
        p.rc[i] = DMC_ENOTREG;
      } else {
        if (idle) {  // :981-984 (prop_delta kept when the trigger does not fire)
          const double trigger = 1.7976931348623157e308 / 3.0;
          const double pd = lowest < trigger ? __dsub_rn(lowest, p.reqs[i].time) : tb.rec[s].pd;
          tb.rec[s].pd = pd;
          const ScanRec r = tb.sc[s];
          if (r.count) tb.sc[s].pk = __dadd_rn(tb.ring[(size_t)s * tb.q + (r.head & tb.qmask)].p, pd);
          tb.sc[s].flags = (uint8_t)(r.flags & ~F_IDLE);
        }
        const uint32_t count0 = tb.sc[s].count;
        AddState st;
        add_chain_slot(tb, p, s, 1, i, nullptr, nullptr, ActBuf{}, &st);
        acc = p.rc[i] == DMC_OK ? 1u : 0u;
        first = count0 == 0 ? 1u : 0u;
      }
    }
    wave_sync();  // (lane 0's stores above precede the wave's loads below)
    acc = uread(acc, 0);
    first = uread(first, 0);
    if (acc) {
      HEnt X[3];
      uint32_t ix[3];
      W.load3(s, X, ix);
      if (first) W.adjust3_twice(s, X, ix);  // a first request (:996-1006, :1011-1016)
      else W.adjust3(s, X, ix);              // (:1011-1016)
    } else if (idle) {
      W.refresh3(s);  // (a rejected activation: prop_delta moved, no heap call)
    }
  }
  if (lane == 0) s_cmd = 2;
  __syncthreads();
  heap_cache_flush(hd, cache, T);
}

// (debug, DMC_HEAP_CLOCKS: where a pull's time goes -- shader-clock cycles
// per phase accumulated by the pulling wave, printed once per k_heap_pull)
struct HClk {
  uint64_t t[10] = {};  // decide, limit sifts, pop loads, pop stores, resv, lim, ready, promote, limit iters, pulls
  uint64_t last = 0;
  __device__ void start() { if (DMC_HEAP_CLOCKS) last = __builtin_amdgcn_s_memtime(); }
  __device__ void lap(int i) {
    if (DMC_HEAP_CLOCKS) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      t[i] += now - last;
      last = now;
    }
  }
};

// The pop of slot s, the top of heap `hsel` (pop_process_request,
// :1046-1073, with reduce_reservation_tags, :1077-1111, for a priority pop):
// the decision, the front popped and (delayed) the new front's tag
// (update_next_tag, :1021-1036), the heap calls with that state, then the
// reduction and resv.promote.  Every lane loads the client's record, cursor
// and the popped and next entries (one request each: the values are
// uniform) and lane i the queue's entry i (an immediate priority pop reduces
// every queued request: one lane each), in two levels of loads; lane 0
// stores what is uniform.  With one wave per heap every wave computes the
// same state, the lead wave stores it, and each wave sifts its own heap.
// The pop's loads, decision and new client state (heap_pop without the
// heap calls): *po0 the front's keys before the reduction (what the demotes
// see), *po after it.  split: a block barrier between every wave's loads and
// the lead wave's stores (each wave computes the same state).
__device__ __forceinline__ void heap_pop_state(const Table& tb, uint32_t s, bool prio, uint64_t tick,
                                               dmc_decision* out, unsigned long long* sched,
                                               uint32_t lane, bool lead, bool split, HClk* ck,
                                               ScanRec* po0, ScanRec* po) {
  // level 1: cursor, record, aux, bound info
  // (the whole ring loaded here instead, lane i its entry i, measured
  // slower: pop loads 2,200 against 1,850 cycles per pull, r06i)
  const ScanRec sr = tb.sc[s];
  ClientRec cr = tb.rec[s];
  ClientAux ax{0, 0, 0};
  BoundInfo bi{0.0, 0.0, 0.0, 0.0};
  if (tb.delayed) {
    ax = tb.aux[s];
    if (tb.binfo) bi = tb.binfo[s];
  }
  // level 2: the queue's entries
  ReqEntry* ring = tb.ring + (size_t)s * tb.q;
  const uint32_t h = sr.head, c = sr.count;
  const uint32_t nh = (h + 1) & tb.qmask, nc = c - 1;
  const ReqEntry popped = ring[h];
  // the new front (delayed: its tag is computed below)
  double fr = 0.0, fp = 0.0, fl = 0.0, farr = 0.0;
  uint32_t fcost = 0;
  if (nc) {
    const ReqEntry& fe = ring[nh];
    fr = fe.r;
    fp = fe.p;
    fl = fe.l;
    farr = fe.arrival;
    fcost = fe.cost;
  }
  double er = 0.0;  // lane i: queue position i's r (immediate priority pop, i >= 2)
  const bool deep = lead && prio && !tb.delayed && lane >= 2 && lane < c;
  if (deep) er = ring[(h + lane) & tb.qmask].r;
  if (DMC_HEAP_CLOCKS && ck) {
    keep(popped.r);
    keep(fr);
    keep(er);
    ck->lap(2);
  }
  if (split) {  // every wave's loads done before the lead wave stores
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    // (with the loads, every earlier memory operation of this wave is
    // complete before the stores below: the decoupled pull's ready-mark
    // atomics on a client's cursor)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (lead && lane == 0) {
    dmc_decision d;
    d.handle = popped.handle;
    d.tag_r = popped.r;
    d.tag_p = popped.p;
    d.tag_l = popped.l;
    d.slot = s;
    d.cost = popped.cost;
    d.phase = prio ? DMC_PHASE_PRIORITY : DMC_PHASE_RESERVATION;
    d.flags = 0;  // (the heap top is the reference's winner: no tie to flag)
    *out = d;
    atomicAdd(&sched[prio ? 1 : 0], 1ull);
  }
  double rinv = cr.r_inv;
  bool f_tagged = false;
  if (tb.delayed && nc) {  // update_next_tag (every lane computes the same)
    const Tag3 pt{popped.r, popped.p, popped.l, popped.arrival};
    Tag3 nt;
    double winv = cr.w_inv, linv = cr.l_inv;
    if (tb.binfo) {  // U1: get_cli_info (:870-875) becomes client.info
      rinv = bi.r_inv;
      winv = bi.w_inv;
      linv = bi.l_inv;
      cr.r_inv = rinv;
      cr.w_inv = winv;
      cr.l_inv = linv;
    }
    if (make_tag(pt, rinv, winv, linv, ax.cur_delta, ax.cur_rho, farr, fcost, tb.antic, &nt)) {
      fr = nt.r;
      fp = nt.p;
      fl = nt.l;
      f_tagged = true;
      assign_unpinned(cr.prev_r, nt.r);
      assign_unpinned(cr.prev_l, nt.l);
      assign_unpinned(cr.prev_p, nt.p);
      cr.prev_arr = nt.arrival;
      if (lead && lane == 0) tb.aux[s].last_tick = tick;
    }
  }
  // the front's keys before the reduction (what the demotes see)
  ScanRec o{0.0, 0.0, 0.0, (uint8_t)nh, (uint8_t)nc, (uint8_t)(sr.flags & ~F_READY), sr.stamp, 0};
  if (nc) {
    o.r = fr;
    o.pk = __dadd_rn(fp, cr.pd);
    o.l = fl;
  }
  const double r_pre = o.r;
  if (prio) {
    // reduce_reservation_tags (immediate: every queued request; delayed: the
    // front) and prev r (:1077-1111)
    const double off = resv_offset(rinv, popped.cost, popped.rho);
    if (nc) fr = __dsub_rn(fr, off);
    if (deep) ring[(h + lane) & tb.qmask].r = __dsub_rn(er, off);
    cr.prev_r = __dsub_rn(cr.prev_r, off);
    if (nc) o.r = fr;
  }
  if (lead && lane == 0) {
    if (nc && (f_tagged || prio)) {
      ReqEntry& fe = ring[nh];
      fe.r = fr;
      if (f_tagged) {
        fe.p = fp;
        fe.l = fl;
        fe.delta = ax.cur_delta;
        fe.rho = ax.cur_rho;
      }
    }
    if (tb.delayed || prio) tb.rec[s] = cr;
    tb.sc[s] = o;
  }
  *po = o;
  *po0 = o;
  po0->r = r_pre;
}

__device__ __forceinline__ void heap_pop(const Table& tb, const WHeaps& W, uint32_t s, bool prio,
                                uint64_t tick, dmc_decision* out, unsigned long long* sched,
                                HClk* ck = nullptr) {
  const uint32_t lane = W.lane;
  // the slot's heap indices (lanes 0-2), with the state's first level
  const uint32_t hv = lane < 3 ? W.hd.hix[(size_t)lane * W.hd.n + s] : 0u;
  ScanRec o0, o;
  heap_pop_state(tb, s, prio, tick, out, sched, lane, W.lead, W.split, ck, &o0, &o);
  uint32_t ix[3];
  _Pragma("unroll") for (int j = 0; j < 3; ++j) ix[j] = uread(hv, j);
  const uint32_t n = W.count();
  if (DMC_HEAP_CLOCKS && ck) {
    keep(o.r);
    ck->lap(3);
  }
  // pop_process_request's heap calls, on the unreduced front (:1063-1069)
  // (a priority pop's resv demote and promote as one operation, K = 2)
  const bool dp = DMC_HEAP_DP && prio && W.hd.k == 2;
  if (W.owns(kHResv)) {
    if (dp) ix[kHResv] = W.h[kHResv].k2_demote_promote(ix[kHResv], n, hent(kHResv, o0, s), hent(kHResv, o, s));
    else ix[kHResv] = W.h[kHResv].sift_down(ix[kHResv], n, hent(kHResv, o0, s));
  }
  if (DMC_HEAP_CLOCKS && ck) ck->lap(4);
  if (W.owns(kHLim)) ix[kHLim] = W.h[kHLim].sift(ix[kHLim], n, hent(kHLim, o0, s));
  if (DMC_HEAP_CLOCKS && ck) ck->lap(5);
  if (W.owns(kHReady)) ix[kHReady] = W.h[kHReady].sift_down(ix[kHReady], n, hent(kHReady, o0, s));
  if (DMC_HEAP_CLOCKS && ck) ck->lap(6);
  if (prio && !dp && W.owns(kHResv))  // resv_heap.promote after the reduction (:1110)
    W.h[kHResv].sift_up(ix[kHResv], hent(kHResv, o, s));
  W.sync();
  if (DMC_HEAP_CLOCKS && ck) ck->lap(7);
}

struct HeapPullRes {
  uint32_t n, n_res, n_prio;
  int32_t type;
  double when;
  uint32_t pend_slot, pend_prio;  // mode 1: the decided pop, left to mode 2
};

// k pull_request(now) calls in order (do_next_request, :1115-1186).
// mode 0: all k; mode 1 (U1 with a host client_info_f, delayed: the host
// fetches the popped client's info between selection and pop, :870-875,
// :1021-1036): one pull decided -- the limit loop's marks made -- and its
// pop left in res->pend_*; mode 2: that pop.
//
// With one wave per heap (kHeapWaves = 3) every wave decides each pull from
// the LDS tops (the same decision), a pop's or limit step's three heap calls
// run one per wave, and the block barrier after them makes the next decision
// see all three heaps.
__global__ void __launch_bounds__(64 * kHeapWaves) k_heap_pull(Table tb, HeapDev hd, double now,
                                                               uint32_t k, int at_limit, uint64_t tick,
                                                               dmc_decision* out, HeapPullRes* res,
                                                               dmc_pull_result* d_result,
                                                               unsigned long long* sched, int mode = 0) {
  __shared__ HEnt cache[3 * kHeapLds];
  const uint32_t T = heap_cache_fill(hd, cache);
  WHeaps W(tb, hd, cache, T, kHeapWaves == 3);
  const uint32_t lane = W.lane;
  HeapPullRes r{0, 0, 0, DMC_NEXT_RETURNING, 0.0, 0, 0};
  if (mode == 2) {
    const HeapPullRes pr = *res;
    heap_pop(tb, W, pr.pend_slot, pr.pend_prio != 0, tick, out, sched);
    r.n = 1;
    if (pr.pend_prio) r.n_prio = 1;
    else r.n_res = 1;
    heap_cache_flush(hd, cache, T);
    if (lane == 0 && W.lead) *res = r;
    return;
  }
  const uint32_t n = W.count();
  HClk ck;
  ck.start();
  // each iteration decides one pull (pop_slot / pop_prio) or stops; the pop
  // is made at its end (mode 1: recorded for mode 2 instead)
  while (r.n < k) {
    uint32_t pop_slot = kNone;
    bool pop_prio = false;
    if (n == 0) {  // no clients: none (:1118-1120)
      r.type = DMC_NEXT_NONE;
      break;
    }
    const HEnt rt = W.top(kHResv);
    if (rt.cls == 0 && hval(rt) <= now) {
      pop_slot = rt.slot;
    } else {
      for (;;) {  // the limit loop
        const HEnt lt = W.top(kHLim);
        if (!(lt.cls == 0 && hval(lt) <= now)) break;
        const uint32_t ls = lt.slot;
        // ready = true (the slot's ready flag: F_READY in its cursor word).
        // The limit entry is the top itself with the ready class (its key
        // is the record's l already): that sift needs no load.
        ck.lap(0);
        if (W.owns(kHReady)) {
          ScanRec lr = tb.sc[ls];
          const uint32_t ixr = hd.hix[(size_t)kHReady * hd.n + ls];
          lr.flags = (uint8_t)(lr.flags | F_READY);
          if (lane == 0) tb.sc[ls].flags = lr.flags;
          W.h[kHReady].sift_up(ixr, hent(kHReady, lr, ls));
        }
        if (W.owns(kHLim)) {
          HEnt X = lt;
          X.cls = 1;  // (hent(kHLim, ...) of the record marked ready)
          W.h[kHLim].sift_down(0, n, X);
        }
        W.sync();
        ck.lap(1);
        if (DMC_HEAP_CLOCKS) ++ck.t[8];
      }
      const HEnt pt = W.top(kHReady);
      const bool ph = pt.cls != kClsNone && hval(pt) < kInf;
      if (pt.cls == 0 && ph) {
        pop_slot = pt.slot;
        pop_prio = true;
      } else if (at_limit == DMC_AT_LIMIT_ALLOW && ph) {
        pop_slot = pt.slot;
        pop_prio = true;
      } else if (at_limit == DMC_AT_LIMIT_ALLOW && rt.cls == 0 && hval(rt) < kInf) {
        pop_slot = rt.slot;
      }
    }
    if (pop_slot == kNone) {
      // future / none (:1170-1185; min_not_0_time excludes exact 0,
      // :1192-1195; kTimeMax = DBL_MAX: an infinite tag is no future)
      constexpr double kTimeMax = 1.7976931348623157e308;
      double next = kTimeMax;
      const HEnt r0 = W.top(kHResv), l0 = W.top(kHLim);
      if (r0.cls != kClsNone) {
        const double v = hval(r0);
        if (v != 0.0) next = v < next ? v : next;
      }
      if (l0.cls != kClsNone) {
        const double v = hval(l0);
        if (v != 0.0) next = v < next ? v : next;
      }
      if (next < kTimeMax) {
        r.type = DMC_NEXT_FUTURE;
        r.when = next;
      } else {
        r.type = DMC_NEXT_NONE;
      }
      break;
    }
    if (mode == 1) {
      r.pend_slot = pop_slot;
      r.pend_prio = pop_prio ? 1u : 0u;
      break;
    }
    ck.lap(0);
    heap_pop(tb, W, pop_slot, pop_prio, tick, out + r.n, sched, &ck);
    ++r.n;
    if (pop_prio) ++r.n_prio;
    else ++r.n_res;
  }
  if (DMC_HEAP_CLOCKS && lane == 0 && r.n > 1000)  // (each wave: its own heap's sifts)
    printf("heap clocks: pulls %u prio %u limit iters %llu | cycles per pull: decide %.0f limit-sifts %.0f "
           "pop-loads %.0f pop-stores %.0f resv %.0f lim %.0f ready %.0f promote %.0f\n",
           r.n, r.n_prio, (unsigned long long)ck.t[8], (double)ck.t[0] / r.n, (double)ck.t[1] / r.n,
           (double)ck.t[2] / r.n, (double)ck.t[3] / r.n, (double)ck.t[4] / r.n, (double)ck.t[5] / r.n,
           (double)ck.t[6] / r.n, (double)ck.t[7] / r.n);
  heap_cache_flush(hd, cache, T);
  if (lane || !W.lead) return;
  *res = r;
  if (d_result) {
    dmc_pull_result x{};
    x.n_decisions = r.n;
    x.next_type = r.type;
    x.when = r.type == DMC_NEXT_FUTURE ? r.when : 0.0;
    x.n_priority = r.n_prio;
    x.n_reservation = r.n_res;
    *d_result = x;
  }
}

// ---------------------------------------------------------------------------
// k pull_request(now) calls in order, the heap waves decoupled from the
// decisions (K = 2, mode 0).  In k_heap_pull every pull ends at a block
// barrier, so each pull costs its decision, its pop's loads and the slowest
// of its three heap calls -- a sift from the root through ~20 levels, of
// which only the first round decides the new top.  Here wave 3 (the
// coordinator) makes the decisions, the limit loop's marks and the pops'
// loads and stores, and publishes each heap operation to an LDS ring; waves
// 0-2 each run every operation on their own heap in order, signalling (an
// LDS counter per heap) as soon as their heap's top holds its value after
// it, and finish the sift's deeper rounds while the coordinator already
// decides the next pull from the three tops.  The operations, their order
// per heap and every move are the same as k_heap_pull's: only the waiting
// changes.  The coordinator alone reads and writes the clients' state
// (ScanRec, record, ring, decisions) -- except the limit loop's ready mark,
// which the ready heap's wave stores before it signals -- and each heap
// wave alone its heap's entries and indices (a pop's index of the popped
// client in the heap it was the top of is 0; the others are looked up by
// the heap's wave when it runs the operation).
#ifndef DMC_HEAP_ASYNC
#define DMC_HEAP_ASYNC 1
#endif
struct HOp {
  uint32_t type;  // kOpLimit, kOpPop, kOpEnd
  uint32_t s;     // the slot
  uint32_t prio;  // pop: a priority pop
  uint32_t pad;
  HEnt X[3];  // pop: the three heaps' entries on the unreduced front; limit: X[1] the limit entry marked ready
  HEnt Xu;    // priority pop: the resv entry after the reduction (resv.promote)
};
enum : uint32_t { kOpLimit = 1, kOpPop = 2, kOpEnd = 3 };
constexpr uint32_t kHOps = 16;  // ring slots (the coordinator waits for a free one)

__device__ __forceinline__ uint32_t lds_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t v) {
  while (lds_u32(p) < v) __builtin_amdgcn_s_sleep(1);
}

__global__ void __launch_bounds__(256) k_heap_pull_async(Table tb, HeapDev hd, double now, uint32_t k,
                                                         int at_limit, uint64_t tick, dmc_decision* out,
                                                         HeapPullRes* res, dmc_pull_result* d_result,
                                                         unsigned long long* sched) {
  __shared__ HEnt cache[3 * kHeapLds];
  __shared__ HOp ring[kHOps];
  __shared__ uint32_t s_pub;      // operations published
  __shared__ uint32_t s_done[3];  // per heap: operations whose effect on the top is in place
  if (threadIdx.x == 0) {
    s_pub = 0;
    s_done[0] = s_done[1] = s_done[2] = 0;
  }
  const uint32_t T = heap_cache_fill(hd, cache);  // (its barrier publishes the counters)
  const uint32_t wid = threadIdx.x >> 6, lane = lane_id();
  const uint32_t n = hd.cnt[0];
  if (wid < 3) {
    // a heap's wave: every operation in order
    const WHeap H{hd.ent + (size_t)wid * hd.n, hd.hix + (size_t)wid * hd.n, 2u, lane,
                  cache + wid * kHeapLds, T};
    HClk ck;
    ck.start();
    for (uint32_t op = 0;; ++op) {
      lds_wait_ge(&s_pub, op + 1);
      ck.lap(0);
      const HOp o = ring[op % kHOps];
      if (o.type == kOpEnd) break;
      auto sig = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the top's LDS store)
        if (lane == 0) __atomic_store_n(&s_done[wid], op + 1, __ATOMIC_RELAXED);
      };
      // An operation that cannot change the heap's top signals before it
      // starts: a sift down from a node other than the top, or a climb by
      // an entry not less than the top (it passes only ancestors it is
      // strictly less than).  (Loading the popped client's index and first
      // round trip at a hint published when the pop is decided, before the
      // coordinator computes its state, measured slower: 5.55 against 5.04
      // us per pull, r06n.)
      const HEnt root = ld_lds<HEnt>(H.c);
      if (o.type == kOpLimit) {
        // ready = true; ready.promote; limit.demote (:1135-1144)
        if (wid == kHResv) {
          sig();
        } else if (wid == kHLim) {
          H.k2_sift_down_sig(0, n, o.X[1], sig);
        } else {
          // (the coordinator sets the ready mark in the client's cursor)
          ScanRec lr = tb.sc[o.s];
          const uint32_t ixr = (uint32_t)__builtin_amdgcn_readfirstlane((int)H.x[o.s]);
          lr.flags = (uint8_t)(lr.flags | F_READY);
          const HEnt X = hent(kHReady, lr, o.s);
          const bool early = !hlt(X, root);
          if (early) sig();
          uint32_t anc;
          const uint32_t d = H.k2_ancestors(ixr, &anc);
          HEnt ae{~0ull, kClsNone + 1, 0};
          if (lane < d) ae = H.ld(anc);
          H.up_anc(ixr, X, d, anc, ae);
          if (!early) sig();
        }
      } else {
        // pop_process_request's calls (:1063-1069) and resv.promote (:1110);
        // the popped client's index is 0 where it is the top
        const bool istop = root.slot == o.s;
        auto index = [&]() {
          return istop ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane((int)H.x[o.s]);
        };
        if (wid == kHResv) {
          if (o.prio) {
            const bool early = !istop && !hlt(o.Xu, root);
            if (early) sig();
            H.k2_demote_promote(index(), n, o.X[0], o.Xu);
            if (!early) sig();
          } else {
            H.k2_sift_down_sig(0, n, o.X[0], sig);  // (the resv top)
          }
        } else if (wid == kHLim) {
          if (!istop && !hlt(o.X[1], root)) {
            sig();
            H.k2_sift(index(), n, o.X[1]);
          } else {
            H.k2_sift_sig(index(), n, o.X[1], sig);
          }
        } else {
          if (istop) {
            H.k2_sift_down_sig(0, n, o.X[2], sig);
          } else {  // (a sift down from below the top)
            sig();
            H.k2_sift_down(index(), n, o.X[2]);
          }
        }
      }
      ck.lap(o.type == kOpLimit ? 1 : 2);
      if (DMC_HEAP_CLOCKS) ++ck.t[o.type == kOpLimit ? 8 : 9];
    }
    if (DMC_HEAP_CLOCKS && lane == 0 && ck.t[9] > 1000)
      printf("async heap wave %u: ops limit %llu pop %llu | cycles per pop: waiting %.0f limit ops %.0f pops %.0f\n",
             wid, (unsigned long long)ck.t[8], (unsigned long long)ck.t[9], (double)ck.t[0] / ck.t[9],
             (double)ck.t[1] / ck.t[9], (double)ck.t[2] / ck.t[9]);
  } else {
    // the coordinator: k_heap_pull's decisions, one pull after another
    HeapPullRes r{0, 0, 0, DMC_NEXT_RETURNING, 0.0, 0, 0};
    uint32_t opn = 0;
    const HEnt* top0 = cache;
    const HEnt* top1 = cache + kHeapLds;
    const HEnt* top2 = cache + 2 * kHeapLds;
    HClk ck;
    ck.start();
    // each decision waits only for the heaps it reads: a due reservation
    // needs the resv top alone, the limit loop the limit top, the priority
    // pick the ready top (after every limit mark of the loop)
    auto wait_top = [&](int h) {
      ck.lap(1);
      lds_wait_ge(&s_done[h], opn);
      ck.lap(0);
    };
    uint32_t taken = 0;  // a lower bound of every heap wave's operations taken
    auto publish = [&](const HOp& o) {
      // (a limit operation's cursor load by the ready heap's wave: the
      // coordinator's stores to it complete first)
      if (o.type == kOpLimit) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // a free ring slot: every heap wave has taken operation opn - kHOps
      // (the counters only grow: re-read only when the last reading is
      // not enough)
      if (opn >= kHOps && taken < opn - kHOps + 1) {
        lds_wait_ge(&s_done[0], opn - kHOps + 1);
        lds_wait_ge(&s_done[1], opn - kHOps + 1);
        lds_wait_ge(&s_done[2], opn - kHOps + 1);
        const uint32_t t0 = lds_u32(&s_done[0]), t1 = lds_u32(&s_done[1]), t2 = lds_u32(&s_done[2]);
        taken = min(t0, min(t1, t2));
      }
      if (lane == 0) ring[opn % kHOps] = o;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ++opn;
      if (lane == 0) __atomic_store_n(&s_pub, opn, __ATOMIC_RELAXED);
    };
    while (r.n < k) {
      uint32_t pop_slot = kNone;
      bool pop_prio = false;
      if (n == 0) {  // no clients: none (:1118-1120)
        r.type = DMC_NEXT_NONE;
        break;
      }
      wait_top(kHResv);
      const HEnt rt = ld_lds<HEnt>(top0);
      if (rt.cls == 0 && hval(rt) <= now) {
        pop_slot = rt.slot;
      } else {
        for (;;) {  // the limit loop
          wait_top(kHLim);
          const HEnt lt = ld_lds<HEnt>(top1);
          if (!(lt.cls == 0 && hval(lt) <= now)) break;
          HOp o{};
          o.type = kOpLimit;
          o.s = lt.slot;
          o.X[1] = lt;
          o.X[1].cls = 1;  // (hent(kHLim, ...) of the record marked ready)
          publish(o);
          // ready = true: F_READY in the cursor word (head | count << 8 |
          // flags << 16 | stamp << 24, ScanRec offset 24), issued after the
          // publication (its completion is not waited for there: the ready
          // heap's wave reads the client's keys, not this bit); no other bit
          // of the word changes before the coordinator's next stores, which
          // heap_pop_state orders behind it
          if (lane == 0)
            __hip_atomic_fetch_or(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(tb.sc + lt.slot) +
                                                              offsetof(ScanRec, head)),
                                  (uint32_t)F_READY << 16, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
        wait_top(kHReady);
        const HEnt pt = ld_lds<HEnt>(top2);
        const bool ph = pt.cls != kClsNone && hval(pt) < kInf;
        if (pt.cls == 0 && ph) {
          pop_slot = pt.slot;
          pop_prio = true;
        } else if (at_limit == DMC_AT_LIMIT_ALLOW && ph) {
          pop_slot = pt.slot;
          pop_prio = true;
        } else if (at_limit == DMC_AT_LIMIT_ALLOW && rt.cls == 0 && hval(rt) < kInf) {
          pop_slot = rt.slot;
        }
      }
      if (pop_slot == kNone) {
        // future / none (:1170-1185), as k_heap_pull
        constexpr double kTimeMax = 1.7976931348623157e308;
        double next = kTimeMax;
        const HEnt r0 = ld_lds<HEnt>(top0), l0 = ld_lds<HEnt>(top1);
        if (r0.cls != kClsNone) {
          const double v = hval(r0);
          if (v != 0.0) next = v < next ? v : next;
        }
        if (l0.cls != kClsNone) {
          const double v = hval(l0);
          if (v != 0.0) next = v < next ? v : next;
        }
        if (next < kTimeMax) {
          r.type = DMC_NEXT_FUTURE;
          r.when = next;
        } else {
          r.type = DMC_NEXT_NONE;
        }
        break;
      }
      ScanRec o0, o1;
      ck.lap(1);
      heap_pop_state(tb, pop_slot, pop_prio, tick, out + r.n, sched, lane, true, false, nullptr,
                     &o0, &o1);
      ck.lap(2);
      HOp o{};
      o.type = kOpPop;
      o.s = pop_slot;
      o.prio = pop_prio ? 1u : 0u;
      _Pragma("unroll") for (int j = 0; j < 3; ++j) o.X[j] = hent(j, o0, pop_slot);
      o.Xu = hent(kHResv, o1, pop_slot);
      publish(o);
      ck.lap(3);
      ++r.n;
      if (pop_prio) ++r.n_prio;
      else ++r.n_res;
    }
    HOp e{};
    e.type = kOpEnd;
    publish(e);
    if (DMC_HEAP_CLOCKS && lane == 0 && r.n > 1000)
      printf("async coordinator: pulls %u | cycles per pull: waiting %.0f deciding %.0f pop state %.0f publish %.0f\n",
             r.n, (double)ck.t[0] / r.n, (double)ck.t[1] / r.n, (double)ck.t[2] / r.n, (double)ck.t[3] / r.n);
    if (lane == 0) {
      *res = r;
      if (d_result) {
        dmc_pull_result x{};
        x.n_decisions = r.n;
        x.next_type = r.type;
        x.when = r.type == DMC_NEXT_FUTURE ? r.when : 0.0;
        x.n_priority = r.n_prio;
        x.n_reservation = r.n_res;
        *d_result = x;
      }
    }
  }
  heap_cache_flush(hd, cache, T);
}
