"""Pin the oracle (CPU restatement) against the reference's own known answers.

The reference is unbuildable in this image (Boost.Variant and GTest are
absent), so the oracle's parity is pinned here, by every known-answer test the
reference's suites hold for this path:
  * test/test_dmclock_server.cc        -> tests/kats.py (SERVER_KATS)
  * support/test/test_indirect_intrusive_heap.cc -> the heap tests below
  * test/test_dmclock_client.cc        -> the tracker tests below
"""
import random

import pytest

import kats
import pyoracle


def mk_oracle(**kw):
    return pyoracle.OracleQueue(**kw)


@pytest.mark.parametrize("kat", kats.SERVER_KATS, ids=lambda f: f.__name__)
def test_server_kat_oracle(kat):
    kat(mk_oracle)


def test_client_idle_erase_oracle():
    """test_dmclock_server.cc:100-185 restated with explicit mark points:
    a client whose last tick is at or before the idle point becomes idle; at or
    before the erase point it is erased (do_clean, dmclock_server.h:1206-1255)."""
    q = mk_oracle()
    q.set_info(17, 100.0, 1.0, 0.0)
    assert q.client_count() == 0
    assert q.add(17, kats.T0) == 0
    st = q.client_state(17)
    assert st.idle == 0 and q.client_count() == 1
    tick = q.tick()
    assert q.clean(0, tick) == 0
    assert q.client_state(17).idle == 1
    assert q.clean(tick, 0) == 1
    assert q.client_count() == 0 and q.client_state(17) is None


def test_clean_erase_max_order_oracle():
    """do_clean erases at most erase_max per pass, in client-id order, and
    idles the rest that are old enough (:1232-1249)."""
    q = mk_oracle()
    for c in (5, 3, 9, 1):
        q.set_info(c, 0.0, 1.0, 0.0)
        q.add(c, kats.T0)
    tick = q.tick()
    assert q.clean(tick, tick, 2) == 2
    assert q.client_state(1) is None and q.client_state(3) is None
    assert q.client_state(5).idle == 1 and q.client_state(9).idle == 1


# ------------------------------------------------------------------ heap KATs
SEVEN = [2, 99, 1, -5, 12, -12, -7]


def _drain(h):
    out = []
    while len(h):
        out.append(h.top())
        h.pop()
    return out


@pytest.mark.parametrize("k", [2, 3, 4, 10])
def test_heap_k(k):
    """test_indirect_intrusive_heap.cc shared_ptr/unique_ptr/regular_ptr/K_3/K_4/K_10."""
    h = pyoracle.IntHeap(k)
    for v in SEVEN:
        h.push_value(v)
    assert _drain(h) == [-12, -7, -5, 1, 2, 12, 99]


def test_heap_multi_k():
    """multi_K: the same random values come out identically from K=2,3,4,10."""
    rng = random.Random(1234)
    heaps = [pyoracle.IntHeap(k) for k in (2, 3, 4, 10)]
    for _ in range(250):
        v = rng.randrange(201) - 100
        for h in heaps:
            h.push_value(v)
    outs = [_drain(h) for h in heaps]
    assert outs[0] == sorted(outs[0])
    for o in outs[1:]:
        assert o == outs[0]


def test_heap_demote():
    h = pyoracle.IntHeap()
    ids = [h.push_value(v) for v in SEVEN]
    top_id = ids[SEVEN.index(-12)]
    h.set(top_id, 24)
    h.demote(h, top_id)
    assert h.top() == -7
    for _ in range(5):
        h.pop()
    assert h.top() == 24


def test_heap_demote_not():
    h = pyoracle.IntHeap()
    ids = [h.push_value(v) for v in SEVEN]
    top_id = ids[SEVEN.index(-12)]
    h.set(top_id, -99)
    h.demote(h, top_id)
    assert h.top() == -99
    h.pop()
    assert h.top() == -7


def test_heap_promote_and_demote():
    h = pyoracle.IntHeap()
    ids = [h.push_value(v) for v in SEVEN]
    d1 = ids[SEVEN.index(1)]
    assert h.top() == -12
    h.set(d1, -99)
    h.promote(h, d1)
    assert h.top() == -99
    h.set(d1, 999)
    h.demote(h, d1)
    assert h.top() == -12
    h.set(d1, 9)
    h.promote(h, d1)
    for _ in range(4):
        h.pop()
    assert h.top() == 9


def test_heap_adjust():
    h = pyoracle.IntHeap()
    ids = [h.push_value(v) for v in SEVEN]
    d1 = ids[SEVEN.index(1)]
    h.set(d1, 999)
    h.adjust(h, d1)
    assert h.top() == -12
    h.set(d1, -99)
    h.adjust(h, d1)
    assert h.top() == -99
    h.set(d1, 9)
    h.adjust(h, d1)
    assert h.top() == -12
    for _ in range(4):
        h.pop()
    assert h.top() == 9


def test_heap_remove_careful():
    """remove must sift (not sift_down) the moved element: array order after
    removing 200 is 0, 10, 40, 20, 30, 100 (:607-648)."""
    h = pyoracle.IntHeap(2)
    for v in (0, 10, 100, 20, 30, 200, 300, 40):
        h.push_value(v)
    assert h.remove_value(200)
    assert h.dump()[:6] == [0, 10, 40, 20, 30, 100]


def test_heap_remove_greatest():
    """:650-700 -- removing the upper half (greatest first in shuffled order)
    leaves the lower half popping in order."""
    num = 4096
    vals = list(range(num))
    rng = random.Random(0)
    rng.shuffle(vals)
    h = pyoracle.IntHeap(2)
    for v in vals:
        h.push_value(v)
    for v in range(num // 2, num):
        assert h.remove_value(v)
    assert _drain(h) == list(range(num // 2))


def test_heap_iterator_remove():
    """HeapFixture1.iterator_remove (:902-935)."""
    h = pyoracle.IntHeap()
    for v in SEVEN:
        h.push_value(v)
    assert h.remove_value(-7)
    assert -7 not in h.dump()
    assert _drain(h) == [-12, -5, 1, 2, 12, 99]


def test_heap_shared_data():
    """HeapFixture1.shared_data: one element set in two heaps with different
    comparators, adjusted in both (:741-800)."""
    src = pyoracle.IntHeap(2, mode=0)
    alt = pyoracle.IntHeap(2, mode=1, alt_index=True)
    ids = [src.new(v) for v in SEVEN]
    for e in ids:
        src.push(src, e)
    for e in ids:
        alt.push(src, e)
    d3 = ids[2]  # data3 == 1
    src.set(d3, 32)
    src.adjust(src, d3)
    alt.adjust(src, d3)
    assert _drain(src) == [-12, -7, -5, 2, 12, 32, 99]
    got = []
    for _ in range(7):
        got.append(alt.top())
        alt.pop()
    assert got == [32, 12, 2, -12, 99, -5, -7]


# ------------------------------------------------------------------ tracker KATs
def test_tracker_orig():
    """test_dmclock_client.cc:231-304 (OrigTracker)."""
    st = pyoracle.Tracker("orig")
    s1, s2 = 101, 7
    R, P = 0, 1
    assert st.get_req_params(s1) == (1, 1)
    assert st.get_req_params(s1) == (0, 0)
    st.track_resp(s1, P)
    assert st.get_req_params(s1) == (0, 0)
    st.track_resp(s2, P)
    assert st.get_req_params(s1) == (1, 0)
    assert st.get_req_params(s1) == (0, 0)
    st.track_resp(s2, R)
    assert st.get_req_params(s1) == (1, 1)
    for s, ph in ((s2, R), (s1, P), (s2, P), (s2, R), (s1, R), (s1, P),
                  (s2, P)):
        st.track_resp(s, ph)
    assert st.get_req_params(s1) == (4, 2)
    assert st.get_req_params(s2) == (3, 1)
    assert st.get_req_params(s1) == (0, 0)
    assert st.get_req_params(s2) == (0, 0)


def test_tracker_borrowing():
    """test_dmclock_client.cc:108-225 (BorrowingTracker)."""
    st = pyoracle.Tracker("borrowing")
    s1, s2 = 101, 7
    R, P = 0, 1
    assert st.get_req_params(s1) == (1, 1)
    assert st.get_req_params(s1) == (1, 1)
    st.track_resp(s1, P)
    assert st.get_req_params(s1) == (1, 1)
    st.track_resp(s2, P)
    assert st.get_req_params(s1) == (1, 1)
    assert st.get_req_params(s1) == (1, 1)
    st.track_resp(s2, R)
    assert st.get_req_params(s1) == (1, 1)
    for s, ph in ((s2, R), (s1, P), (s2, P), (s2, R), (s1, R), (s1, P),
                  (s2, P)):
        st.track_resp(s, ph)
    assert st.get_req_params(s1) == (5, 1)
    assert st.get_req_params(s2) == (9, 4)
    assert st.get_req_params(s1) == (1, 1)
    assert st.get_req_params(s2) == (1, 1)
