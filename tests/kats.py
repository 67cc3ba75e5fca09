"""Known-answer tests of the reference, restated engine-independently.

Each function re-expresses one gtest of /root/reference/test/test_dmclock_server.cc
with explicit times in place of get_time(); `mk(**params)` builds a queue
(the oracle restatement or the HIP engine, both exposing the same Python API:
set_info / add / pull / pull_batch / request_count / client_count /
remove_by_client / remove_by_req_filter / update_client_info).

The expected values are the reference's own assertions (cited per test).
"""
import errno

from dmclock_amd._abi import (AT_LIMIT_ALLOW, AT_LIMIT_REJECT, AT_LIMIT_WAIT,
                              DMC_EBADTAG, NEXT_FUTURE, NEXT_NONE,
                              NEXT_RETURNING, PHASE_PRIORITY,
                              PHASE_RESERVATION)

T0 = 1000.0  # explicit time base standing in for get_time()


def _count(q, now, n, c1, c2, phase=None, skip_after=None):
    a = b = 0
    for i in range(n):
        t, d, _ = q.pull(now)
        assert t == NEXT_RETURNING, (i, t)
        if skip_after is not None and i > skip_after:
            continue
        if phase is not None:
            assert d["phase"] == phase
        if d["slot"] == c1:
            a += 1
        elif d["slot"] == c2:
            b += 1
        else:
            raise AssertionError("got request from neither of two clients")
    return a, b


def kat_pull_weight(mk):
    """test_dmclock_server.cc:822-874 -- weights 1:2 give 2:4 of 6."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1, c2 = 17, 98
    q.set_info(c1, 0.0, 1.0, 0.0)
    q.set_info(c2, 0.0, 2.0, 0.0)
    t = T0
    for _ in range(5):
        assert q.add(c1, t) == 0
        t += 1e-6
        assert q.add(c2, t) == 0
        t += 1e-6
    assert _count(q, T0 + 1.0, 6, c1, c2, PHASE_PRIORITY) == (2, 4)


def kat_pull_reservation(mk):
    """test_dmclock_server.cc:877-929 -- reservations 2:1 give 4:2 of 6."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1, c2 = 52, 8
    q.set_info(c1, 2.0, 0.0, 0.0)
    q.set_info(c2, 1.0, 0.0, 0.0)
    old = T0 - 100.0
    for _ in range(5):
        assert q.add(c1, old) == 0
        assert q.add(c2, old) == 0
        old += 0.001
    assert _count(q, T0, 6, c1, c2, PHASE_RESERVATION) == (4, 2)


def kat_update_client_info(mk):
    """test_dmclock_server.cc:932-1018 -- 2:4 before, 3:3 after the update."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1, c2 = 17, 98
    q.set_info(c1, 0.0, 100.0, 0.0)
    q.set_info(c2, 0.0, 200.0, 0.0)
    t = T0
    for _ in range(5):
        assert q.add(c1, t) == 0
        t += 1e-6
        assert q.add(c2, t) == 0
        t += 1e-6
    assert _count(q, T0 + 0.5, 10, c1, c2, PHASE_PRIORITY,
                  skip_after=5) == (2, 4)
    # `info1 = dmc::ClientInfo(0.0, 200.0, 0.0); pq->update_client_info(17);`
    q.set_info(c1, 0.0, 200.0, 0.0)
    q.update_client_info(c1)
    t = T0 + 1.0
    for _ in range(5):
        assert q.add(c1, t) == 0
        t += 1e-6
        assert q.add(c2, t) == 0
        t += 1e-6
    assert _count(q, T0 + 1.5, 6, c1, c2, PHASE_PRIORITY) == (3, 3)


def kat_dynamic_cli_info_f(mk):
    """test_dmclock_server.cc:1021-1114 -- Delayed + U1: 2:4 then 6:2."""
    q = mk(at_limit=AT_LIMIT_WAIT, delayed=True, dynamic_info=True)
    c1, c2 = 17, 98
    q.set_info(c1, 0.0, 100.0, 0.0)
    q.set_info(c2, 0.0, 200.0, 0.0)
    t = T0
    for _ in range(5):
        assert q.add(c1, t) == 0
        t += 1e-6
        assert q.add(c2, t) == 0
        t += 1e-6
    assert _count(q, T0 + 0.5, 10, c1, c2, PHASE_PRIORITY,
                  skip_after=5) == (2, 4)
    # cli_info_group = 1: client_info_f now returns different objects
    q.set_info(c1, 0.0, 150.0, 0.0, fresh=True)
    q.set_info(c2, 0.0, 50.0, 0.0, fresh=True)
    t = T0 + 1.0
    for _ in range(6):
        assert q.add(c1, t) == 0
        t += 1e-6
        assert q.add(c2, t) == 0
        t += 1e-6
    assert _count(q, T0 + 1.5, 8, c1, c2, PHASE_PRIORITY) == (6, 2)


def kat_ready_and_under_limit(mk):
    """test_dmclock_server.cc:1120-1181 -- retn, retn, future, x3, then none."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1, c2 = 52, 8
    q.set_info(c1, 1.0, 0.0, 0.0)
    q.set_info(c2, 1.0, 0.0, 0.0)
    st = T0 - 100.0
    for _ in range(3):
        assert q.add(c1, st, delta=0, rho=0) == 0
        assert q.add(c2, st, delta=0, rho=0) == 0
    seq = []
    for now in (st + 0.5, st + 1.5, st + 2.5):
        for _ in range(3):
            seq.append(q.pull(now)[0])
    R, F, N = NEXT_RETURNING, NEXT_FUTURE, NEXT_NONE
    assert seq == [R, R, F, R, R, F, R, R, N]


def kat_pull_none(mk):
    """test_dmclock_server.cc:1184-1205."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    assert q.pull(T0 + 100)[0] == NEXT_NONE


def kat_pull_future(mk):
    """test_dmclock_server.cc:1208-1236 -- future at exactly now + 100."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1 = 52
    q.set_info(c1, 1.0, 0.0, 1.0)
    assert q.add(c1, T0 + 100) == 0
    t, _, when = q.pull(T0)
    assert t == NEXT_FUTURE
    assert when == T0 + 100


def kat_pull_future_limit_break_weight(mk):
    """test_dmclock_server.cc:1239-1267."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1 = 52
    q.set_info(c1, 0.0, 1.0, 1.0)
    assert q.add(c1, T0 + 100) == 0
    t, d, _ = q.pull(T0)
    assert t == NEXT_RETURNING
    assert d["slot"] == c1


def kat_pull_future_limit_break_reservation(mk):
    """test_dmclock_server.cc:1270-1298."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1 = 52
    q.set_info(c1, 1.0, 0.0, 1.0)
    assert q.add(c1, T0 + 100) == 0
    t, d, _ = q.pull(T0)
    assert t == NEXT_RETURNING
    assert d["slot"] == c1


def kat_pull_reject_at_limit(mk):
    """test_dmclock_server.cc:1301-1336 -- 0,0,0,EAGAIN,EAGAIN,0; 0,EAGAIN."""
    q = mk(at_limit=AT_LIMIT_REJECT)
    c1, c2 = 52, 53
    q.set_info(c1, 0.0, 1.0, 1.0)
    q.set_info(c2, 0.0, 1.0, 1.0)
    got = [q.add(c1, t, delta=0, rho=0) for t in (1.0, 2.0, 3.0, 3.9, 4.0, 6.0)]
    assert got == [0, 0, 0, errno.EAGAIN, errno.EAGAIN, 0]
    assert q.add(c2, 1.0, delta=0, rho=0, handle=1) == 0
    assert q.add(c2, 1.0, delta=0, rho=0, handle=2) == errno.EAGAIN


def kat_pull_reject_threshold(mk):
    """test_dmclock_server.cc:1339-1360 -- threshold 3.0."""
    q = mk(at_limit=AT_LIMIT_REJECT, reject_threshold=3.0)
    c1 = 52
    q.set_info(c1, 0.0, 1.0, 1.0)
    got = [q.add(c1, t, delta=0, rho=0) for t in (1.0, 1.0, 1.0, 1.0, 1.0, 3.0)]
    assert got == [0, 0, 0, 0, errno.EAGAIN, 0]


def kat_pull_wait_at_limit(mk):
    """test_dmclock_server.cc:1363-1471."""
    q = mk(at_limit=AT_LIMIT_WAIT)
    c1, c2 = 52, 8
    q.set_info(c1, 1.0, 2.0, 100.0)
    q.set_info(c2, 1.0, 1.0, 2.0)
    old = T0
    t = old
    for _ in range(50):
        assert q.add(c1, t) == 0
        assert q.add(c2, t) == 0
        t += 0.01
    assert q.client_count() == 2
    assert q.request_count() == 100
    now = old + 1.0 + 1e-3
    assert _count(q, now, 2, c1, c2, PHASE_RESERVATION) == (1, 1)
    assert q.request_count() == 98
    a, b = _count(q, now, 50, c1, c2, PHASE_PRIORITY)
    assert q.request_count() == 48
    assert (a + 1, b + 1) == (50, 2)
    t, _, when = q.pull(now)
    assert t == NEXT_FUTURE
    assert when == old + 2.0
    t, d, _ = q.pull(old + 2.0)
    assert t == NEXT_RETURNING
    assert d["slot"] == c2
    assert q.request_count() == 47


def kat_delayed_tag_calc(mk):
    """test_dmclock_server.cc:273-316 -- Delayed: future t+11; Immediate: t+12."""
    c1 = 17
    t = 1.0
    q = mk(delayed=True)
    q.set_info(c1, 0.0, 1.0, 1.0)
    q.add(c1, t, delta=0, rho=0)
    q.add(c1, t + 1, delta=0, rho=0)
    q.add(c1, t + 2, delta=10, rho=10)
    assert q.pull(t)[0] == NEXT_RETURNING
    tt, _, when = q.pull(t + 1)
    assert tt == NEXT_FUTURE and when == t + 11
    q = mk(delayed=False)
    q.set_info(c1, 0.0, 1.0, 1.0)
    q.add(c1, t, delta=0, rho=0)
    q.add(c1, t + 1, delta=0, rho=0)
    q.add(c1, t + 2, delta=10, rho=10)
    assert q.pull(t)[0] == NEXT_RETURNING
    assert q.pull(t + 1)[0] == NEXT_RETURNING
    tt, _, when = q.pull(t + 2)
    assert tt == NEXT_FUTURE and when == t + 12


def _add_ids(q, seq, t0=T0, delta=1, rho=1):
    """add (client, id) pairs with the id as request handle."""
    t = t0
    for c, rid in seq:
        assert q.add(c, t, delta=delta, rho=rho, handle=rid) == 0
        t += 1e-6


def kat_remove_by_req_filter(mk):
    """test_dmclock_server.cc:373-440 -- sum of captured = 146."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1, c2 = 17, 98
    q.set_info(c1, 0.0, 1.0, 0.0)
    q.set_info(c2, 0.0, 1.0, 0.0)
    assert q.client_count() == 0 and q.request_count() == 0
    _add_ids(q, [(c1, 1), (c1, 11), (c2, 2), (c2, 0), (c2, 13), (c2, 2),
                 (c2, 13), (c2, 98), (c1, 44)])
    assert q.client_count() == 2 and q.request_count() == 9
    q.remove_by_req_filter(lambda h: h % 2 == 1)
    assert q.request_count() == 5
    capture = []

    def f(h):
        if h % 2 == 0:
            capture.insert(0, h)
            return True
        return False
    q.remove_by_req_filter(f, backwards=True)
    assert q.request_count() == 0
    assert len(capture) == 5
    assert sum(capture) == 146


def kat_remove_by_req_filter_forwards(mk):
    """test_dmclock_server.cc:443-523."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1 = 17
    q.set_info(c1, 0.0, 1.0, 0.0)
    _add_ids(q, [(c1, i) for i in range(1, 7)])
    assert q.client_count() == 1 and q.request_count() == 6
    cap = []

    def odd(h):
        if h % 2 == 1:
            cap.append(h)
            return True
        return False
    q.remove_by_req_filter(odd, backwards=False)
    assert q.request_count() == 3 and cap == [1, 3, 5]
    cap2 = []

    def even(h):
        if h % 2 == 0:
            cap2.insert(0, h)
            return True
        return False
    q.remove_by_req_filter(even, backwards=False)
    assert q.request_count() == 0 and cap2 == [6, 4, 2]


def kat_remove_by_req_filter_backwards(mk):
    """test_dmclock_server.cc:526-605."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1 = 17
    q.set_info(c1, 0.0, 1.0, 0.0)
    _add_ids(q, [(c1, i) for i in range(1, 7)])
    cap = []

    def odd(h):
        if h % 2 == 1:
            cap.insert(0, h)
            return True
        return False
    q.remove_by_req_filter(odd, backwards=True)
    assert q.request_count() == 3 and cap == [1, 3, 5]
    cap2 = []

    def even(h):
        if h % 2 == 0:
            cap2.append(h)
            return True
        return False
    q.remove_by_req_filter(even, backwards=True)
    assert q.request_count() == 0 and cap2 == [6, 4, 2]


def kat_remove_by_client(mk):
    """test_dmclock_server.cc:608-681."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1, c2 = 17, 98
    q.set_info(c1, 0.0, 1.0, 0.0)
    q.set_info(c2, 0.0, 1.0, 0.0)
    _add_ids(q, [(c1, 1), (c1, 11), (c2, 2), (c2, 0), (c2, 13), (c2, 2),
                 (c2, 13), (c2, 98), (c1, 44)])
    assert q.client_count() == 2 and q.request_count() == 9
    removed = []
    for h in q.remove_by_client(c1, reverse=True):
        removed.insert(0, int(h))
    assert removed == [1, 11, 44]
    assert q.request_count() == 6
    t, d, _ = q.pull(T0 + 1.0)
    assert t == NEXT_RETURNING and d["handle"] == 2
    t, d, _ = q.pull(T0 + 1.0)
    assert t == NEXT_RETURNING and d["handle"] == 0
    q.remove_by_client(c2)
    assert q.request_count() == 0


def kat_add_req_ref(mk):
    """test_dmclock_server.cc:684-751 -- sum 9."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1, c2 = 22, 44
    q.set_info(c1, 0.0, 1.0, 0.0)
    q.set_info(c2, 0.0, 1.0, 0.0)
    _add_ids(q, [(c1, 1), (c2, 2), (c1, 3), (c2, 4), (c2, 5)])
    assert q.client_count() == 2 and q.request_count() == 5
    q.remove_by_req_filter(lambda h: h % 2 == 0)
    assert q.request_count() == 3
    cap = []

    def odd(h):
        if h % 2 == 1:
            cap.insert(0, h)
            return True
        return False
    q.remove_by_req_filter(odd, backwards=True)
    assert q.request_count() == 0 and len(cap) == 3 and sum(cap) == 9


def kat_add_req_ref_null_req_params(mk):
    """test_dmclock_server.cc:754-819 -- null ReqParams, sum 6."""
    q = mk(at_limit=AT_LIMIT_ALLOW)
    c1, c2 = 22, 44
    q.set_info(c1, 0.0, 1.0, 0.0)
    q.set_info(c2, 0.0, 1.0, 0.0)
    _add_ids(q, [(c1, 1), (c2, 2), (c1, 3), (c2, 4), (c2, 5)], delta=0, rho=0)
    assert q.client_count() == 2 and q.request_count() == 5
    q.remove_by_req_filter(lambda h: h % 2 == 1)
    assert q.request_count() == 2
    cap = []

    def even(h):
        if h % 2 == 0:
            cap.insert(0, h)
            return True
        return False
    q.remove_by_req_filter(even, backwards=True)
    assert q.request_count() == 0 and len(cap) == 2 and sum(cap) == 6


def kat_bad_tag(mk):
    """test_dmclock_server.cc:51-97 -- r = w = 0 is refused (the reference
    asserts; here a status code comes back)."""
    q = mk(delayed=True)
    c1, c2 = 17, 18
    q.set_info(c1, 0.0, 0.0, 0.0)
    q.set_info(c2, 0.0, 0.0, 1.0)
    assert q.add(c1, T0) == DMC_EBADTAG
    assert q.add(c2, T0) == DMC_EBADTAG


SERVER_KATS = [
    kat_pull_weight, kat_pull_reservation, kat_update_client_info,
    kat_dynamic_cli_info_f, kat_ready_and_under_limit, kat_pull_none,
    kat_pull_future, kat_pull_future_limit_break_weight,
    kat_pull_future_limit_break_reservation, kat_pull_reject_at_limit,
    kat_pull_reject_threshold, kat_pull_wait_at_limit, kat_delayed_tag_calc,
    kat_remove_by_req_filter, kat_remove_by_req_filter_forwards,
    kat_remove_by_req_filter_backwards, kat_remove_by_client, kat_add_req_ref,
    kat_add_req_ref_null_req_params, kat_bad_tag,
]
