"""Trace-level parity between the HIP engine and the oracle (test helper)."""
import numpy as np

import pyoracle
from dmclock_amd import workloads

STATE_FIELDS = ("prev_r", "prev_p", "prev_l", "prev_arrival", "prop_delta",
                "front_r", "front_p", "front_l", "front_arrival", "count",
                "cur_delta", "cur_rho", "idle", "front_ready")


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def compare_decisions(dg, do, where):
    assert len(dg) == len(do), (where, len(dg), len(do))
    for f in ("slot", "phase", "cost", "handle"):
        bad = np.nonzero(dg[f] != do[f])[0]
        assert bad.size == 0, (where, f, int(bad[0]), dg[bad[0]], do[bad[0]])
    for f in ("tag_r", "tag_p", "tag_l"):
        bad = np.nonzero(bits(dg[f]) != bits(do[f]))[0]
        assert bad.size == 0, (where, f, int(bad[0]), dg[bad[0]], do[bad[0]])


INFO_FIELDS = ("r_inv", "w_inv", "l_inv")  # the cached client.info


def compare_states(qg, qo, slots, where="", info=False):
    fields = STATE_FIELDS + (INFO_FIELDS if info else ())
    for s in slots:
        sg, so = qg.client_state(int(s)), qo.client_state(int(s))
        assert (sg is None) == (so is None), (where, s)
        if sg is None:
            continue
        for f in fields:
            a, b = getattr(sg, f), getattr(so, f)
            if isinstance(a, float):
                if f.startswith("front") and not so.count:
                    continue
                assert np.float64(a).view(np.uint64) == \
                    np.float64(b).view(np.uint64), (where, s, f, a, b)
            else:
                assert a == b, (where, s, f, a, b)


def run_parity(trace, mk_gpu, queue_kw=None, state_sample=64, require_tie_free=True,
               gpu_kw=None, info=False):
    """Replay `trace` on both engines op by op and compare every output."""
    queue_kw = queue_kw or {}
    qo = pyoracle.OracleQueue(**queue_kw)
    qg = mk_gpu(max_clients=int(trace.clients.slots.max()) + 1, **queue_kw,
                **(gpu_kw or {}))
    outs_o = workloads.replay(qo, trace)
    ties = qo.ties
    if require_tie_free:
        assert ties == 0, f"trace has {ties} tied decisions; pick another seed"
    outs_g = workloads.replay(qg, trace)
    n_dec = 0
    for i, (a, b) in enumerate(zip(outs_g, outs_o)):
        assert a[0] == b[0]
        if a[0] == "add":
            assert np.array_equal(a[1], b[1]), (i, np.nonzero(a[1] != b[1]))
        elif a[0] == "pull":
            compare_decisions(a[1], b[1], f"op {i}")
            assert a[2] == b[2], (i, a[2], b[2])
            n_dec += len(a[1])
    rng = np.random.default_rng(0)
    slots = trace.clients.slots
    sample = rng.choice(slots, min(state_sample, len(slots)), replace=False)
    compare_states(qg, qo, sample, "final", info=info)
    assert qg.request_count() == qo.request_count()
    assert tuple(qg.sched_counts()) == tuple(qo.sched_counts())
    return n_dec, qg, qo



def activation_batches(trace, queue_kw):
    """Replays `trace` on the oracle one request at a time and returns (add
    batches holding an activation, of those the batches with a "hard" one:
    an activated client left with an empty queue -- its activating request
    rejected under AtLimit::Reject -- whose proportion basis a later request
    of the same batch moves; the engine resolves those batches in order with
    one wave, k_act_hard, and counts them in act_seq_batches)."""
    qo = pyoracle.OracleQueue(**queue_kw)
    c = trace.clients
    qo.register(c.slots, c.r, c.w, c.l, c.active)
    n_act = n_hard = 0
    for op in trace.ops:
        if op[0] == "add":
            reqs = op[1]
            act = hard = False
            watched = {}  # activated, still empty: slot -> basis bits
            for i in range(len(reqs)):
                s = int(reqs["slot"][i])
                pre = qo.client_state(s)
                qo.add_batch(reqs[i:i + 1])
                if pre is None or not pre.registered:
                    continue
                post = qo.client_state(s)
                basis = post.front_p if post.count else post.prev_p
                if pre.idle and reqs["rho"][i] <= reqs["delta"][i]:
                    act = True
                    if post.count == 0:
                        watched[s] = np.float64(basis).view(np.uint64)
                elif s in watched:
                    if np.float64(basis).view(np.uint64) != watched[s]:
                        hard = True
                    if post.count:
                        del watched[s]
                    else:
                        watched[s] = np.float64(basis).view(np.uint64)
            n_act += act
            n_hard += hard
        elif op[0] == "pull":
            qo.pull_batch(op[1], op[2])
        elif op[0] == "idle":
            for s in op[1].tolist():
                qo.mark_idle(s)
        else:
            raise ValueError(op[0])
    return n_act, n_hard
