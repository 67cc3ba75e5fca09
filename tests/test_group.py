"""Queue groups (dmc_group, BASELINE config 5's per-GPU shape) against the same
queues driven one by one (needs an MI355X).

A group step must do, for every member, exactly what dmc_tracker_fill +
dmc_add_pull_batch_device + dmc_tracker_tally do on that queue alone
(include/dmclock_gpu.h; servers are independent queues,
sim/src/simulate.h:118-136).  The oracle-checked multi-table parity is
tests/test_concurrency.py::test_group_queues_trackers_parity_8; here:

  * the bench's own shape, 8 tables of 2,097,152 slots (bench.py --config 5):
    the grouped run and a run of eight separate queues on the same workload
    produce byte-identical decisions, result records, add statuses and
    tracker state (the same shape against eight oracle queues and the epoch
    restatement: tests/test_concurrency.py::test_group_bench_shape_vs_oracle);
  * a group whose steps cannot be fused (k below the round size, idle
    clients waiting for activation) falls back to per-member calls with the
    same results.
"""
import hashlib

import numpy as np
import pytest

from dmclock_amd import workloads
from dmclock_amd._abi import DECISION_DTYPE, PullResult

pytestmark = pytest.mark.gpu


def _workload(S, N, depth, n_steps, batch, seed):
    out = []
    for s in range(S):
        tab = workloads.client_table(np.random.default_rng([seed, s]), N)
        rng = np.random.default_rng([seed, 1000, s])
        perm = rng.permutation(N)
        tab.r, tab.w, tab.l = tab.r[perm], tab.w[perm], tab.l[perm]
        cmap = (s * N + perm).astype(np.int32)
        pre = workloads.arrivals(rng, N, depth * N, 1.0, 2.0 * N)
        t = float(pre["time"][-1])
        steps, h = [], len(pre)
        for _ in range(n_steps):
            b = workloads.arrivals(rng, N, batch, t, 2.0 * N, handle_base=h)
            h += batch
            t = float(b["time"][-1])
            steps.append(b)
        out.append((tab, cmap, pre, steps))
    return out


def _drive(wl, N, k, grouped, settle, idle_every=0, epoch=4, options=(), lagged=False):
    """one pass over the workload; returns digests of every output"""
    import torch
    from dmclock_amd.multiserver import DeviceTrackers, GpuGroup, make_queues
    dev = torch.device("cuda", 0)
    S = len(wl)
    chunk = 1 << 20
    qs = make_queues(S, N, device=0, ring_capacity=64, max_batch=chunk)
    for q in qs:
        for opt, val in options:
            q.set_option(opt, val)
    trk = DeviceTrackers(qs, N, dev, n_clients=S * N,
                         client_of_slot=np.stack([w[1] for w in wl]), lagged=lagged)
    group = GpuGroup(qs) if grouped else None
    if group is not None and lagged:
        trk.attach_group(group)
    d_rc = [torch.zeros(chunk, dtype=torch.int32, device=dev) for _ in range(S)]
    n_steps = len(wl[0][3])
    d_out = [torch.zeros(max(k, chunk) * DECISION_DTYPE.itemsize, dtype=torch.uint8,
                         device=dev) for _ in range(S)]
    d_res = torch.zeros((S, n_steps + 64, 24), dtype=torch.uint8, device=dev)
    digest = [hashlib.sha256() for _ in range(S)]
    for s, (tab, _, pre, _) in enumerate(wl):
        q = qs[s]
        q.register_active(tab.slots, tab.r, tab.w, tab.l)
        for i in range(0, len(pre), chunk):
            part = torch.from_numpy(pre[i:i + chunk].view(np.uint8)).to(dev)
            n = len(pre[i:i + chunk])
            torch.cuda.synchronize()
            trk.fill(s, part.data_ptr(), n)
            q.add_batch_device(part.data_ptr(), n, d_rc[s].data_ptr())
            q.sync()
            assert int((d_rc[s][:n] != 0).sum()) == 0
        done, j = 0, n_steps
        while done < settle:
            kk = min(settle - done, chunk)
            q.pull_batch_device(float(pre["time"][-1]), kk, d_out[s].data_ptr(),
                                d_res[s, j].data_ptr())
            trk.tally(s, d_out[s].data_ptr(), d_res[s, j].data_ptr(), kk)
            q.sync()
            done += kk
            j += 1
    trk.deliver()
    for q in qs:
        q.counters(reset=True)  # (the steps' own)
    d_steps = [[torch.from_numpy(b.view(np.uint8)).to(dev) for b in w[3]] for w in wl]
    torch.cuda.synchronize()
    gtrk = trk.group_trackers()
    rng = np.random.default_rng(5)
    for i in range(n_steps):
        if idle_every and i % idle_every == idle_every - 1:
            for s in range(S):  # do_clean's idle marking between steps
                qs[s].mark_idle_batch(rng.choice(N, N // 20, replace=False)
                                      .astype(np.uint32))
        nows = [float(w[3][i]["time"][-1]) for w in wl]
        if grouped:
            if lagged:  # (the current tally half)
                gtrk = trk.group_trackers()
            group.step(len(wl[0][3][i]), [d_steps[s][i].data_ptr() for s in range(S)],
                       [d.data_ptr() for d in d_rc], nows, k,
                       [d.data_ptr() for d in d_out],
                       [d_res[s, i].data_ptr() for s in range(S)], gtrk)
        else:
            for s in range(S):
                q = qs[s]
                trk.fill(s, d_steps[s][i].data_ptr(), len(wl[s][3][i]))
                q.add_pull_batch_device(d_steps[s][i].data_ptr(), len(wl[s][3][i]),
                                        d_rc[s].data_ptr(), nows[s], k, d_out[s].data_ptr(),
                                        d_res[s, i].data_ptr())
                trk.tally(s, d_out[s].data_ptr(), d_res[s, i].data_ptr(), k)
        for q in qs:
            q.sync()
        for s in range(S):
            r = PullResult.from_buffer_copy(d_res[s, i].cpu().numpy().tobytes())
            digest[s].update(d_res[s, i].cpu().numpy().tobytes())
            digest[s].update(d_out[s][:r.n_decisions * DECISION_DTYPE.itemsize]
                             .cpu().numpy().tobytes())
            digest[s].update(d_rc[s][:len(wl[s][3][i])].cpu().numpy().tobytes())
        if (i + 1) % epoch == 0:
            trk.deliver()
    if lagged:
        trk.finish()
    st = trk.state()
    ctr = [q.counters() for q in qs]
    out = {"digest": [d.hexdigest() for d in digest],
           "trk": hashlib.sha256(b"".join(st[f].tobytes() for f in
                                          ("gd", "gr", "xd", "xr", "known"))).hexdigest(),
           "fused": [c["fused_calls"] for c in ctr],
           "decisions": [c["decisions"] for c in ctr],
           "retries": [c["sample_retries"] for c in ctr],
           "rounds": [c["rounds"] for c in ctr]}
    if group is not None:
        group.close()
    for q in qs:
        q.close()
    torch.cuda.synchronize()
    return out


@pytest.mark.timeout(600)
def test_group_bench_shape_vs_separate_queues():
    """8 tables x 2,097,152 slots (bench.py --config 5 per GPU), depth 4,
    a 2M-pull settle per table, then 8 steps of 64K adds + 64K pulls per table
    with device trackers and an epoch delivery every 4 steps: the grouped run
    (one launch per kernel over the eight tables) and eight separate queues
    give identical bytes everywhere."""
    S, N, k = 8, 1 << 21, 1 << 16
    wl = _workload(S, N, 4, 8, k, seed=42)
    a = _drive(wl, N, k, grouped=True, settle=1 << 21)
    b = _drive(wl, N, k, grouped=False, settle=1 << 21)
    assert a["fused"] == [8] * S, a["fused"]
    assert a["digest"] == b["digest"]
    assert a["trk"] == b["trk"]
    assert a["decisions"] == b["decisions"]


@pytest.mark.timeout(300)
def test_group_lagged_side_stream_sums():
    """the overlapped (lagged) epoch delivery with the per-client sums on the
    group's side stream beside the next epoch's steps
    (dmc_group_tracker_collect_sums / _join): identical bytes and tracker
    state to separate queues collecting on their own streams"""
    S, N, k = 4, 1 << 16, 1 << 12
    wl = _workload(S, N, 4, 9, k, seed=17)
    a = _drive(wl, N, k, grouped=True, settle=N, epoch=2, lagged=True)
    b = _drive(wl, N, k, grouped=False, settle=N, epoch=2, lagged=True)
    assert a["digest"] == b["digest"]
    assert a["trk"] == b["trk"]
    assert a["decisions"] == b["decisions"]


@pytest.mark.timeout(300)
def test_group_fallback_steps_match():
    """steps a group cannot fuse -- idle clients marked before every other
    step (their activations are not part of the multi-table graph), and
    small k -- run per member with the same results as separate queues"""
    S, N = 3, 1 << 14
    wl = _workload(S, N, 2, 6, 1 << 11, seed=9)
    for k in (1 << 11, 4):
        a = _drive(wl, N, k, grouped=True, settle=N, idle_every=2, epoch=3)
        b = _drive(wl, N, k, grouped=False, settle=N, idle_every=2, epoch=3)
        assert a["digest"] == b["digest"], k
        assert a["trk"] == b["trk"], k


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["rerun", "terminal"])
def test_group_tallies_rerun_and_terminal_rounds(mode):
    """a group step's tallies are split -- the fused round's
    decisions tallied where k_rrank_m / k_rapply_m write them, the decisions
    of rounds the host drives afterwards by k_tally_m.  Pin that split on the
    two paths the clean steps never take, against separate queues (whose
    tallies are dmc_tracker_tally's pass over each call's decisions):
      rerun: sampled thresholds with no margin (DMC_OPT_SAMPLE = 2) -- fused
        rounds fail their exact count, nothing of them is applied or tallied,
        and the host re-runs them exactly;
      terminal: k far above the eligible requests -- every step's round runs
        out of work and the host's terminal pull follows it.
    Decisions, result records, statuses and every tracker word identical."""
    from dmclock_amd._abi import OPT_SAMPLE
    S, N = 3, 1 << 16  # (sampled thresholds: tables of >= 65,536 slots)
    if mode == "rerun":
        wl = _workload(S, N, 2, 6, 1 << 12, seed=13)
        k, settle, opts = 1 << 12, N, ((OPT_SAMPLE, 2),)
    else:
        wl = _workload(S, N, 1, 6, 1 << 11, seed=14)
        k, settle, opts = 1 << 15, N, ()
    a = _drive(wl, N, k, grouped=True, settle=settle, epoch=2, options=opts)
    b = _drive(wl, N, k, grouped=False, settle=settle, epoch=2, options=opts)
    assert a["fused"] == [6] * S, a["fused"]
    if mode == "rerun":
        assert min(a["retries"]) > 0, a["retries"]
    else:
        assert all(d < 6 * k for d in a["decisions"]), a["decisions"]
    assert a["digest"] == b["digest"]
    assert a["trk"] == b["trk"]
    assert a["decisions"] == b["decisions"]
