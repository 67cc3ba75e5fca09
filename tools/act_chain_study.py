#!/usr/bin/env python3
"""Structure of the idle-reset recurrence of batched activations (debug dumps
of k_act_resolve's inputs, DMC_DEBUG=1 DMC_DUMP_ACT=path) and a CPU model of
the engine's speculate-and-verify resolution (act_chain in dmc_engine.hip).

Recurrence (dmclock_server.h:957-984), per activation j in batch order:
    L_j = min(X_j, M_j); pd_j = L_j - t_j; c_j = p_j + pd_j; M_{j+1} = min(M_j, c_j)
Prints: new-minimum and X-restart counts, and for the window model the number
of windows, failed checks and where they fail.
"""
import math
import struct
import sys

import numpy as np

KMAX = 0xFFFFFFFFFFFFFFFF
DMAX = 1.7976931348623157e308
TRIG = DMAX / 3.0


def from_okey(k):
    k = int(k)
    u = (k & 0x7FFFFFFFFFFFFFFF) if (k >> 63) else (~k & 0xFFFFFFFFFFFFFFFF)
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def read_dumps(path):
    raw = open(path, "rb").read()
    off = 0
    out = []
    while off < len(raw):
        m, = struct.unpack_from("<I", raw, off)
        base, = struct.unpack_from("<Q", raw, off + 4)
        off += 12
        arrs = []
        for dt in ("<u8", "<f8", "<f8", "<f8"):
            arrs.append(np.frombuffer(raw, dtype=dt, count=m, offset=off))
            off += 8 * m
        out.append((m, base) + tuple(arrs))
    return out


def exact(M, xs, ps, ts, pd0s):
    pds, Ms, newmin, xr = [], [], 0, 0
    for x, p, t, pd0 in zip(xs, ps, ts, pd0s):
        L = M if M < x else x
        if x < M:
            xr += 1
        lowest = L if L < DMAX else DMAX
        pd = lowest - t if lowest < TRIG else pd0
        c = p + pd
        if c < M:
            newmin += 1
        Ms.append(M)
        M = c if c < M else M
        pds.append(pd)
    return pds, Ms, M, newmin, xr


def grid(ref):
    if ref == 0 or not math.isfinite(ref):
        return math.ldexp(1.0, -53)
    _, e = math.frexp(ref)
    return math.ldexp(1.0, e - 53)


def window_model(M, xs, ps, ts, pd0s, W=1024):
    j0, n = 0, len(xs)
    windows = fails = waves = 0
    fail_pos = []
    while j0 < n:
        windows += 1
        w = min(W, n - j0)
        ref = M if M < math.inf else xs[j0]
        g = grid(ref)
        # speculation (python ints stand in for the grid's integer doubles)
        m = M / g
        spec = []
        cur = m
        for j in range(j0, j0 + w):
            d = round(ps[j] / g) - round(ts[j] / g)  # round-half-even as rint
            b = round(xs[j] / g) + d if xs[j] < math.inf else math.inf
            cur = min(cur + min(0, d), b)
            spec.append(cur * g)
        # verification
        Mj = M
        fl = w
        for i, j in enumerate(range(j0, j0 + w)):
            x, p, t, pd0 = xs[j], ps[j], ts[j], pd0s[j]
            L = Mj if Mj < x else x
            lowest = L if L < DMAX else DMAX
            pd = lowest - t if lowest < TRIG else pd0
            c = p + pd
            Mn = c if c < Mj else Mj
            if Mn != spec[i] or math.copysign(1, Mn) != math.copysign(1, spec[i]):
                fl = i
                M = Mn
                break
            Mj = spec[i]
        if fl == w:
            M = spec[-1]
            j0 += w
        else:
            fails += 1
            fail_pos.append(j0 + fl)
            j0 += fl + 1
            if fl + 1 < 64 and j0 < n:
                e = min(W, n - j0)
                _, _, M, _, _ = exact(M, xs[j0:j0 + e], ps[j0:j0 + e], ts[j0:j0 + e],
                                      pd0s[j0:j0 + e])
                waves += 1
                j0 += e
    return windows, fails, waves, fail_pos[:20]


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/act_dump.bin"
    for i, (m, base, ax, ap, at, apd) in enumerate(read_dumps(path)):
        xs = [from_okey(min(int(a), base)) if min(int(a), base) != KMAX else math.inf
              for a in ax]
        ps, ts, pd0s = ap.tolist(), at.tolist(), apd.tolist()
        pds, Ms, Mend, newmin, xr = exact(math.inf, xs, ps, ts, pd0s)
        print(f"dump {i}: m={m} new minima {newmin} X-restarts {xr} "
              f"M range [{min(Ms[1:] or [0]):.6g}, {Ms[1] if m > 1 else 0:.6g}] "
              f"X median {np.median([x for x in xs if x < math.inf]):.6g} "
              f"t range [{min(ts):.6g}, {max(ts):.6g}] p-t median {np.median(np.array(ps) - np.array(ts)):.4g}")
        w, f, wv, fp = window_model(math.inf, xs, ps, ts, pd0s)
        print(f"  window model: {w} windows, {f} failed checks, {wv} wave fallbacks, first fails at {fp}")


if __name__ == "__main__":
    main()
