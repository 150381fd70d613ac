"""CPU model of nas_place's commit walk + gathered rescore slots on a
full-range herd (configs.C3_fullrange scaled down by N / 10,000): chunks of
pods get their 8-lists against the capacity `lag` chunks back, the walk takes
each pod's first usable candidate that still fits, and a dry pod halts it
for a slot that rescores the first R pods (pods, not chunks, scaled) with
fewer than `min_fit` usable fitting candidates.  Prints the slots and the
pods rescored per policy.  Not the product; a design aid.
  python tools/herd_model.py [N] [P]"""
import sys
import time

import numpy as np

rng = np.random.default_rng(1)
N, P = int(sys.argv[1]) if len(sys.argv) > 1 else 2000, int(sys.argv[2]) if len(sys.argv) > 2 else 20000
L = rng.integers(1, 128, (N, N)).astype(np.float64)
L = np.triu(L, 1)
L = L + L.T
WA = rng.integers(0, 128, (P, N)).astype(np.float64)
t0 = time.time()
C = (WA @ L).astype(np.int64)  # exact (< 2^53)
print("cost", time.time() - t0, file=sys.stderr)
cap0 = np.stack([np.where(rng.random(N) < .5, 4000, 8000), np.where(rng.random(N) < .5, 4 << 20, 8 << 20),
                 np.full(N, 110)], 1).astype(np.int64)
lc0, lc1, lm0, lm1 = -3.6716, -0.2695, 6.8833, 8.4928
req = np.stack([np.maximum(1, np.ceil(10 ** (lc0 + (lc1 - lc0) * rng.random(P)) * 1000)),
                np.ceil(10 ** (lm0 + (lm1 - lm0) * rng.random(P)) / 1024), np.ones(P)], 1).astype(np.int64)
KEY = C * N + np.arange(N)[None, :]  # (cost, node) order
INF = np.iinfo(np.int64).max


def lists(pods, cap):
    fit = (req[pods][:, None, :] <= cap[None, :, :]).all(axis=2)
    k = np.where(fit, KEY[pods], INF)
    part = np.partition(k, 8, axis=1)[:, :9]
    part.sort(axis=1)
    keys = part[:, :8]
    bound = part[:, 8] - 1  # every key < the 9th is present
    bound = np.where(part[:, 7] == INF, INF, np.minimum(bound, part[:, 7]))
    return keys, bound


SC = N / 10000


def run(chunk=12288, lag=2, R=1024, min_fit=2, contiguous=False):
    chunk, R = max(64, int(chunk * SC)), max(32, int(R * SC))
    cap = cap0.copy()
    keys = np.full((P, 8), INF)
    bound = np.zeros(P, np.int64)
    node = np.full(P, -1)
    snaps = {}
    slots = 0
    rescored = 0
    # chunk c scored against the capacity after chunk c - lag committed
    starts = list(range(0, P, chunk))
    # commit walk with chunk snapshots recorded as the walk passes chunk ends
    # (approximation: lists of chunk c were scored against cap after chunk c-lag;
    # recompute lazily in order)
    cap = cap0.copy()
    for ci, s in enumerate(starts):
        e = min(P, s + chunk)
        ref = ci - lag
        snap = snaps.get(ref, cap0)
        keys[s:e], bound[s:e] = lists(np.arange(s, e), snap)
        p = s
        while p < e:
            placed = False
            for j in range(8):
                k = keys[p, j]
                if k == INF or k > bound[p]:
                    break
                n = k % N
                if (req[p] <= cap[n]).all():
                    cap[n] -= req[p]
                    node[p] = n
                    placed = True
                    break
            if placed:
                p += 1
                continue
            if bound[p] == INF:  # complete list: nothing fits
                p += 1
                continue
            # halt: gathered slot
            slots += 1
            rest = np.arange(p, P)
            if contiguous:
                flag = rest[:R]
            else:
                kk = keys[rest]
                ok = (kk != INF) & (kk <= bound[rest][:, None])
                nn = np.where(ok, kk % N, 0)
                fits = ok & (req[rest][:, None, :] <= cap[nn]).all(axis=2)
                nfit = fits.sum(axis=1)
                flag = rest[(nfit < min_fit) & (bound[rest] != INF)][:R]
            rescored += len(flag)
            keys[flag], bound[flag] = lists(flag, cap)
        snaps[ci] = cap.copy()
    return slots, rescored


for kw in (dict(), dict(R=2048), dict(R=4096), dict(min_fit=4), dict(min_fit=8), dict(R=2048, min_fit=8),
           dict(contiguous=True), dict(contiguous=True, R=2048), dict(lag=1), dict(chunk=2048, lag=1)):
    t0 = time.time()
    print(kw, run(**kw), round(time.time() - t0, 1), flush=True)
