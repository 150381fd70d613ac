"""Seeded input generators shared by the CPU and GPU tests, and the
multi-process harness (file-based gloo rendezvous, fail-fast children)."""
import itertools
import os
import subprocess
import time

import numpy as np

from golden.make_golden import random_snapshot  # noqa: F401  (re-export)


def rdv_url(tmp_path):
    """A gloo rendezvous that needs no TCP port: a probed port can be taken
    (or held on another address) between the probe and the TCPStore's listen,
    which is what failed the round-4 driver run with EADDRINUSE.  The file
    must not exist yet; every rank of one group passes the same URL."""
    path = os.path.join(str(tmp_path), "rdv")
    if os.path.exists(path):
        os.unlink(path)
    return "file://" + path


def run_children(cmds, timeout, env=None, logs=None, cwd=None):
    """Start one child per command and wait for all of them.  As soon as one
    exits non-zero, or the deadline passes, every child still running is
    killed, so a rank that died never leaves its peer waiting in a
    rendezvous; children are always reaped (no process is left behind).
    `env` is one mapping for all children or a list of one per child; `logs`
    optional file paths taking each child's stdout + stderr.
    Returns the exit codes in command order (negative = killed here)."""
    envs = env if isinstance(env, list) else [env] * len(cmds)
    files = [open(f, "w") if f else None for f in (logs or [None] * len(cmds))]
    procs = [subprocess.Popen(c, env=e, cwd=cwd, stdout=f, stderr=subprocess.STDOUT if f else None)
             for c, e, f in zip(cmds, envs, files)]
    rcs = [None] * len(procs)
    deadline = time.monotonic() + timeout
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
            if any(rc not in (None, 0) for rc in rcs) or time.monotonic() > deadline:
                break
            time.sleep(0.05)
    finally:
        for i, p in enumerate(procs):
            if p.poll() is None:
                p.kill()
            p.wait()
            if rcs[i] is None:
                rcs[i] = p.returncode
        for f in files:
            if f:
                f.close()
    return rcs


def stack_snapshots(snaps):
    return {k: np.stack([s[k] for s in snaps]) for k in snaps[0]}


def f32_to_bf16_bits(x):
    """Round-to-nearest-even float32 -> bf16 bits (finite inputs)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_bits_to_f64(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def cluster(rng, P, N, dtype="i8", lo=0, hi=20, cap_scale=1.0, int_valued=True):
    """Random extended-mode instance: WA (P,N), L (N,N), free (N,3), req (P,3)."""
    if dtype == "i8":
        WA = rng.integers(lo, hi, (P, N)).astype(np.int8)
        L = rng.integers(lo, hi, (N, N)).astype(np.int8)
    elif int_valued:
        WA = f32_to_bf16_bits(rng.integers(lo, hi, (P, N)).astype(np.float32))
        L = f32_to_bf16_bits(rng.integers(lo, hi, (N, N)).astype(np.float32))
    else:
        WA = f32_to_bf16_bits(rng.random((P, N)).astype(np.float32))
        L = f32_to_bf16_bits((1.0 + 999.0 * rng.random((N, N))).astype(np.float32))
    free = np.stack([rng.integers(int(2000 * cap_scale), int(8000 * cap_scale) + 1, N),
                     rng.integers(int(2e6 * cap_scale), int(8e6 * cap_scale) + 1, N),
                     np.full(N, max(1, int(110 * cap_scale)))], 1).astype(np.int32)
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P),
                    np.ones(P, np.int64)], 1).astype(np.int32)
    return WA, L, free, req


def all_perms(n):
    return np.array(list(itertools.permutations(range(n))), np.int32)


KEY_INVALID = np.uint64(0xFFFFFFFFFFFFFFFF)


def keys_from_costs(nodes, costs):
    """int costs (< 2^31 in magnitude) + node ids -> packed keys (cost ^ 2^31) << 32 | node."""
    nodes = np.asarray(nodes)
    k = ((np.asarray(costs).astype(np.int64) ^ np.int64(-2**31)) & 0xFFFFFFFF).astype(np.uint64)
    k = (k << np.uint64(32)) | (nodes.astype(np.int64) & 0xFFFFFFFF).astype(np.uint64)
    return np.where(nodes >= 0, k, KEY_INVALID)


def merge_lists(parts, K=8):
    """Merge per-shard candidate lists [(keys (P,K), bounds (P,)), ...] with the
    engine's rule: keep the K smallest keys, bound = min(bounds, kept[K-1])."""
    keys = np.sort(np.concatenate([k for k, _ in parts], axis=1), axis=1)[:, :K]
    bound = np.minimum.reduce([b for _, b in parts] + [keys[:, K - 1]])
    return keys, bound


def usable(keys, bound):
    """Exact prefix of each list: node ids and count."""
    ok = (keys != KEY_INVALID) & (keys <= bound[:, None])
    nodes = np.where(ok, (keys & np.uint64(0xFFFFFFFF)).astype(np.int64), -1).astype(np.int32)
    return nodes, ok.sum(axis=1).astype(np.int32)
