"""RCCL path hardening (include/nas.h NAS_OPT_COMM_TIMEOUT_MS): a call that
issued collectives waits under a deadline; on expiry the communicators are
aborted, the call returns NAS_ERR_COMM and the context is poisoned.  Tested
at world 1 with an injected device-side stall (NAS_OPT_INJECT_STALL_MS) in
front of the pass -- the stand-in for a peer rank that never arrives."""
import os
import time

import numpy as np
import pytest

from kubernetesnetawarescheduler_amd import Engine, NasError, _lib

pytestmark = pytest.mark.gpu


def test_comm_deadline_aborts_and_poisons():
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        e.synth_cluster(7, 512, 2048, "i8", peers=8)
        node, _, _ = e.place()  # healthy pass through the one-rank communicator
        assert (node >= -1).all()
        e.set_option("COMM_TIMEOUT_MS", 200)
        e.set_option("INJECT_STALL_MS", 1500)
        with pytest.raises(NasError) as ei:  # (the same pass without the stall succeeds)
            e.place()
        assert ei.value.code == _lib.NAS_ERR_COMM
        assert "did not complete within 200 ms" in str(ei.value)
        with pytest.raises(NasError) as ei:  # poisoned: every later call fails fast
            e.reset_capacity()
        assert ei.value.code == _lib.NAS_ERR_COMM
    # a fresh context on the same device is unaffected
    with Engine(0) as e:
        e.synth_cluster(7, 512, 2048, "i8", peers=8)
        e.place()


def test_comm_deadline_not_hit_when_healthy():
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        e.set_option("COMM_TIMEOUT_MS", 5000)
        e.set_option("INJECT_STALL_MS", 100)  # shorter than the deadline: just slower
        e.synth_cluster(8, 512, 2048, "i8", peers=8)
        a, _, _ = e.place()
        e.reset_capacity()
        b, _, _ = e.place()
        assert (a == b).all()


def test_options_reject_bad_values():
    with Engine(0) as e:
        for key, val in (("STAGE_TIMINGS", 2), ("COMM_TIMEOUT_MS", -1), ("INJECT_STALL_MS", -5)):
            with pytest.raises(NasError) as ei:
                e.set_option(key, val)
            assert ei.value.code == _lib.NAS_ERR_ARG
        with pytest.raises(NasError):
            e.set_option(99, 1)
        e.set_option("STAGE_TIMINGS", 0)
        e.synth_cluster(9, 256, 1024, "i8", peers=8)
        e.place()
        t = e.timings()
        assert t["total_ms"] > 0 and t["cost_ms"] == 0  # only the synchronising events
        e.set_option("STAGE_TIMINGS", 1)
        e.reset_capacity()
        e.place()
        assert e.timings()["cost_ms"] > 0
    assert np.int32(_lib.NAS_OPT_REHEARSE_WORLD) == 3


def _threads():
    return len(os.listdir("/proc/self/task"))


def test_comm_init_deadline_when_a_rank_never_joins():
    """Rank 0 of a two-rank communicator whose rank 1 never arrives: a
    blocking ncclCommInitRank would wait forever; nas_comm_init polls a
    non-blocking init under the deadline, aborts it on expiry and returns
    NAS_ERR_COMM.  The context keeps its world-1 geometry (placements equal a
    fresh context's), a retry fails the same way, and no thread started by
    the attempts survives nas_destroy."""
    ids = [Engine.comm_unique_id() for _ in range(2)]  # (RCCL's bootstrap roots start here)
    with Engine(0) as ref:
        ref.synth_cluster(9, 512, 2048, "i8", peers=8)
        want, _, want_cost = ref.place()
    base = _threads()
    with Engine(0) as e:
        e.set_option("COMM_TIMEOUT_MS", 3000)
        for uid in ids:  # a host that retries must not pile up stuck threads
            t0 = time.monotonic()
            with pytest.raises(NasError) as ei:
                e.comm_init(uid, 0, 2)
            assert ei.value.code == _lib.NAS_ERR_COMM
            assert "did not complete within 3000 ms" in str(ei.value)
            assert time.monotonic() - t0 < 30
        e.synth_cluster(9, 512, 2048, "i8", peers=8)
        node, _, cost = e.place()
        assert (node == want).all() and (cost == want_cost).all()
    deadline = time.monotonic() + 10
    while _threads() > base and time.monotonic() < deadline:
        time.sleep(0.1)
    assert _threads() <= base, (_threads(), base)


def test_comm_init_with_the_system_rccl():
    """The Go host loads /opt/rocm's RCCL (libnas.so's own dependency), the
    Python tests torch's copy, which this process already mapped: run the
    one-rank communicator + a pass in a child that never imports torch."""
    import subprocess
    import sys
    code = ("import sys; from kubernetesnetawarescheduler_amd import Engine\n"
            "with Engine(0) as e:\n"
            "    e.comm_init(Engine.comm_unique_id(), 0, 1)\n"
            "    e.synth_cluster(7, 512, 2048, 'i8', peers=8)\n"
            "    n, _, _ = e.place()\n"
            "    assert (n >= -1).all()\n"
            "assert 'torch' not in sys.modules\n"
            "print('rccl', [l.split()[-1] for l in open('/proc/self/maps') if 'librccl' in l][:1])\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "/opt/rocm" in r.stdout, r.stdout


# the tail commit's bounded wait for the commit stream
# (k_flag_wait) -- its budget, and how its expiry is reported.  The stall is
# injected on the commit stream ahead of its last flag store
# (NAS_OPT_INJECT_COMMIT_STALL_MS); 30,000 pods over 2,000 nodes is a
# three-chunk pass, so the tail chunk waits for the commit stream.
def _three_chunk_cluster(e):
    e.synth_cluster(11, 2000, 30000, "i8", peers=8)


def test_commit_wait_timeout_without_comm_is_an_error_not_a_hang():
    with Engine(0) as e:
        _three_chunk_cluster(e)
        want, _, wscore = e.place()
        e.set_option("COMMIT_WAIT_MS", 100)
        e.set_option("INJECT_COMMIT_STALL_MS", 1500)
        e.reset_capacity()
        with pytest.raises(NasError) as ei:
            e.place()
        assert ei.value.code == _lib.NAS_ERR_HIP
        assert "NAS_OPT_COMMIT_WAIT_MS" in str(ei.value) and "100 ms" in str(ei.value)
        # not poisoned: the next pass (the stall is used up) is the same as before
        e.set_option("COMMIT_WAIT_MS", 0)
        e.reset_capacity()
        node, _, score = e.place()
        assert (node == want).all() and (score == wscore).all()


def test_commit_wait_timeout_with_comm_aborts_and_poisons():
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        _three_chunk_cluster(e)
        e.place()
        # the host's own deadline is far away: the device-side wait expires first
        e.set_option("COMM_TIMEOUT_MS", 20000)
        e.set_option("COMMIT_WAIT_MS", 100)
        e.set_option("INJECT_COMMIT_STALL_MS", 1500)
        e.reset_capacity()
        t0 = time.monotonic()
        with pytest.raises(NasError) as ei:
            e.place()
        assert ei.value.code == _lib.NAS_ERR_COMM
        assert "communicators aborted" in str(ei.value)
        assert time.monotonic() - t0 < 15
        with pytest.raises(NasError) as ei:
            e.reset_capacity()
        assert ei.value.code == _lib.NAS_ERR_COMM
    # (nas_destroy of the poisoned context returned: the aborted communicators
    # are torn down before its streams are synchronised)


def test_commit_wait_budget_defaults_to_comm_deadline():
    """With a communicator the wait takes NAS_OPT_COMM_TIMEOUT_MS, so a stall
    shorter than that deadline (but longer than the old fixed 2 s) passes."""
    with Engine(0) as e:
        e.comm_init(Engine.comm_unique_id(), 0, 1)
        _three_chunk_cluster(e)
        want, _, _ = e.place()
        e.set_option("COMM_TIMEOUT_MS", 8000)
        e.set_option("INJECT_COMMIT_STALL_MS", 2500)
        e.reset_capacity()
        node, _, _ = e.place()
        assert (node == want).all()
