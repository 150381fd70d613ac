"""NAS_OPT_SYNTH_PROFILE 1: SURVEY.md §8(d)'s C3 operand
distribution over the full int8 range -- latency U{1..127} (symmetric, zero
diagonal), traffic U{0..127} to every node -- generated on the device.  The
inputs are checked for that distribution, and a whole placement pass over
them against the sequential oracle (placements, integer scores, capacity)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
SEED = 0x4E4153


@pytest.mark.parametrize("N,P", [(1000, 6000), (3000, 20000)])
def test_fullrange_inputs_and_placement_equal_oracle(engine, N, P):
    engine.synth_cluster(SEED, N, P, "i8", peers=8, profile=1)
    WA, L, cap, req = engine.read_inputs(0, P, want_L=True)
    off = ~np.eye(N, dtype=bool)
    assert (np.diag(L) == 0).all() and (L == L.T).all()
    assert L[off].min() == 1 and L[off].max() == 127
    assert WA.min() == 0 and WA.max() == 127 and abs(WA.mean() - 63.5) < 0.5
    # (uniform: every value of the range occurs, none dominates)
    counts = np.bincount(WA.reshape(-1).astype(np.int64), minlength=128)
    assert counts.min() > 0.8 * WA.size / 128 and counts.max() < 1.2 * WA.size / 128
    engine.reset_capacity()
    node, _, score = engine.place()
    want, wcost, wfree = oracle.place(WA, L, req, cap, "i8")
    assert (node == want).all(), np.nonzero(node != want)[0][:8]
    assert (score == wcost).all()
    assert (engine.get_capacity() == wfree).all()


def test_profile_option_is_per_call(engine):
    """synth_cluster(profile=0) after a profile-1 cluster is the default
    generator again (the option is set on every synth call)."""
    engine.synth_cluster(SEED, 600, 512, "i8", peers=8, profile=1)
    _, L1, _, _ = engine.read_inputs(0, 0, want_L=True)
    engine.synth_cluster(SEED, 600, 512, "i8", peers=8, profile=0)
    _, L0, _, _ = engine.read_inputs(0, 0, want_L=True)
    assert L1.max() > 105 and L0.max() <= 105  # distance classes top out at 104


def test_fullsize_fullrange_herd_passes_stay_few_rounds(engine):
    """The full-size full-range herd (configs.C3_fullrange): after the pass
    that discovers the herd, the herd plan with the cost-row cache and the
    stale-scan threshold of 4 (k_rescore.hip STALE_MIN_FIT) needs only a few
    rescore rounds per pass (27-56 with a threshold of 2), and every pass
    places identically; the first pods equal the sequential oracle."""
    N, P, sample = 10000, 100000, 512
    engine.synth_cluster(SEED, N, P, "i8", peers=8, profile=1)
    WA, L, cap, req = engine.read_inputs(0, sample, want_L=True)
    runs = []
    for _ in range(3):
        engine.reset_capacity()
        node, _, score = engine.place()
        runs.append((node.copy(), score.copy(), engine.timings()["rescore_rounds"]))
    first_rounds = runs[0][2]
    assert first_rounds >= 8  # the discovery pass: pipelined plan, no cache
    for node, score, rounds in runs[1:]:
        assert (node == runs[0][0]).all() and (score == runs[0][1]).all()
        assert rounds <= 16, rounds
    want, wcost, _ = oracle.place(WA, L, req[:sample], cap, "i8")
    assert (runs[0][0][:sample] == want).all() and (runs[0][1][:sample] == wcost).all()
