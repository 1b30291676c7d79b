"""The 8-wave GEMMs' K-tile schedules checked by simulation on the CPU (no GPU): the two-phase schedule (round 6
default, kernels_gemm8.hip g8_ops2 / g8_count2 / g8_issue2) and the four-phase one (g8_target / g8_count), restated
here as tables of (phase -> half-tiles issued, half-tiles read).  For every K-tile count the invariants the kernels
rely on are asserted:

  RAW  every half-tile a phase reads was issued earlier and is retired by the counted wait at the end of the
       previous phase's L-section (vmcnt(N) leaves the N youngest ops in flight: at least N were issued after it);
  WAR  a half-tile slot (buffer tile & 1, half) is re-filled only in a phase after every read of its previous
       occupant (group 1 reads one barrier after group 0, i.e. within the same phase's M-section: a slot read in
       phase p is free from phase p + 1 on);
  all  every half of every K-tile is issued exactly once and read where the MFMAs need it.
"""
import pytest

MX_SCALE_OPS = 1   # MX: the K-tile's scale DMA rides with A0


def _two_phase(nk, mx=False):
    """phase j (prologue j = -3..-1, then 2t + h) -> list of (tile, half) issued, reads, ops, count."""
    issues, reads = {}, {}
    for j in range(-3, 2 * nk):
        t = j >> 1
        if j % 2 == 0:
            issues[j] = [(t + 1, 1)] if t + 1 < nk else []
        else:
            issues[j] = [(t + 2, 0), (t + 2, 2), (t + 2, 3)] if t + 2 < nk else []
    for t in range(nk):
        reads[2 * t] = [(t, 0), (t, 2), (t, 3)]
        reads[2 * t + 1] = [(t, 1)]

    def ops(j):
        if j < -3:
            return 0
        n = 2 * len(issues.get(j, []))
        return n + (MX_SCALE_OPS if mx and any(h == 0 for _, h in issues.get(j, [])) else 0)

    def count(j):   # g8_count2: ops(j) + ops(j - 1)
        return ops(j) + ops(j - 1)
    return issues, reads, ops, count, -3


def _four_phase(nk, mx=False):
    issues, reads = {}, {}

    def target(k):   # g8_target
        t = (k + 8) // 4 - 2
        p = (k + 8) & 3
        tile = t + 1 if p < 2 else t + 2
        half = 3 if p == 0 else (1 if p == 1 else (0 if p == 2 else 2))
        return tile, half
    for k in range(-6, 4 * nk):
        tl, h = target(k)
        issues[k] = [(tl, h)] if tl < nk else []
    for t in range(nk):
        reads[4 * t] = [(t, 0), (t, 2)]
        reads[4 * t + 1] = [(t, 3)]
        reads[4 * t + 2] = [(t, 1)]
        reads[4 * t + 3] = []

    def ops(j):
        if j < -6:
            return 0
        n = 2 * len(issues.get(j, []))
        return n + (MX_SCALE_OPS if mx and any(h == 0 for _, h in issues.get(j, [])) else 0)

    def count(k):   # g8_count: ops issued at k-3 .. k
        return sum(ops(k - d) for d in range(4))
    return issues, reads, ops, count, -6


@pytest.mark.parametrize("sched", [_two_phase, _four_phase])
@pytest.mark.parametrize("mx", [False, True])
@pytest.mark.parametrize("nk", [1, 2, 3, 4, 5, 12, 48])
def test_schedule_invariants(sched, mx, nk):
    issues, reads, ops, count, first = sched(nk, mx)
    last = max(issues)
    # the ordered op stream: (phase, op index within the phase, (tile, half) or 'scale')
    stream = []
    for j in range(first, last + 1):
        for th in issues.get(j, []):
            if mx and th[1] == 0:
                stream.append((j, ("scale", th[0])))
            stream.append((j, th))
            stream.append((j, th))   # two DMA ops per half-tile and wave
    issued_at = {}
    for j, th in stream:
        issued_at.setdefault(th, j)
    # all: every half of every K-tile issued exactly once (2 ops each)
    halves = [th for _, th in stream if th[0] != "scale"]
    assert sorted(set(halves)) == sorted((t, h) for t in range(nk) for h in range(4))
    assert all(halves.count(th) == 2 for th in set(halves))
    # RAW: reads of phase j covered by the wait at the end of L(j - 1) (the prologue wait for the first phase)
    for j, rd in reads.items():
        for th in rd:
            i_ph = issued_at[th]
            assert i_ph < j, (th, i_ph, j)
            # vmcnt(N) leaves the N youngest ops in flight: the half's last op is retired when at least N ops
            # were issued after it by the end of phase j - 1
            idx = max(n for n, (p, x) in enumerate(stream) if x == th)
            younger = sum(1 for p, _ in stream[idx + 1:] if p <= j - 1)
            assert younger >= count(j - 1), (th, j, younger, count(j - 1))
    # WAR: slot (tile & 1, half) re-filled only after its previous occupant's last read phase
    last_read = {}
    for j, rd in reads.items():
        for t, h in rd:
            last_read[(t, h)] = max(last_read.get((t, h), j), j)
    for (t, h), j in issued_at.items():
        if t == "scale" or t < 2:
            continue
        prev = (t - 2, h)
        assert last_read[prev] < j, ((t, h), j, last_read[prev])


def test_two_phase_steady_counts():
    """The steady loop's uniform waits: vmcnt(8) (bf16) / vmcnt(9) (MX) are the counted waits' values there."""
    nk = 12
    _, _, _, count, _ = _two_phase(nk)
    _, _, _, count_mx, _ = _two_phase(nk, mx=True)
    for t in range(1, nk - 2):
        assert count(2 * t) == count(2 * t + 1) == 8
        assert count_mx(2 * t) == count_mx(2 * t + 1) == 9
